"""R2D2 prioritized sequence replay.

The replay half of acme/agents/tf/r2d2: the prioritized sequence table, SequenceAdder and
sequence dataset the agent wires up (agents/tf/r2d2/agent.py:72-103), and the learner's
two replay-facing computations as device kernels (csrc/r2d2.hip):
  compute_priority     learning.py:230-236 (written back with update_priorities, :196-199)
  importance_weights   learning.py:178-183
and the learner itself, R2D2Learner (learning.py: csrc/r2d2_learner.hip, the recurrent
duelling Q-network with burn-in and the transformed n-step loss).
"""

from __future__ import annotations

from typing import Optional

import torch

from acme_amd import replay
from acme_amd.adders import reverb as adders
from acme_amd.datasets import make_reverb_dataset
from acme_amd.agents.r2d2.learning import R2D2Learner  # noqa: F401


def _check(name, t, dtype):
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.is_contiguous() and t.dtype == dtype):
        raise ValueError(f"{name} must be a contiguous {dtype} device tensor")


def compute_priority(errors: torch.Tensor, alpha: float, stream=None) -> torch.Tensor:
    """errors [T, B] float32 (device) -> priorities [B] float64:
    alpha * max_t |e| + (1 - alpha) * mean_t |e| (learning.py:230-236)."""
    from acme_amd._lib import check, lib, stream_ptr
    _check("errors", errors, torch.float32)
    if errors.dim() != 2:
        raise ValueError("errors must be [T, B]")
    T, B = errors.shape
    out = torch.empty(B, dtype=torch.float64, device=errors.device)
    check(lib().acme_r2d2_priorities(errors.data_ptr(), T, B, float(alpha), out.data_ptr(),
                                     stream_ptr(stream)), "r2d2 priorities")
    return out


def importance_weights(probabilities: torch.Tensor, max_replay_size: int, beta: float,
                       stream=None) -> torch.Tensor:
    """probabilities [B] float64 (device) -> [B] float32 weights
    (1 / (N p))^beta / max (learning.py:178-183; constant over a sequence's T steps)."""
    from acme_amd._lib import check, lib, stream_ptr
    _check("probabilities", probabilities, torch.float64)
    B = probabilities.shape[0]
    out = torch.empty(B, dtype=torch.float32, device=probabilities.device)
    check(lib().acme_r2d2_importance_weights(probabilities.data_ptr(), B, int(max_replay_size),
                                             float(beta), out.data_ptr(), stream_ptr(stream)),
          "r2d2 importance weights")
    return out


def make_replay(environment_spec, extra_spec, burn_in_length: int, trace_length: int,
                replay_period: int, batch_size: int = 32, max_replay_size: int = 1_000_000,
                priority_exponent: float = 0.6, prefetch_size: Optional[int] = None,
                seed: int = 1234, device=None):
    """The replay wiring of R2D2 (agents/tf/r2d2/agent.py:72-103): a Prioritized(priority
    exponent) + Fifo table of sequence_length = burn_in + trace + 1 steps, the
    SequenceAdder(period=replay_period) that fills it and the sequence dataset.
    Returns (server, adder, dataset)."""
    table = replay.Table(adders.DEFAULT_PRIORITY_TABLE,
                         replay.selectors.Prioritized(priority_exponent),
                         replay.selectors.Fifo(), max_replay_size,
                         replay.rate_limiters.MinSize(1),
                         signature=adders.SequenceAdder.signature(environment_spec, extra_spec),
                         seed=seed, device=device)
    server = replay.Server([table])
    sequence_length = burn_in_length + trace_length + 1
    adder = adders.SequenceAdder(client=replay.Client(server), period=replay_period,
                                 sequence_length=sequence_length)
    dataset = make_reverb_dataset(server_address=server, batch_size=batch_size,
                                  prefetch_size=prefetch_size, sequence_length=sequence_length)
    return server, adder, dataset
