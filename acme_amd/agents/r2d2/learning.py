"""R2D2Learner — drop-in for acme/agents/tf/r2d2/learning.py:40-236.

Same constructor (environment_spec, network, target_network, burn_in_length,
sequence_length, dataset, reverb_client, counter=None, logger=None, discount=0.99,
target_update_period=100, importance_sampling_exponent=0.2, max_replay_size=1_000_000,
learning_rate=1e-3, store_lstm_state=True, max_priority_weight=0.9, n_step=5) and
`step()` contract.  One call takes a [B, T] batch of sequences from the dataset
(Step(observation=OAR(observation, action, reward), action, reward, discount,
extras={'core_state': LSTMState})) and runs the whole step on the GPU (acme_r2d2_step):
burn-in of both networks, online and target unrolls, the transformed n-step double-Q loss
with importance weights, BPTT to the end of the burn-in, snt.Adam(lr, epsilon=1e-3), the
periodic target copy, then writes the priorities eta max |e| + (1 - eta) mean |e| back to
replay (learning.py:192-199).  Nothing synchronises the host with the device.

`network` / `target_network` are acme_amd.networks.R2D2AtariNetwork descriptors (the
reference takes Sonnet RNN cores); the target starts from its own initialisation.
"""

from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np
import torch

from acme_amd import core
from acme_amd.adders import reverb as adders
from acme_amd.native import NativeR2D2
from acme_amd.utils import counting, loggers


def _state_parts(core_state):
    if isinstance(core_state, dict):
        return core_state["hidden"], core_state["cell"]
    hidden, cell = core_state
    return hidden, cell


class R2D2Learner(core.Learner, core.Saveable):

    def __init__(self, environment_spec, network, target_network, burn_in_length: int,
                 sequence_length: int, dataset, reverb_client=None,
                 counter: Optional[counting.Counter] = None,
                 logger: Optional[loggers.Logger] = None, discount: float = 0.99,
                 target_update_period: int = 100, importance_sampling_exponent: float = 0.2,
                 max_replay_size: int = 1_000_000, learning_rate: float = 1e-3,
                 store_lstm_state: bool = True, max_priority_weight: float = 0.9,
                 n_step: int = 5, batch_size: Optional[int] = None, seed: int = 0,
                 target_seed: Optional[int] = None, device=None,
                 on_plane_overflow: str = "skip"):
        # A step whose f16 planes overflowed (or whose LSTM unroll timed out) is skipped on
        # the device and the scales recalibrated ("skip", as IMPALA), or raises
        # FloatingPointError at the next step() ("raise").
        if on_plane_overflow not in ("skip", "raise"):
            raise ValueError("on_plane_overflow must be 'skip' or 'raise'")
        self._on_overflow = on_plane_overflow
        self._env_spec = environment_spec
        self._network = network
        self._iterator = iter(dataset)
        self._client = reverb_client
        self._burn_in = int(burn_in_length)
        self._T = int(sequence_length)
        B = batch_size or getattr(dataset, "batch_size", None) or 32
        self._native = NativeR2D2(
            num_actions=network.num_actions, max_batch=B, max_sequence_length=self._T,
            burn_in_length=self._burn_in, torso=network.torso, obs_dim=network.obs_dim,
            lstm_size=network.lstm_size, head_size=network.head_size, n_step=n_step,
            discount=discount, importance_sampling_exponent=importance_sampling_exponent,
            max_replay_size=max_replay_size, max_priority_weight=max_priority_weight,
            target_update_period=target_update_period, learning_rate=learning_rate,
            store_lstm_state=store_lstm_state, device=device)
        self._native.set_params(network.init(seed),
                                target_network.init(seed + 1 if target_seed is None
                                                    else target_seed))
        self._skips_seen = 0
        self._counter = counter or counting.Counter(None, "learner")
        self._logger = logger or loggers.TerminalLogger("learner", time_delta=100.)
        self._timestamp = None

    def _check_guard(self) -> int:
        n = self._native.skipped_steps  # pinned host word: no synchronisation
        if n != self._skips_seen:
            self._skips_seen = n
            if self._on_overflow == "raise":
                raise FloatingPointError(
                    f"R2D2 learner: {n} step(s) skipped on f16 plane overflow or an LSTM "
                    "timeout (their updates were not applied)")
            self._native.params_changed()  # recalibrate the plane scales before the next step
        return n

    def step(self):
        skipped = self._check_guard()
        sample = next(self._iterator)
        data = sample.data
        obs = data.observation
        if not hasattr(obs, "observation"):
            raise ValueError("R2D2AtariNetwork takes OAR observations "
                             "(wrap the environment in ObservationActionRewardWrapper)")
        n = self._native
        dt = torch.uint8 if self._network.torso == "atari" else torch.float32
        c = lambda x, t: x.to(t).contiguous()  # noqa: E731
        B, T = int(data.action.shape[0]), int(data.action.shape[1])
        h0 = c0 = None
        if n.store_lstm_state:
            hidden, cell = _state_parts(data.extras["core_state"])
            h0, c0 = hidden.to(torch.float32)[:, 0], cell.to(torch.float32)[:, 0]
        keys, probs = sample.info.key, sample.info.probability
        if probs.dim() == 2:  # per-step info of a sequence item: the item's own
            keys, probs = keys[:, 0], probs[:, 0]
        n.step(c(obs.observation.reshape((B, T, -1)) if dt == torch.float32
                 else obs.observation, dt),
               c(obs.action.reshape(B, T), torch.int32),
               c(obs.reward.reshape(B, T), torch.float32),
               c(data.action.reshape(B, T), torch.int32),
               c(data.reward.reshape(B, T), torch.float32),
               c(data.discount.reshape(B, T), torch.float32),
               c(probs, torch.float64), h0, c0)
        if self._client is not None:  # learning.py:195-198; a skipped step writes none
            kw = {"skip_word": n.skip_word} if n.skip_word else {}
            self._client.update_priorities(table=adders.DEFAULT_PRIORITY_TABLE, keys=keys,
                                           priorities=n.priorities[:B], **kw)
        now = time.time()
        elapsed = now - self._timestamp if self._timestamp else 0
        self._timestamp = now
        result = {"loss": n.loss[0]}
        if skipped:
            result["skipped_steps"] = skipped
        result.update(self._counter.increment(steps=1, walltime=elapsed))
        self._logger.write(result)

    # ------------------------------------------------------------------ variables
    def get_variables(self, names: List[str]) -> List[List[np.ndarray]]:
        # As the TF learner (learning.py:216-217): one collection, names ignored.
        p = self._native.get_params("params")
        return [[p[k] for k in sorted(p)]]

    @property
    def num_steps(self) -> int:
        return self._native.num_steps

    @property
    def native(self) -> NativeR2D2:
        return self._native

    @property
    def state(self) -> Dict:
        return self.save()

    def save(self) -> Dict:
        n = self._native
        # The DQN / IMPALA learners' format: Adam's t (the updates applied) as
        # optimizer["step"], num_steps the step() calls, and the f16 plane scales, so a
        # resumed run is bit-identical to an uninterrupted one.
        return {"network": n.get_params("params"), "target_network": n.get_params("target"),
                "optimizer": {"m": n.get_params("m"), "v": n.get_params("v"),
                              "step": n.guard_state()["applied"]},
                "num_steps": n.num_steps,
                "plane_scales": n.scale_state()}

    def restore(self, state: Dict):
        n = self._native
        n.set_params(state["network"], state["target_network"])
        for buf, src in ((n.m, state["optimizer"]["m"]), (n.v, state["optimizer"]["v"])):
            for k, t in n.views(buf).items():
                t.copy_(torch.as_tensor(np.asarray(src[k], np.float32)).view(t.shape))
        n.params_changed()
        if "plane_scales" in state:
            n.set_scale_state(state["plane_scales"])
        n.num_steps = int(state["num_steps"])
        opt = state["optimizer"]
        # round-4 checkpoints: "step" = num_steps, the applied count in "applied_steps"
        n.set_applied_steps(int(opt.get("applied_steps", opt.get("step", state["num_steps"]))))
