"""Parity at the headline configuration (BASELINE configs[1]):
DQN Nature CNN (18 actions) at batch 512 through exactly the path bench.py times — a
1,000,000-slot prioritized GPU Table filled by the device generator -> make_reverb_dataset
(prefetch_size 4, the reference DQN agent's) -> DQNLearner.step() -> update_priorities.

Each step is checked teacher-forced against the f64 oracle (oracle/dqn_oracle.py, a
restatement of agents/tf/dqn/learning.py:112-161) started from the GPU's own pre-step state:
  the draw (slots, keys, probabilities, table_size, priorities): bit-exact against the C
      sum-tree oracle mirroring every priority write-back;
  q / loss: rtol 1e-5; TD / priorities: 1e-5 of |target| + |q_tm1[a]| (_td_close);
  gradients: per tensor |g - g_ref| <= 1e-4 |g_ref| + 2e-5 max|g_ref|, conditional on the
      kernel's own ReLU pattern (tests/test_dqn_gpu.py::_relu_masks);
  Adam on the GPU's own gradients: 1e-6 relative to the update's terms; target copy after
      steps with num_steps % period == 0 (learning.py:157-161): bit-identical;
  the tree after update_priorities: leaves bit-exact against the oracle at every touched
      slot.
At B = 512 the GEMMs run the bench's grids (fc_fwd split-K 4/8 over 1024 / 512 rows, the
XCD-remapped block order, full two-frame image blocks), which smaller batches never reach.
"""

import numpy as np
import pytest
import torch

from oracle import dqn_oracle as O
from tests.test_dqn_gpu import _check_grads, _relu_masks

pytestmark = pytest.mark.gpu

B = 512
CAPACITY = 1_000_000
SEED = 1234
PERIOD = 2   # target copies after steps 0 and 2 (the bench uses 100; cadence is the same code)


class _Recorder:
    """Wraps the dataset iterator to keep the sample each learner step consumed."""

    def __init__(self, it):
        self.it, self.last = it, None

    def __iter__(self):
        return self

    def __next__(self):
        self.last = next(self.it)
        return self.last


def _host(sample):
    o_tm1, a, r, d, o_t = (x.cpu().numpy() for x in sample.data[:5])
    info = dict(keys=sample.info.key.view(torch.int64).cpu().numpy().view(np.uint64),
                probabilities=sample.info.probability.cpu().numpy(),
                table_size=sample.info.table_size.cpu().numpy(),
                priorities=sample.info.priority.cpu().numpy())
    batch = dict(o_tm1=o_tm1, a_tm1=a.astype(np.int32), r_t=r, d_t=d, o_t=o_t,
                 probabilities=info["probabilities"])
    return batch, info


def _td_close(got, out, batch, absolute=False):
    """TD errors (and |td| priorities) at rtol 1e-5 of the magnitudes they are the
    difference of: td = target - q_tm1[a] cancels, so its error is relative to |target| +
    |q_tm1[a]| (the q values themselves are checked at rtol 1e-5 by _relu_masks' forward
    and the loss)."""
    td = out["td_error"]
    qa = out["q_tm1"][np.arange(len(td)), batch["a_tm1"]]
    scale = np.abs(td + qa) + np.abs(qa)
    ref = np.abs(td) if absolute else td
    err = np.abs(np.asarray(got, np.float64) - ref)
    assert (err <= 1e-5 * scale + 1e-7).all(), float((err / (scale + 1e-30)).max())


def test_bench_path_b512_teacher_forced():
    from acme_amd import replay, specs
    from acme_amd.adders import reverb as adders
    from acme_amd.agents.dqn import DQNLearner
    from acme_amd.datasets import make_reverb_dataset
    from acme_amd.networks import DQNAtariNetwork
    from acme_amd.utils import loggers
    from tests._oracle import OracleTable

    A = 18
    spec = specs.EnvironmentSpec(
        observations=specs.Array((84, 84, 4), np.uint8), actions=specs.DiscreteArray(A, np.int32),
        rewards=specs.Array((), np.float32), discounts=specs.BoundedArray((), np.float32, 0, 1))
    table = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Prioritized(0.6),
                         replay.selectors.Fifo(), CAPACITY, replay.rate_limiters.MinSize(1),
                         signature=adders.NStepTransitionAdder.signature(spec), seed=SEED)
    table.native.fill_synthetic(CAPACITY, layout=0, num_actions=A, seed=0)
    mirror = OracleTable(CAPACITY, True, 0.6, SEED)
    mirror.insert(np.ones(CAPACITY))  # fill_synthetic: every priority 1.0, keys 0..C-1
    server = replay.Server([table])
    net = DQNAtariNetwork(A)
    learner = DQNLearner(net, net, discount=0.99, importance_sampling_exponent=0.2,
                         learning_rate=1e-3, target_update_period=PERIOD,
                         dataset=make_reverb_dataset(server, batch_size=B, prefetch_size=4),
                         replay_client=replay.Client(server), logger=loggers.NoOpLogger(),
                         seed=0)
    rec = _Recorder(learner._iterator)  # noqa: SLF001
    learner._iterator = rec  # noqa: SLF001
    n = learner.native
    cfg = O.DQNConfig(num_actions=A, target_update_period=PERIOD)

    class _Net:  # what _relu_masks needs to know about the network
        kind, num_actions = "nature", A

    # Draw k is issued when batch k - 4 is handed out, i.e. after the priority write-back of
    # step k - 5 (prefetch 4): the mirror applies write-backs in that order.
    pending = []
    for step in range(6):
        pre = {w: n.get_params(w) for w in ("params", "target", "m", "v")}
        pre_steps = n.num_steps
        learner.step()
        torch.cuda.synchronize()
        batch, info = _host(rec.last)
        while pending and pending[0][0] <= step - 5:
            mirror.update(*pending.pop(0)[1:])
        ref_draw = mirror.sample(B, step)
        for k in ("keys", "probabilities", "table_size", "priorities"):
            np.testing.assert_array_equal(info[k], ref_draw[k], err_msg=f"step {step} {k}")
        prio = n.priorities[:B].cpu().numpy()
        pending.append((step, info["keys"], prio))
        if step >= 3:  # later steps: the draws after write-backs (checked above)
            continue
        # Forward activations and the ReLU pattern of the o_tm1 rows, then the step.
        masks = _relu_masks(n, _Net, batch, pre["params"], B)
        out, grads = O.dqn_loss_and_grads(cfg, pre["params"], pre["target"], batch,
                                          np.float64, masks=masks)
        np.testing.assert_allclose(n.loss.item(), out["loss"], rtol=1e-5)
        _td_close(n.td_error[:B].cpu().numpy(), out, batch)
        _td_close(prio, out, batch, absolute=True)
        g = n.get_params("grads")
        _check_grads(g, grads)
        post = {w: n.get_params(w) for w in ("params", "target", "m", "v")}
        for k in pre["params"]:
            p1, m1, v1 = O.adam_update(pre["params"][k], g[k], pre["m"][k], pre["v"][k],
                                       pre_steps + 1, 1e-3)
            # m = b1 m + (1 - b1) g cancels when the two terms have opposite signs (the
            # kernel fuses it into one FMA): its error is relative to the terms.
            m_terms = 0.9 * np.abs(pre["m"][k]) + 0.1 * np.abs(g[k])
            assert (np.abs(post["m"][k] - m1) <= 1e-6 * m_terms + 1e-30).all(), k
            np.testing.assert_allclose(post["v"][k], v1, rtol=1e-6, atol=1e-30)
            # The update lr mhat / (sqrt(vhat) + eps) inherits m's cancellation: bound it by
            # the same expression evaluated on m's terms.
            t = pre_steps + 1
            vhat = np.asarray(v1, np.float64) / (1 - 0.999 ** t)
            upd_terms = 1e-3 * (m_terms / (1 - 0.9 ** t)) / (np.sqrt(vhat) + 1e-8)
            p_terms = np.abs(pre["params"][k]) + upd_terms
            assert (np.abs(post["params"][k] - p1) <= 1e-6 * p_terms + 1e-30).all(), k
            want = post["params"][k] if pre_steps % PERIOD == 0 else pre["target"][k]
            np.testing.assert_array_equal(post["target"][k], want)
        assert n.num_steps == pre_steps + 1
    # The tree after the write-backs: every touched slot's leaf equals the oracle's.
    for _, keys, prio in pending:
        mirror.update(keys, prio)
    leaves = table.native.debug_state()["leaves"]
    ref = mirror.leaves()[:CAPACITY]
    touched = np.unique(np.concatenate([k for _, k, _ in pending]).astype(np.int64) % CAPACITY)
    np.testing.assert_array_equal(leaves[touched], ref[touched])
    assert np.array_equal(leaves[:CAPACITY], ref)
