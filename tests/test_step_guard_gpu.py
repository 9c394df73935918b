"""The plane engine's step guard and its long-horizon behaviour.

The uint8 Nature DQN path runs every GEMM on two scaled f16 planes (csrc/gemm_p3.h) whose
scales lag one step (the previous step's maximum with 2^8 of headroom).  A tensor whose
maximum grows more than ~2^8-fold in one step overflows its planes; the step guard
(kernels.h StepGuard) then skips the step on the device, the rule of automatic mixed
precision: no parameter, Adam moment / count, target or priority changes, and the rescale
sets the next step's scales from the skipped step's true maxima.

  * test_overflow_skips_step_and_recovers: a batch with |TD| ~ 1e-4 (a head scaled down by
    1e-4, r = d = 0) then one with |TD| ~ 1 (r = 1): the second step's head dZ grows ~2^13-fold
    and overflows.  Checked: nothing changed (bitwise), the priorities of the batch's keys
    were not written, the counts; then the same batch again is applied and matches the f64
    oracle teacher-forced from the GPU's state (loss / TD at 1e-5, gradients at the suite's
    bar, Adam at t = 2: the skipped step did not count).
  * test_gradient_error_matches_f32_engine: teacher-forced, every gradient tensor of the
    plane engine within 1.5x the exact-f32 engine's error against float64 (B = 64).
  * test_long_horizon_drift: free-running steps at B = 64 x 100, 256 x 50 and 512 x 20 from
    identical batches on the plane engine, on the exact-f32 engine
    (acme_set_matmul_engine(ACME_MATMUL_F32)) and on the float64 torch restatement
    (oracle/dqn_torch.py on the GPU, the reference trajectory), over 4 seeds.  The plane
    engine skips no step; its parameter drift and the maximum and median of its loss error,
    averaged over the seeds, are within 2x the f32 engine's (see the test).
  * test_underflow_only_skip_writes_no_priority / test_skipped_step_makes_no_target_copy:
    a skip decided by the rescale alone writes no priority on the fused path; a target copy
    due on a skipped step is not made.
  * test_learner_reissues_skipped_step: DQNLearner re-issues a skipped step (and the step
    held after it) so every step() applies one update, bit-identical to a learner that never
    skipped.
  * test_impala_timeout_skips_update: an LSTM unroll timeout (the timeout word set before the
    step) leaves parameters, moments and Adam's count unchanged and raises the skip count.

Reference: DQNLearner._step (acme/agents/tf/dqn/learning.py:121-148), IMPALALearner._step
(acme/agents/tf/impala/learning.py:97-169).
"""

import ctypes

import numpy as np
import pytest
import torch

from oracle import dqn_oracle as O

pytestmark = pytest.mark.gpu

HEAD = ("duelling_q_network/mlp/linear_1/w", "duelling_q_network/mlp_1/linear_1/w")


def _dev(batch):
    return [torch.as_tensor(batch[k]).cuda().contiguous()
            for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t", "probabilities")]


def _batch(rng, B, A, r=None, d=None):
    o1 = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    o2 = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
    rr = (rng.standard_normal(B) * 1.5).astype(np.float32) if r is None else np.full(B, r, np.float32)
    dd = (np.where(rng.random(B) < 0.2, 0.0, 0.99 ** 4).astype(np.float32) if d is None
          else np.full(B, d, np.float32))
    return dict(o_tm1=o1, a_tm1=rng.integers(0, A, B).astype(np.int32), r_t=rr, d_t=dd, o_t=o2,
                probabilities=rng.uniform(1e-6, 1e-3, B))


def _check_grads(g_gpu, g_ref):
    for name, ref in g_ref.items():
        got = g_gpu[name].reshape(ref.shape).astype(np.float64)
        scale = np.abs(ref).max()
        err = np.abs(got - ref)
        bound = 1e-4 * np.abs(ref) + 2e-5 * scale + 1e-30
        assert (err <= bound).all(), (name, float(err.max()), float(scale))


def _masks(d, params, o_tm1):
    """The kernel's ReLU pattern (forward checked against the f64 oracle first)."""
    cfg = O.DQNConfig(num_actions=18, network="nature")
    _, cache = O.forward(cfg, params, o_tm1, np.float64)
    masks = {}
    for name, ref in (("x1", cache["x1"]), ("x2", cache["x2"]), ("x3", cache["x3"]),
                      ("hid", cache["h"])):
        got = d.debug_buffer(name)[:ref.size].reshape(ref.shape)
        scale = np.abs(ref).max()
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=2e-6 * scale)
        m = got > 0
        flips = m != (ref > 0)
        assert (np.abs(ref[flips]) <= 2e-6 * scale).all(), name
        masks[name] = m
    return masks


def test_overflow_skips_step_and_recovers():
    from acme_amd.native import NativeDQN, NativeReplay
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    B = 64
    p0, t0 = net.init(1), net.init(2)
    for k in HEAD:  # q ~ 1e-4: |TD| ~ 1e-4 when r = d = 0
        p0[k] = p0[k] * 1e-4
        t0[k] = t0[k] * 1e-4
    d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
    d.set_params(p0, t0)
    table = NativeReplay(1000, [4], prioritized=True, priority_exponent=0.6, seed=5)
    rows = np.arange(600, dtype=np.uint32).view(np.uint8).reshape(600, 4)
    table.insert([rows], np.linspace(0.5, 2.0, 600))
    rng = np.random.default_rng(3)
    small = _batch(rng, B, 18, r=0.0, d=0.0)
    large = _batch(rng, B, 18, r=1.0, d=0.0)
    # Step 1: calibrated on the small batch, applied.
    keys = table.sample(B, 0)["keys"]
    d.step(*_dev(small), priority_update=(table.handle, keys))
    torch.cuda.synchronize()
    g1 = d.guard_state()
    assert g1["applied"] == 1 and g1["skipped"] == 0, g1
    state1 = {buf: d.get_params(buf) for buf in ("params", "target", "m", "v")}
    raw1 = table.export_state()["raw_priorities"].copy()
    # Step 2: |TD| jumps ~1e4-fold: the head dZ planes overflow; nothing may change.
    keys2 = table.sample(B, 1)["keys"]
    d.step(*_dev(large), priority_update=(table.handle, keys2))
    torch.cuda.synchronize()
    g2 = d.guard_state()
    assert g2["applied"] == 1 and g2["skipped"] == 1 and g2["last_skipped"] == 1, g2
    assert d.skipped_steps == 1  # the pinned host mirror
    assert d.num_steps == 2      # step() calls (the target period)
    for buf, ref in state1.items():
        got = d.get_params(buf)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{buf}/{k}")
    np.testing.assert_array_equal(table.export_state()["raw_priorities"], raw1)
    # Step 3: the same batch at the rescaled planes: applied, and exact against the oracle.
    params1, target1 = state1["params"], state1["target"]
    q = torch.empty(B, 18, device="cuda")
    d.step(*_dev(large), q_tm1=q)
    torch.cuda.synchronize()
    g3 = d.guard_state()
    assert g3["applied"] == 2 and g3["skipped"] == 1 and g3["last_skipped"] == 0, g3
    masks = _masks(d, params1, large["o_tm1"])
    cfg = O.DQNConfig(num_actions=18, network="nature")
    out, grads = O.dqn_loss_and_grads(cfg, params1, target1, large, np.float64, masks=masks)
    np.testing.assert_allclose(q.cpu().numpy(), out["q_tm1"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(d.loss.item(), out["loss"], rtol=1e-5)
    np.testing.assert_allclose(d.td_error[:B].cpu().numpy(), out["td_error"], rtol=1e-5, atol=1e-6)
    gg = d.get_params("grads")
    _check_grads(gg, grads)
    # Adam at t = 2 on the GPU's own gradients (the skipped step did not count).
    got = d.get_params("params")
    for k in got:
        want, _, _ = O.adam_update(params1[k], gg[k], state1["m"][k], state1["v"][k], 2, 1e-3)
        np.testing.assert_allclose(got[k], want, rtol=1e-6, atol=1e-9, err_msg=k)


def _head_scaled_params(net, scale=1e-4):
    p0, t0 = net.init(1), net.init(2)
    for k in HEAD:  # q ~ scale: |TD| ~ scale when r = d = 0
        p0[k] = p0[k] * scale
        t0[k] = t0[k] * scale
    return p0, t0


def test_underflow_only_skip_writes_no_priority():
    """A step whose only fault is an underflow (a tensor's maximum fell more than ~2^7-fold
    below its scale, so its planes carry too few bits) is skipped by the end-of-step
    rescale, and the priority write-back fused into the same launch (acme_dqn_step_update)
    must follow that verdict: no priority of the batch is written."""
    from acme_amd.native import NativeDQN, NativeReplay
    from acme_amd.networks import DQNAtariNetwork
    B = 64
    p0, t0 = _head_scaled_params(DQNAtariNetwork(18))
    # A small learning rate keeps q ~ 1e-4 after the first update (Adam moves every
    # parameter by about lr), so the second batch's |TD| stays ~1e-4.
    d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8",
                  learning_rate=1e-7)
    d.set_params(p0, t0)
    table = NativeReplay(1000, [4], prioritized=True, priority_exponent=0.6, seed=5)
    rows = np.arange(600, dtype=np.uint32).view(np.uint8).reshape(600, 4)
    table.insert([rows], np.linspace(0.5, 2.0, 600))
    rng = np.random.default_rng(4)
    large = _batch(rng, B, 18, r=1.0, d=0.0)   # |TD| ~ 1
    small = _batch(rng, B, 18, r=0.0, d=0.0)   # |TD| ~ 1e-4: the head dZ shrinks ~2^13-fold
    d.step(*_dev(large), priority_update=(table.handle, table.sample(B, 0)["keys"]))
    torch.cuda.synchronize()
    assert d.guard_state()["applied"] == 1
    raw1 = table.export_state()["raw_priorities"].copy()
    state1 = {buf: d.get_params(buf) for buf in ("params", "m", "v")}
    d.step(*_dev(small), priority_update=(table.handle, table.sample(B, 1)["keys"]))
    torch.cuda.synchronize()
    g = d.guard_state()
    assert g["skipped"] == 1 and g["last_skipped"] == 1, g
    assert not d.plane_overflow(), "the skip must come from the underflow test alone"
    np.testing.assert_array_equal(table.export_state()["raw_priorities"], raw1)
    for buf, ref in state1.items():
        got = d.get_params(buf)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{buf}/{k}")


def test_skipped_step_makes_no_target_copy():
    """A target copy due on a skipped step (num_steps % period == 0) is not made: the stale
    target stays (agents/tf/dqn/learning.py:157-161 copies after an update)."""
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    B = 64
    p0, t0 = _head_scaled_params(DQNAtariNetwork(18))
    # A small learning rate keeps q ~ 1e-4 after the updates (Adam moves every parameter by
    # about lr), so only the large batch jumps.
    d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8",
                  target_update_period=2, learning_rate=1e-7)
    d.set_params(p0, t0)
    rng = np.random.default_rng(5)
    small = [_batch(rng, B, 18, r=0.0, d=0.0) for _ in range(2)]
    large = _batch(rng, B, 18, r=1.0, d=0.0)
    d.step(*_dev(small[0]))  # num_steps 0: copy
    d.step(*_dev(small[1]))  # num_steps 1: the online parameters move, the target is stale
    torch.cuda.synchronize()
    tgt1, prm1 = d.get_params("target"), d.get_params("params")
    assert any(not np.array_equal(tgt1[k], prm1[k]) for k in tgt1)
    d.step(*_dev(large))     # num_steps 2: copy due, the step overflows and is skipped
    torch.cuda.synchronize()
    g = d.guard_state()
    assert g["skipped"] == 1 and g["last_skipped"] == 1, g
    for k, v in d.get_params("target").items():
        np.testing.assert_array_equal(v, tgt1[k], err_msg=k)


class _FixedBatches:
    """A dataset of fixed device batches, each ReplaySample handed out once (each in its own
    tensors, so every batch stays intact)."""
    holds_last_batches = 1 << 30

    def __init__(self, samples):
        self.samples = list(samples)
        self.batch_size = int(samples[0].data[1].shape[0])

    def __iter__(self):
        return self

    def __next__(self):
        return self.samples.pop(0)


class _ReusingBatches:
    """A dataset that writes every batch into the same device buffers (a foreign iterator
    without the repo iterators' buffer ring): the learner must hold its own copies."""

    def __init__(self, samples):
        self.samples = list(samples)
        self.batch_size = int(samples[0].data[1].shape[0])
        self.buf = None

    def __iter__(self):
        return self

    def __next__(self):
        from acme_amd import replay
        s = self.samples.pop(0)
        flat = list(s.data) + [s.info.key, s.info.probability]
        if self.buf is None:
            self.buf = [torch.empty_like(x) for x in flat]
        for dst, src in zip(self.buf, flat):
            dst.copy_(src)
        info = replay.SampleInfo(key=self.buf[5], probability=self.buf[6],
                                 table_size=s.info.table_size, priority=s.info.priority)
        return replay.ReplaySample(info=info, data=tuple(self.buf[:5]))


def _sample(b, first_key):
    from acme_amd import replay
    dev = _dev(b)
    B = dev[1].shape[0]
    keys = torch.arange(first_key, first_key + B, dtype=torch.int64, device="cuda").view(
        torch.uint64)
    zeros = torch.zeros(B, dtype=torch.float64, device="cuda")
    info = replay.SampleInfo(key=keys, probability=dev[5],
                             table_size=torch.zeros(B, dtype=torch.int64, device="cuda"),
                             priority=zeros)
    return replay.ReplaySample(info=info, data=tuple(dev[:5]))


@pytest.mark.parametrize("dataset", ["fixed", "reusing"])
def test_learner_reissues_skipped_step(dataset):
    """DQNLearner.step() applies every step, as the reference (agents/tf/dqn/learning.py:
    147-161): a step the guard skips (here the forced ~2^13-fold head-dZ jump) holds the
    steps after it skipped too, and the learner re-issues them in order at the next step()
    (or when its state is read), with their step counters, so the due target copy lands.
    Checked bit for bit against a learner that recalibrated before the large batch (so it
    never skips), both writing their priorities back into their own tables.  With a dataset
    that reuses one set of buffers ("reusing") the learner holds copies of the
    batches it may re-issue."""
    from acme_amd import replay, specs
    from acme_amd.adders import reverb as adders
    from acme_amd.agents.dqn import DQNLearner
    from acme_amd.networks import DQNAtariNetwork
    from acme_amd.utils import loggers
    B, A = 64, 18
    net = DQNAtariNetwork(A)
    p0, t0 = _head_scaled_params(net)
    rng = np.random.default_rng(6)
    batches = [_batch(rng, B, A, r=0.0, d=0.0), _batch(rng, B, A, r=1.0, d=0.0),
               _batch(rng, B, A), _batch(rng, B, A), _batch(rng, B, A)]
    spec = specs.EnvironmentSpec(
        observations=specs.Array((84, 84, 4), np.uint8), actions=specs.DiscreteArray(A, np.int32),
        rewards=specs.Array((), np.float32), discounts=specs.BoundedArray((), np.float32, 0, 1))

    def make(recalibrate_before=None):
        table = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Prioritized(0.6),
                             replay.selectors.Fifo(), 1000, replay.rate_limiters.MinSize(1),
                             signature=adders.NStepTransitionAdder.signature(spec), seed=3)
        table.native.fill_synthetic(1000, layout=0, num_actions=A, seed=0)
        server = replay.Server([table])
        kind = _ReusingBatches if recalibrate_before is None and dataset == "reusing" \
            else _FixedBatches
        ds = kind([_sample(b, 64 * i) for i, b in enumerate(batches)])
        lr = DQNLearner(net, net, discount=0.99, importance_sampling_exponent=0.2,
                        learning_rate=1e-3, target_update_period=2, dataset=ds,
                        replay_client=replay.Client(server), logger=loggers.NoOpLogger(),
                        seed=0)
        lr.native.set_params(p0, t0)
        for i in range(len(batches)):
            if i == recalibrate_before:
                torch.cuda.synchronize()
                lr.native.params_changed()
            lr.step()
        state = lr.save()  # settles: every issued step decided, a skipped one re-issued
        return lr, state, table.native.export_state()["raw_priorities"]

    got, s_got, raw_got = make()
    ref, s_ref, raw_ref = make(recalibrate_before=1)
    g_got, g_ref = got.native.guard_state(), ref.native.guard_state()
    assert g_ref["skipped"] == 0 and g_ref["applied"] == len(batches), g_ref
    # The large batch was skipped, with the batch issued after it held; both re-issued.
    assert g_got["skipped"] == 2 and g_got["applied"] == len(batches), g_got
    assert got._reissued == 2  # noqa: SLF001
    assert got._copy_held == (dataset == "reusing")  # noqa: SLF001
    assert s_got["num_steps"] == s_ref["num_steps"] == len(batches)
    assert s_got["optimizer"]["step"] == s_ref["optimizer"]["step"] == len(batches)
    for part in ("network", "target_network"):
        for k in s_ref[part]:
            np.testing.assert_array_equal(s_got[part][k], s_ref[part][k], err_msg=f"{part}/{k}")
    for mom in ("m", "v"):
        for k in s_ref["optimizer"][mom]:
            np.testing.assert_array_equal(s_got["optimizer"][mom][k], s_ref["optimizer"][mom][k],
                                          err_msg=f"{mom}/{k}")
    np.testing.assert_array_equal(raw_got, raw_ref)
    assert not np.array_equal(raw_got[:64 * len(batches)], np.ones(64 * len(batches)))


def _rel(a, b, base):
    num = sum(float(np.sum((a[k].astype(np.float64) - b[k]) ** 2)) for k in a)
    den = sum(float(np.sum((b[k] - base[k].astype(np.float64)) ** 2)) for k in a)
    return (num / max(den, 1e-300)) ** 0.5


def _teacher_forced(d, params, target, b, B):
    """The step just taken against the f64 oracle from the GPU's own pre-step state."""
    masks = _masks(d, params, b["o_tm1"])
    cfg = O.DQNConfig(num_actions=18, network="nature")
    out, grads = O.dqn_loss_and_grads(cfg, params, target, b, np.float64, masks=masks)
    np.testing.assert_allclose(d.loss.item(), out["loss"], rtol=1e-5)
    # TD = target - q_tm1[a] cancels: its absolute error follows |q| (which grows as
    # training moves the head), so the floor scales with max |q|.
    qs = float(np.abs(out["q_tm1"]).max())
    np.testing.assert_allclose(d.td_error[:B].cpu().numpy(), out["td_error"], rtol=1e-5,
                               atol=1e-6 * max(1.0, qs))
    _check_grads(d.get_params("grads"), grads)


def _grad_errors(B, seed=0):
    """Per-tensor relative Frobenius error of one step's gradients against float64, teacher-
    forced from the same parameters, for the plane and the exact-f32 engine."""
    from acme_amd._lib import lib
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    from oracle.dqn_torch import TorchDQN
    net = DQNAtariNetwork(18)
    p0, t0 = net.init(11 + 2 * seed), net.init(12 + 2 * seed)
    b = _batch(np.random.default_rng(1000 + B + 7919 * seed), B, 18)
    ref = TorchDQN(p0, 18, target=t0, dtype=torch.float64, device="cuda")
    dev = {k: torch.as_tensor(b[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
    ref.step(dev["o_tm1"], dev["a_tm1"], dev["r_t"].double(), dev["d_t"].double(), dev["o_t"],
             b["probabilities"])
    g_ref = {k: ref.m[k].cpu().numpy() / 0.1 for k in ref.names}  # Adam's m = 0.1 g at t = 1
    out = {}
    for eng, code in (("plane", 1), ("f32", 0)):
        lib().acme_set_matmul_engine(code)
        try:
            d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
            d.set_params(p0, t0)
            d.forward_backward(*_dev(b))
            torch.cuda.synchronize()
            g = d.get_params("grads")
        finally:
            lib().acme_set_matmul_engine(1)
        out[eng] = {k: float(np.linalg.norm(g[k].reshape(r.shape) - r) / np.linalg.norm(r))
                    for k, r in g_ref.items()}
    return out


def test_gradient_error_matches_f32_engine():
    """The plane engine's gradients are as accurate as the exact-f32 engine's, tensor by
    tensor, teacher-forced from the same parameters against float64 (B = 64, the batch where
    round 5 found its conv weight gradients at 2.5-7x the f32 engine's error: a biased f16
    MFMA accumulation, now split, csrc/gemm_p3.h P3Acc; profiles/r06/accuracy/).  Bar: within
    1.5x the f32 engine's error, for every weight and bias."""
    e = _grad_errors(64)
    for k in e["f32"]:
        print(f"{k:42s} plane {e['plane'][k]:.2e} f32 {e['f32'][k]:.2e}")
    for k in e["f32"]:
        assert e["plane"][k] <= 1.5 * e["f32"][k] + 1e-8, (k, e["plane"][k], e["f32"][k])


DRIFT_SEEDS = 6


@pytest.mark.parametrize("B,steps", [(64, 100), (256, 50), (512, 20)])
def test_long_horizon_drift(B, steps):
    """Free-running trajectories (each side applies its own gradients) of the plane engine
    and the exact-f32 engine from identical batches, against the float64 torch restatement
    (oracle/dqn_torch.py on the GPU, the reference trajectory), at a small batch, the
    reference DQN agent's default batch (256, agents/tf/dqn/agent.py:49) and the headline
    one, over DRIFT_SEEDS seeds (initial parameters and batch streams).

    A ReLU whose pre-activation lies within an engine's rounding of zero switches on one side
    and not on the other, and from there the trajectories part chaotically, so a single
    seed's numbers are draws (profiles/r06/drift/: per seed, either engine's maximum loss
    error ranges over 100x, and each engine is ahead at some seeds).  Asserted (VERDICT r5
    item 1): no skipped step; every seed's first loss matches float64 at the north star's
    1e-5 on both engines; the plane engine's parameter drift from the float64 trajectory
    (relative to how far training moved the parameters), and the maximum and the median of
    its loss trajectory's relative error, each averaged over the seeds, within 2x the
    exact-f32 engine's.  At seed 0 the plane engine's step is also checked teacher-forced
    against the f64 oracle from its own pre-step state at the first and last step (loss and
    TD at 1e-5, the suite's gradient bar), so per-step accuracy does not degrade as the
    scales follow training."""
    from acme_amd._lib import lib
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    from oracle.dqn_torch import TorchDQN
    net = DQNAtariNetwork(18)
    metrics = {"plane": [], "f32": []}
    for seed in range(DRIFT_SEEDS):
        p0, t0 = net.init(11 + 2 * seed), net.init(12 + 2 * seed)

        def batches():
            rng = np.random.default_rng(1000 + B + 7919 * seed)
            for _ in range(steps):
                yield _batch(rng, B, 18)

        ref = TorchDQN(p0, 18, target=t0, dtype=torch.float64, device="cuda")
        ref_loss = []
        for b in batches():
            dev = {k: torch.as_tensor(b[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
            loss, _ = ref.step(dev["o_tm1"], dev["a_tm1"], dev["r_t"].double(),
                               dev["d_t"].double(), dev["o_t"], b["probabilities"])
            ref_loss.append(loss)
        ref_p = {k: v.detach().cpu().numpy() for k, v in ref.p.items()}
        ref_loss = np.array(ref_loss)

        def run(engine, check=()):
            lib().acme_set_matmul_engine(engine)
            try:
                d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8")
                d.set_params(p0, t0)
                losses = []
                for i, b in enumerate(batches()):
                    pre = (d.get_params("params"), d.get_params("target")) if i in check else None
                    d.step(*_dev(b))
                    losses.append(d.loss.clone())
                    if pre is not None:
                        torch.cuda.synchronize()
                        _teacher_forced(d, pre[0], pre[1], b, B)
                torch.cuda.synchronize()
                return (np.array([x.item() for x in losses]), d.get_params("params"),
                        d.guard_state())
            finally:
                lib().acme_set_matmul_engine(1)

        for eng, code in (("plane", 1), ("f32", 0)):
            losses, params, g = run(code, (0, steps - 1) if seed == 0 and eng == "plane" else ())
            assert g["skipped"] == 0 and g["applied"] == steps, (eng, seed, g)
            np.testing.assert_allclose(losses[:1], ref_loss[:1], rtol=1e-5)
            e = np.abs(losses - ref_loss) / np.abs(ref_loss)
            metrics[eng].append((_rel(params, ref_p, p0), e.max(), np.median(e)))
        print(f"B={B} seed {seed}: " + "  ".join(
            f"{eng} drift {m[-1][0]:.3e} loss max {m[-1][1]:.3e} median {m[-1][2]:.3e}"
            for eng, m in metrics.items()))
    mp, mf = np.mean(metrics["plane"], axis=0), np.mean(metrics["f32"], axis=0)
    print(f"B={B} steps={steps}, mean over {DRIFT_SEEDS} seeds: drift plane {mp[0]:.3e} f32 "
          f"{mf[0]:.3e}; loss rel err max plane {mp[1]:.3e} f32 {mf[1]:.3e}; median plane "
          f"{mp[2]:.3e} f32 {mf[2]:.3e}")
    for i, name in enumerate(("drift", "loss max", "loss median")):
        assert mp[i] <= 2.0 * mf[i] + 1e-6, (name, mp[i], mf[i])


def test_impala_timeout_skips_update():
    from acme_amd import _lib
    from acme_amd.native import NativeIMPALA, _memcpy_dtod
    from acme_amd.networks import IMPALAAtariNetwork
    net = IMPALAAtariNetwork(18)
    B, T = 4, 20
    n = NativeIMPALA(num_actions=18, max_batch=B, max_sequence_length=T, torso="atari",
                     learning_rate=1e-3)
    n.set_params(net.init(0))
    rng = np.random.default_rng(0)

    def batch():
        return [torch.as_tensor(x).cuda().contiguous() for x in (
            rng.integers(0, 256, (B, T, 84, 84, 4), dtype=np.uint8),
            rng.integers(0, 18, (B, T)).astype(np.int32), rng.standard_normal((B, T)).astype(np.float32),
            rng.integers(0, 18, (B, T)).astype(np.int32), rng.standard_normal((B, T)).astype(np.float32),
            np.full((B, T), 0.99, np.float32), rng.standard_normal((B, T, 18)).astype(np.float32),
            np.zeros((B, 256), np.float32), np.zeros((B, 256), np.float32))]

    n.step(*batch())
    torch.cuda.synchronize()
    assert n.guard_state()["applied"] == 1
    before = {buf: n.get_params(buf) for buf in ("params", "m", "v")}
    # The timeout word the one-launch LSTM unroll writes on a spin timeout.
    p, c = ctypes.c_void_p(), ctypes.c_int64()
    _lib.check(_lib.lib().acme_impala_debug_buffer(n._h, b"lstm_timeout_step", ctypes.byref(p),
                                                   ctypes.byref(c)))
    one = torch.ones(1, dtype=torch.int32, device=n.device)
    torch.cuda.synchronize()
    _memcpy_dtod(p.value, one.data_ptr(), 4)
    n.step(*batch())
    torch.cuda.synchronize()
    g = n.guard_state()
    assert g["applied"] == 1 and g["skipped"] == 1 and g["last_skipped"] == 1, g
    assert g["lstm_timeouts"] == 1 and n.skipped_steps == 1
    for buf, ref in before.items():
        got = n.get_params(buf)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{buf}/{k}")
    n.step(*batch())
    torch.cuda.synchronize()
    assert n.guard_state()["applied"] == 2
    assert any(not np.array_equal(n.get_params("params")[k], before["params"][k])
               for k in before["params"])
