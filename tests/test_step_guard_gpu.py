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
  * test_long_horizon_drift: 100 free-running steps at B = 64 (and 20 at the headline
    B = 512) from identical batches on the plane engine, on the exact-f32 engine
    (acme_set_matmul_engine(ACME_MATMUL_F32)) and on the float64 torch restatement
    (oracle/dqn_torch.py on the GPU, the reference trajectory).  The plane engine skips no
    step, and its drift from the f64 trajectory (parameters, relative to how far training
    moved them; the loss trajectory) stays within the f32 engine's own drift (x2, plus a
    floor at f32 rounding).
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
# Free-running drift from the f64 trajectory relative to the exact-f32 engine's.  A plane
# product drops the l*l term (<= 2^-22 of the product) where the f32 MFMA rounds at 2^-24,
# so the plane engine's per-step error is up to ~4x the f32 engine's, and free-running
# trajectories (chaotic: Adam's normalised steps flip on near-zero gradients) leave the f64
# one earlier.  Measured at B = 64 x 100 steps: 0.152 against 0.065 (round 4).  A build
# with -DP3_FOUR_TERMS=1 adds the l*l term (+5% step time).
PLANE_DRIFT_FACTOR = 4.0


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


@pytest.mark.parametrize("B,steps,checks", [(64, 100, (0, 33, 66, 99)), (512, 20, (0, 19))])
def test_long_horizon_drift(B, steps, checks):
    """Free-running trajectories (each side applies its own gradients) of the plane engine,
    the exact-f32 engine and the float64 restatement, from identical batches; at the
    `checks` steps the plane engine's step is also checked teacher-forced against the f64
    oracle from its own pre-step state (the north star's 1e-5 on the loss and TD, the
    suite's gradient bar), so the per-step accuracy is shown not to degrade while the
    scales follow 100 steps of training."""
    from acme_amd._lib import lib
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    from oracle.dqn_torch import TorchDQN
    net = DQNAtariNetwork(18)
    p0, t0 = net.init(11), net.init(12)

    def batches():
        rng = np.random.default_rng(1000 + B)
        for _ in range(steps):
            yield _batch(rng, B, 18)

    # The float64 reference trajectory (torch on the GPU).
    ref = TorchDQN(p0, 18, target=t0, dtype=torch.float64, device="cuda")
    ref_loss = []
    for b in batches():
        dev = {k: torch.as_tensor(b[k]).cuda() for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
        loss, _ = ref.step(dev["o_tm1"], dev["a_tm1"], dev["r_t"].double(), dev["d_t"].double(),
                           dev["o_t"], b["probabilities"])
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

    plane_loss, plane_p, plane_g = run(1, checks)
    f32_loss, f32_p, f32_g = run(0)
    assert plane_g["skipped"] == 0 and plane_g["applied"] == steps, plane_g
    assert f32_g["skipped"] == 0 and f32_g["applied"] == steps, f32_g
    # The first steps match the f64 trajectory at the north star's 1e-5.
    np.testing.assert_allclose(plane_loss[:2], ref_loss[:2], rtol=1e-5)
    np.testing.assert_allclose(f32_loss[:2], ref_loss[:2], rtol=1e-5)
    d_plane = _rel(plane_p, ref_p, p0)
    d_f32 = _rel(f32_p, ref_p, p0)
    e_plane = np.abs(plane_loss - ref_loss) / np.abs(ref_loss)
    e_f32 = np.abs(f32_loss - ref_loss) / np.abs(ref_loss)
    print(f"B={B} steps={steps}: parameter drift plane {d_plane:.3e} f32 {d_f32:.3e}; "
          f"max loss rel err plane {e_plane.max():.3e} f32 {e_f32.max():.3e}")
    assert d_plane <= PLANE_DRIFT_FACTOR * d_f32 + 1e-5, (d_plane, d_f32)


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
