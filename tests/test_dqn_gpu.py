"""HIP DQN learner step vs the numpy oracle (oracle/dqn_oracle.py, float64).

Reference: DQNLearner._step (acme/agents/tf/dqn/learning.py:112-168).
Tolerances (fp32 kernels against an fp64 restatement):
  q values, loss, TD errors, priorities: rtol 1e-5 (north_star loss parity 1e-5)
  gradients: per tensor |g - g_ref| <= 1e-4 |g_ref| + 2e-5 max|g_ref| (fp32 sums over
             up to 225,792 terms in a different order)
  Adam given identical gradients: rtol 1e-6 (same f32 op order).
"""

import numpy as np
import pytest
import torch

from oracle import dqn_oracle as O

pytestmark = pytest.mark.gpu


def _batch(rng, B, obs_shape, A, u8=True, probs=None):
    if u8:
        o1 = rng.integers(0, 256, (B,) + obs_shape, dtype=np.uint8)
        o2 = rng.integers(0, 256, (B,) + obs_shape, dtype=np.uint8)
    else:
        o1 = rng.standard_normal((B,) + obs_shape).astype(np.float32)
        o2 = rng.standard_normal((B,) + obs_shape).astype(np.float32)
    return dict(o_tm1=o1, a_tm1=rng.integers(0, A, B).astype(np.int32),
                r_t=(rng.standard_normal(B) * 1.5).astype(np.float32),
                d_t=np.where(rng.random(B) < 0.2, 0.0, 0.99 ** 4).astype(np.float32),
                o_t=o2,
                probabilities=probs if probs is not None else rng.uniform(1e-6, 1e-3, B))


def _dev(batch):
    return [torch.as_tensor(batch[k]).cuda().contiguous()
            for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t", "probabilities")]


def _learner(net, B, **kw):
    from acme_amd.native import NativeDQN
    if net.kind == "nature":
        return NativeDQN(network="nature", num_actions=net.num_actions, max_batch=B,
                         obs_dtype=net.obs_dtype, **kw)
    return NativeDQN(network="mlp", num_actions=net.num_actions, max_batch=B,
                     obs_dtype=net.obs_dtype, obs_dim=net.obs_dim, hidden=net.hidden, **kw)


def _cfg(net, **kw):
    if net.kind == "nature":
        return O.DQNConfig(num_actions=net.num_actions, network="nature", **kw)
    return O.DQNConfig(num_actions=net.num_actions, network="mlp", obs_dim=net.obs_dim,
                       hidden=net.hidden, **kw)


def _check_grads(g_gpu, g_ref):
    for name, ref in g_ref.items():
        got = g_gpu[name].reshape(ref.shape).astype(np.float64)
        scale = np.abs(ref).max()
        err = np.abs(got - ref)
        bound = 1e-4 * np.abs(ref) + 2e-5 * scale + 1e-30
        assert (err <= bound).all(), (name, float(err.max()), float(scale))


def _relu_masks(d, net, batch, params, B):
    """Forward activations of the kernel vs the f64 oracle (tolerance), then the kernel's
    own ReLU pattern, so that the backward comparison is conditional on the same branch
    decisions.  Disagreements are only allowed where the f64 pre-activation is within
    fp32 rounding of zero."""
    cfg = _cfg(net)
    _, cache = O.forward(cfg, params, batch["o_tm1"], np.float64)
    if net.kind == "nature":
        pairs = [("x1", cache["x1"]), ("x2", cache["x2"]), ("x3", cache["x3"]),
                 ("hid", cache["h"])]
    else:
        pairs = [(f"act{i}", cache["acts"][i + 1]) for i in range(len(net.hidden))]
    masks = {}
    for name, ref in pairs:
        got = d.debug_buffer(name)[:ref.size].reshape(ref.shape)
        scale = np.abs(ref).max()
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=2e-6 * scale)
        m = got > 0
        flips = m != (ref > 0)
        assert (np.abs(ref[flips]) <= 2e-6 * scale).all(), name
        assert flips.mean() < 1e-4, (name, flips.mean())
        masks[name] = m
    return masks


NETS = {
    "nature": lambda: __import__("acme_amd.networks", fromlist=["x"]).DQNAtariNetwork(18),
    # A != 18 takes the generic head kernel (fc_head_forward_kernel) instead of the Nature one.
    "nature_a6": lambda: __import__("acme_amd.networks", fromlist=["x"]).DQNAtariNetwork(6),
    "cartpole_mlp": lambda: __import__("acme_amd.networks", fromlist=["x"]).MLP(4, [50, 50], 2),
    "mlp_vec": lambda: __import__("acme_amd.networks", fromlist=["x"]).MLP(24, [64, 32], 6),
}


@pytest.mark.parametrize("netname,B", [("nature", 1), ("nature", 4), ("nature", 37),
                                       ("nature", 200), ("nature", 512), ("nature_a6", 37),
                                       ("cartpole_mlp", 32), ("mlp_vec", 100)])
def test_forward_backward_matches_oracle(netname, B):
    net = NETS[netname]()
    rng = np.random.default_rng(B)
    params = net.init(seed=1)
    target = net.init(seed=2)
    u8 = net.obs_dtype == "uint8"
    batch = _batch(rng, B, net.obs_shape, net.num_actions, u8=u8)
    d = _learner(net, B)
    d.set_params(params, target)
    q = torch.empty(B, net.num_actions, device="cuda")
    d.forward_backward(*_dev(batch), q_tm1=q)
    torch.cuda.synchronize()
    masks = _relu_masks(d, net, batch, params, B)
    out, grads = O.dqn_loss_and_grads(_cfg(net), params, target, batch, np.float64,
                                      masks=masks)
    np.testing.assert_allclose(q.cpu().numpy(), out["q_tm1"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(d.loss.item(), out["loss"], rtol=1e-5)
    np.testing.assert_allclose(d.td_error[:B].cpu().numpy(), out["td_error"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(d.priorities[:B].cpu().numpy(), out["priorities"], rtol=1e-5,
                               atol=1e-6)
    _check_grads(d.get_params("grads"), grads)


def test_single_stream_schedule_bitwise():
    """ACME_V_SIDE=1 at creation (every launch on the caller's stream, the profiling
    schedule) computes the same step as the default two-stream schedule: the side stream
    only reorders independent launches, each with its own deterministic split-K scratch."""
    from acme_amd._lib import lib
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    B = 37
    p0, t0 = net.init(3), net.init(4)
    a = _learner(net, B)
    lib().acme_tune_set(b"SIDE", 1)  # read once, at the learner's creation
    try:
        b = _learner(net, B)
    finally:
        lib().acme_tune_set(b"SIDE", 0)
    a.set_params(p0, t0)
    b.set_params(p0, t0)
    rng = np.random.default_rng(8)
    for _ in range(2):
        dev = _dev(_batch(rng, B, (84, 84, 4), 18))
        a.step(*dev)
        b.step(*dev)
        torch.cuda.synchronize()
        assert a.loss.item() == b.loss.item()
        for buf in ("grads", "params", "m", "v"):
            ga, gb = a.get_params(buf), b.get_params(buf)
            for k in ga:
                np.testing.assert_array_equal(ga[k], gb[k], err_msg=f"{buf}/{k}")


def test_warp_specialised_gemms_bitwise():
    """fc_fwd, fc_dgrad, conv2_fwd and conv1_wgrad run on gemm_p3ws_kernel (producer / consumer waves,
    fragment reads one k16 step ahead): the consumers execute
    the same fragment reads and MFMAs over the same stages as the single-role kernels
    (ACME_V_WSN=1), so the step is bit-identical (B = 37: partial tiles; B = 512: the
    bench's grids)."""
    from acme_amd._lib import lib
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    for B in (37, 512):
        p0, t0 = net.init(3), net.init(4)
        lib().acme_tune_set(b"WSN", 1)  # read once, at the learner's creation
        try:
            a = _learner(net, B)
        finally:
            lib().acme_tune_set(b"WSN", 0)
        b = _learner(net, B)
        a.set_params(p0, t0)
        b.set_params(p0, t0)
        rng = np.random.default_rng(B)
        for _ in range(2):
            dev = _dev(_batch(rng, B, (84, 84, 4), 18))
            a.step(*dev)
            b.step(*dev)
            torch.cuda.synchronize()
            assert a.loss.item() == b.loss.item(), B
            for buf in ("grads", "params", "m", "v"):
                ga, gb = a.get_params(buf), b.get_params(buf)
                for k in ga:
                    np.testing.assert_array_equal(ga[k], gb[k], err_msg=f"B={B} {buf}/{k}")


def test_adam_and_target_copy_cadence():
    from acme_amd.networks import MLP
    net = MLP(4, [50, 50], 2)
    B = 32
    rng = np.random.default_rng(0)
    p0 = net.init(seed=3)
    d = _learner(net, B, target_update_period=2, learning_rate=1e-3)
    d.set_params(p0, p0)
    cfg = _cfg(net, target_update_period=2)
    m = {k: np.zeros_like(v) for k, v in p0.items()}
    v = {k: np.zeros_like(v) for k, v in p0.items()}
    params, target = p0, p0
    for step in range(4):
        batch = _batch(rng, B, net.obs_shape, net.num_actions, u8=False)
        d.forward_backward(*_dev(batch))
        g = d.get_params("grads")
        d.apply()
        torch.cuda.synchronize()
        # Adam on the GPU's own gradients (isolates the optimizer kernel).
        newp = {}
        for k in params:
            newp[k], m[k], v[k] = O.adam_update(params[k], g[k], m[k], v[k], step + 1, 1e-3)
        got = d.get_params("params")
        for k in newp:
            np.testing.assert_allclose(got[k], newp[k], rtol=1e-6, atol=1e-9)
        params = got
        if step % 2 == 0:  # copy AFTER the update (learning.py:157-161)
            target = got
        tg = d.get_params("target")
        for k in target:
            np.testing.assert_array_equal(tg[k], target[k])
        assert d.num_steps == step + 1
    del cfg


def test_full_step_trajectory_matches_oracle():
    """Three consecutive steps (incl. the step-0 target copy) vs the f64 oracle."""
    from acme_amd.networks import MLP
    net = MLP(8, [32, 32], 4)
    B = 64
    rng = np.random.default_rng(11)
    p0 = net.init(seed=5)
    t0 = net.init(seed=6)
    d = _learner(net, B, target_update_period=100)
    d.set_params(p0, t0)
    cfg = _cfg(net)
    state = dict(params=p0, target=t0, m={k: np.zeros_like(x) for k, x in p0.items()},
                 v={k: np.zeros_like(x) for k, x in p0.items()}, num_steps=0)
    for _ in range(3):
        batch = _batch(rng, B, net.obs_shape, net.num_actions, u8=False)
        d.step(*_dev(batch))
        out, _, state = O.dqn_step(cfg, state, batch, np.float64)
        torch.cuda.synchronize()
        np.testing.assert_allclose(d.loss.item(), out["loss"], rtol=1e-5)
        got = d.get_params("params")
        # Adam normalises the update: elements whose gradient is at the fp32 noise
        # floor may move by up to lr in either direction, so compare with atol = lr.
        for k in got:
            np.testing.assert_allclose(got[k], state["params"][k], rtol=1e-5, atol=1e-3 + 1e-6)
            frac = np.mean(np.abs(got[k] - state["params"][k]) <= 1e-5 * np.abs(state["params"][k]) + 1e-6)
            assert frac > 0.98, (k, frac)


def test_fused_step_equals_staged_step_bitwise():
    """acme_dqn_step (dense Adam on the side stream beside the torso backward, one join)
    and forward_backward + apply (single ordering) give bit-identical parameters, Adam
    moments, target and planes over steps that include a target copy."""
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    B = 32
    p0, t0 = net.init(1), net.init(2)
    a = _learner(net, B, target_update_period=2)
    b = _learner(net, B, target_update_period=2)
    a.set_params(p0, t0)
    b.set_params(p0, t0)
    rng = np.random.default_rng(11)
    for _ in range(3):
        dev = _dev(_batch(rng, B, (84, 84, 4), 18))
        a.step(*dev)
        b.forward_backward(*dev)
        b.apply()
        torch.cuda.synchronize()
        for buf in ("params", "target", "m", "v"):
            ga, gb = a.get_params(buf), b.get_params(buf)
            for k in ga:
                np.testing.assert_array_equal(ga[k], gb[k], err_msg=f"{buf}/{k}")
        assert a.loss.item() == b.loss.item()


@pytest.mark.parametrize("path", ["stages_2_4_1", "rccl_world1"])
def test_data_parallel_step_equals_fused_step_bitwise(path):
    """The data-parallel rank's step on one GPU equals acme_dqn_step bit for bit, over steps
    with a target copy: stages 2, 4 (no join of the dense gradients; the caller's stream is
    ordered after them by dense_grads_ready), 1 and apply; and acme_dqn_dp_step over a
    one-rank RCCL communicator (every all-reduce of one rank is the identity)."""
    from acme_amd import native as N
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    B = 32
    p0, t0 = net.init(5), net.init(6)
    a = _learner(net, B, target_update_period=2)
    b = _learner(net, B, target_update_period=2)
    a.set_params(p0, t0)
    b.set_params(p0, t0)
    comm = None
    if path == "rccl_world1":
        comm = N.nccl_comm_init(N.nccl_unique_id(), 1, 0)
        b.dp_init(comm, 1)
    rng = np.random.default_rng(13)
    try:
        for _ in range(3):
            dev = _dev(_batch(rng, B, (84, 84, 4), 18))
            a.step(*dev)
            if comm is None:
                b.forward_backward_stage(2, *dev)
                b.forward_backward_stage(4, *dev)
                b.dense_grads_ready()
                b.forward_backward_stage(1, *dev)
                b.apply()
            else:
                b.dp_step(*dev)
            torch.cuda.synchronize()
            assert a.loss.item() == b.loss.item()
            for buf in ("params", "target", "m", "v"):
                ga, gb = a.get_params(buf), b.get_params(buf)
                for k in ga:
                    np.testing.assert_array_equal(ga[k], gb[k], err_msg=f"{buf}/{k}")
        assert a.num_steps == b.num_steps == 3
    finally:
        if comm is not None:
            torch.cuda.synchronize()
            N.nccl_comm_destroy(comm)


def test_adjacent_frames_layout_bitwise():
    """The GPU dataset hands o_t directly after o_tm1 in one allocation; the step on that
    layout is bit-identical to the step on separate buffers."""
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    B = 24
    p0, t0 = net.init(3), net.init(4)
    a = _learner(net, B)
    b = _learner(net, B)
    a.set_params(p0, t0)
    b.set_params(p0, t0)
    rng = np.random.default_rng(5)
    for _ in range(2):
        dev = _dev(_batch(rng, B, (84, 84, 4), 18))
        pair = torch.empty(2, B, 84 * 84 * 4, dtype=torch.uint8, device="cuda")
        pair[0].copy_(dev[0].reshape(B, -1))
        pair[1].copy_(dev[4].reshape(B, -1))
        a.step(pair[0], *dev[1:4], pair[1], dev[5])
        b.step(dev[0].reshape(B, -1).clone(), *dev[1:4], dev[4].reshape(B, -1).clone(), dev[5])
        torch.cuda.synchronize()
        assert a.loss.item() == b.loss.item()
        for buf in ("params", "m", "v"):
            ga, gb = a.get_params(buf), b.get_params(buf)
            for k in ga:
                np.testing.assert_array_equal(ga[k], gb[k], err_msg=f"{buf}/{k}")


@pytest.mark.parametrize("kind", ["nature", "mlp"])
def test_split_forward_stages_bitwise(kind):
    """Stage 0 issued as stage 2 (forwards) + stage 3 (loss, dense backward; the only reader
    of global_min_probability), as the data-parallel learner does to overlap the IS
    normaliser's all-reduce with the forwards, gives the same gradients, loss, TD errors and
    priorities as stage 0; stage 3 without its stage 2 is rejected."""
    from acme_amd.networks import DQNAtariNetwork, MLP
    net = DQNAtariNetwork(18) if kind == "nature" else MLP(6, [32, 32], 4)
    obs = (84, 84, 4) if kind == "nature" else (6,)
    B = 37
    p0, t0 = net.init(5), net.init(6)
    rng = np.random.default_rng(9)
    dev = _dev(_batch(rng, B, obs, net.num_actions, u8=kind == "nature"))
    if kind == "mlp":
        dev = [x.reshape(B, -1).contiguous() if x.dim() > 1 else x for x in dev]
    gmin = torch.tensor([float(dev[5].min()) * 0.5], dtype=torch.float64, device="cuda")
    res = []
    for split in (False, True):
        n = _learner(net, B)
        n.set_params(p0, t0)
        if split:
            n.forward_backward_stage(2, *dev)
            n.forward_backward_stage(3, *dev, global_min_probability=gmin)
        else:
            n.forward_backward_stage(0, *dev, global_min_probability=gmin)
        n.forward_backward_stage(1, *dev)
        torch.cuda.synchronize()
        res.append((n.get_params("grads"), n.loss.item(), n.td_error.cpu().numpy(),
                    n.priorities.cpu().numpy()))
    (g0, l0, td0, p_0), (g1, l1, td1, p_1) = res
    for k in g0:
        np.testing.assert_array_equal(g0[k], g1[k], err_msg=k)
    assert l0 == l1
    np.testing.assert_array_equal(td0, td1)
    np.testing.assert_array_equal(p_0, p_1)
    n = _learner(net, B)
    n.set_params(p0, t0)
    with pytest.raises(Exception):
        n.forward_backward_stage(3, *dev, global_min_probability=gmin)


@pytest.mark.parametrize("kind", ["nature", "mlp"])
def test_step_with_priority_update_equals_step_then_update(kind):
    """acme_dqn_step_update (the write-back issued inside the step, on the second stream on
    the plane path; after the step otherwise) equals acme_dqn_step followed by
    acme_replay_update_priorities: same parameters, same raw priorities, same next draws."""
    from acme_amd.native import NativeReplay
    from acme_amd.networks import MLP, DQNAtariNetwork
    net = DQNAtariNetwork(18) if kind == "nature" else MLP(8, [32, 32], 4)
    B = 32
    obs_shape = (84, 84, 4) if kind == "nature" else (8,)
    p0, t0 = net.init(3), net.init(4)
    a = _learner(net, B, target_update_period=2)
    b = _learner(net, B, target_update_period=2)
    a.set_params(p0, t0)
    b.set_params(p0, t0)
    tables = [NativeReplay(1000, [4], prioritized=True, priority_exponent=0.6, seed=77)
              for _ in range(2)]
    rows = np.arange(600, dtype=np.uint32).view(np.uint8).reshape(600, 4)
    for t in tables:
        t.insert([rows], np.linspace(0.5, 2.0, 600))
    torch.cuda.synchronize()
    rng = np.random.default_rng(21)
    for step in range(3):
        keys = tables[0].sample(B, step)["keys"]
        assert torch.equal(keys, tables[1].sample(B, step)["keys"])
        dev = _dev(_batch(rng, B, obs_shape, net.num_actions, u8=kind == "nature"))
        a.step(*dev, priority_update=(tables[0].handle, keys))
        b.step(*dev)
        tables[1].update_priorities(keys, b.priorities[:B])
        torch.cuda.synchronize()
        assert a.loss.item() == b.loss.item()
        sa, sb = tables[0].export_state(), tables[1].export_state()
        np.testing.assert_array_equal(sa["raw_priorities"], sb["raw_priorities"])
        for buf in ("params", "target"):
            ga, gb = a.get_params(buf), b.get_params(buf)
            for k in ga:
                np.testing.assert_array_equal(ga[k], gb[k], err_msg=f"{buf}/{k}")
    da, db = tables[0].sample(B, 99), tables[1].sample(B, 99)
    for k in da:
        assert torch.equal(da[k], db[k]), k


def test_early_target_forward_bitwise():
    """With the batch's inputs event (acme_transition_batch.inputs_event) the target forward
    starts on the second stream from that event alone and may overlap the previous step's
    Adam; results equal the ordered schedule's bit for bit, across target copies (which
    fall back to the ordered fork) and a q_values call between steps."""
    from acme_amd._lib import OrderEvent
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(18)
    B = 64
    p0, t0 = net.init(7), net.init(8)
    a = _learner(net, B, target_update_period=3)
    b = _learner(net, B, target_update_period=3)
    a.set_params(p0, t0)
    b.set_params(p0, t0)
    rng = np.random.default_rng(17)
    for step in range(7):
        dev = _dev(_batch(rng, B, (84, 84, 4), 18))
        fb = torch.cat([dev[0], dev[4]]).reshape(2 * B, -1).to(torch.float16).view(torch.int16)
        ev = OrderEvent()
        ev.record()
        a.step(*dev, obs_f16=fb, inputs_event=ev)
        b.step(*dev, obs_f16=fb)
        if step == 4:
            qa = a.q_values(dev[4].reshape(B, -1), use_target=True)
            qb = b.q_values(dev[4].reshape(B, -1), use_target=True)
            assert torch.equal(qa, qb)
        torch.cuda.synchronize()
        assert a.loss.item() == b.loss.item(), step
        assert torch.equal(a.priorities, b.priorities), step
        for buf in ("params", "target", "m", "v"):
            ga, gb = a.get_params(buf), b.get_params(buf)
            for k in ga:
                np.testing.assert_array_equal(ga[k], gb[k], err_msg=f"{step} {buf}/{k}")
