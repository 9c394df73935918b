"""GPU replay table vs the C oracle: bit-exact slots/keys/probabilities under a fixed seed.

Replaces Reverb Prioritized(alpha)/Uniform + Fifo (acme/agents/tf/dqn/agent.py:95-101,
acme/agents/tf/d4pg/agent.py:96-102) and TFClient.update_priorities
(acme/agents/tf/dqn/learning.py:151-154).  Reverb's own sampler is unseeded, so index
parity is against oracle/replay_oracle.c.
"""

import numpy as np
import pytest
import torch

from tests._oracle import OracleTable

pytestmark = pytest.mark.gpu


def _native(capacity, fields, prioritized, alpha=0.6, seed=1234):
    from acme_amd.native import NativeReplay
    return NativeReplay(capacity, fields, prioritized=prioritized, priority_exponent=alpha,
                        seed=seed)


def _cmp_sample(r, o, batch, step):
    g = {k: v.cpu().numpy() for k, v in r.sample(batch, step).items()}
    ref = o.sample(batch, step)
    np.testing.assert_array_equal(g["slots"], ref["slots"])
    np.testing.assert_array_equal(g["keys"].view(np.uint64), ref["keys"])
    np.testing.assert_array_equal(g["probabilities"], ref["probabilities"])  # bitwise
    np.testing.assert_array_equal(g["table_size"], ref["table_size"])
    np.testing.assert_array_equal(g["priorities"], ref["priorities"])
    return g


@pytest.mark.parametrize("capacity,n_insert", [(1, 3), (64, 10), (65, 200), (5000, 7000),
                                               (4096 * 64 + 7, 300000)])
def test_prioritized_sample_bit_exact(capacity, n_insert):
    rng = np.random.default_rng(capacity)
    r = _native(capacity, [4], True)
    o = OracleTable(capacity, True, 0.6, 1234)
    pr = rng.uniform(0.0, 5.0, n_insert)
    pr[rng.random(n_insert) < 0.05] = 0.0  # zero priorities are never drawn
    pr[-1] = 1.0
    r.insert([np.arange(n_insert, dtype=np.int32)], pr)
    o.insert(pr)
    for step in (0, 1, 12345):
        g = _cmp_sample(r, o, 512, step)
        assert (g["priorities"] > 0).all()
    st = r.debug_state()
    np.testing.assert_array_equal(st["leaves"], o.leaves()[:capacity])


def test_uniform_sample_bit_exact():
    r = _native(1000, [8], False)
    o = OracleTable(1000, False, 0.0, 1234)
    pr = np.ones(1500)
    r.insert([np.zeros((1500, 8), np.uint8)], pr)
    o.insert(pr)
    g = _cmp_sample(r, o, 256, 3)
    assert (g["probabilities"] == 1.0 / 1000).all()


def test_priority_updates_last_wins_and_stale_keys():
    rng = np.random.default_rng(7)
    cap = 3000
    r = _native(cap, [4], True)
    o = OracleTable(cap, True, 0.6, 1234)
    pr = rng.uniform(0.1, 2.0, 4000)
    r.insert([np.zeros((4000, 1), np.int32)], pr)
    o.insert(pr)
    for it in range(5):
        s = r.sample(512, it)
        keys = s["keys"].cpu().numpy().view(np.uint64).copy()
        # duplicates (sampling with replacement) + a stale key evicted by the FIFO.
        keys[:8] = keys[8]
        keys[9] = 5  # key 5 was evicted (capacity 3000, 4000 inserted)
        newp = rng.uniform(0.0, 3.0, 512)
        r.update_priorities(torch.as_tensor(keys.view(np.int64)).cuda().view(torch.uint64),
                            torch.as_tensor(newp).cuda())
        o.update(keys, newp)
        st = r.debug_state()
        np.testing.assert_array_equal(st["leaves"], o.leaves()[:cap])
        _cmp_sample(r, o, 512, 100 + it)


def test_gather_rows():
    rng = np.random.default_rng(3)
    cap, n = 300, 500
    obs = rng.integers(0, 256, (n, 84 * 84 * 4), dtype=np.uint8)
    act = rng.integers(0, 18, n).astype(np.int32)
    rew = rng.standard_normal(n).astype(np.float32)
    r = _native(cap, [84 * 84 * 4, 4, 4], True)
    keys = r.insert([obs, act, rew], np.ones(n))
    s = r.sample(64, 0)
    outs = [torch.empty(64, 84 * 84 * 4, dtype=torch.uint8, device="cuda"),
            torch.empty(64, dtype=torch.int32, device="cuda"),
            torch.empty(64, dtype=torch.float32, device="cuda")]
    r.gather(s["slots"], outs)
    k = s["keys"].cpu().numpy().view(np.int64)
    np.testing.assert_array_equal(outs[0].cpu().numpy(), obs[k])
    np.testing.assert_array_equal(outs[1].cpu().numpy(), act[k])
    np.testing.assert_array_equal(outs[2].cpu().numpy(), rew[k])
    assert (k >= n - cap).all()  # only live items are drawn
    assert keys[-1] == n - 1


def test_sampling_distribution_matches_priorities():
    """Empirical frequencies follow p^alpha / sum p^alpha (chi-square, 1M draws)."""
    cap = 100
    pr = np.linspace(0.0, 4.0, cap)
    r = _native(cap, [4], True, alpha=0.6, seed=99)
    r.insert([np.zeros((cap, 1), np.int32)], pr)
    counts = np.zeros(cap)
    for step in range(256):
        s = r.sample(4096, step)["slots"].cpu().numpy()
        counts += np.bincount(s, minlength=cap)
    w = pr ** 0.6
    expect = w / w.sum() * counts.sum()
    nz = expect > 0
    assert counts[~nz].sum() == 0
    chi2 = (((counts - expect) ** 2)[nz] / expect[nz]).sum()
    assert chi2 < 160, chi2  # 98 dof: p ~ 1e-4 threshold


def test_empty_table_raises():
    r = _native(10, [4], True)
    with pytest.raises(RuntimeError):
        r.sample(4, 0)


def test_synthetic_fill_atari_layout():
    r = _native(2048, [84 * 84 * 4, 4, 4, 4, 84 * 84 * 4], True)
    r.fill_synthetic(3000, 0, num_actions=18, seed=5)
    assert r.size() == 2048
    s = r.sample(256, 0)
    outs = [torch.empty(256, 28224, dtype=torch.uint8, device="cuda"),
            torch.empty(256, dtype=torch.int32, device="cuda"),
            torch.empty(256, dtype=torch.float32, device="cuda"),
            torch.empty(256, dtype=torch.float32, device="cuda"),
            torch.empty(256, 28224, dtype=torch.uint8, device="cuda")]
    r.gather(s["slots"], outs)
    a = outs[1].cpu().numpy()
    assert a.min() >= 0 and a.max() < 18
    d = outs[3].cpu().numpy()
    f = np.float32(0.99)
    assert set(np.unique(d)).issubset({0.0, ((f * f) * f) * f})
    assert (s["probabilities"].cpu().numpy() == 1.0 / 2048).all()


@pytest.mark.parametrize("n_upd", [512, 4096, 5000])
def test_priority_updates_deep_tree(n_upd):
    """Four-level tree (the 1M-slot shape): the one-launch update (n <= 4096) and the
    multi-launch path (n > 4096) both match the oracle bit for bit."""
    rng = np.random.default_rng(n_upd)
    cap = 300_000
    r = _native(cap, [4], True)
    o = OracleTable(cap, True, 0.6, 1234)
    pr = rng.uniform(0.1, 2.0, cap + 1000)
    r.insert([np.zeros((cap + 1000, 1), np.int32)], pr)
    o.insert(pr)
    for it in range(3):
        keys = rng.integers(1000, cap + 1000, n_upd).astype(np.uint64)
        keys[:16] = keys[16]          # duplicates: the last one wins
        keys[17] = 3                  # evicted key: ignored
        newp = rng.uniform(0.0, 3.0, n_upd)
        r.update_priorities(torch.as_tensor(keys.view(np.int64)).cuda().view(torch.uint64),
                            torch.as_tensor(newp).cuda())
        o.update(keys, newp)
        np.testing.assert_array_equal(r.debug_state()["leaves"], o.leaves()[:cap])
        _cmp_sample(r, o, 512, 200 + it)


def test_priority_updates_many_per_workgroup():
    """ADVICE r5 (the LDS race of the one-launch update): 4096 updates on a 1M-slot table give
    each of the 256 update workgroups ~16 updates under distinct level-1 nodes, so the rows of
    children a workgroup prefetches are filled by other waves than the threads substituting
    the new leaves.  Every iteration: the leaves, the sampling mass (recomputed from the
    stored level sums: a level-1 node missing its update changes it) and 512 draws bit-exact
    against the oracle."""
    import ctypes
    from acme_amd._lib import lib
    rng = np.random.default_rng(77)
    cap = 1_000_000
    r = _native(cap, [4], True)
    o = OracleTable(cap, True, 0.6, 1234)
    pr = rng.uniform(0.1, 2.0, cap)
    r.insert([np.zeros((cap, 1), np.int32)], pr)
    o.insert(pr)
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    for it in range(6):
        keys = rng.choice(cap, 4096, replace=False).astype(np.uint64)
        newp = rng.uniform(0.0, 3.0, 4096)
        r.update_priorities(torch.as_tensor(keys.view(np.int64)).cuda().view(torch.uint64),
                            torch.as_tensor(newp).cuda())
        o.update(keys, newp)
        assert lib().acme_replay_total(r._h, ctypes.c_void_p(out.data_ptr()), None) == 0
        torch.cuda.synchronize()
        assert out.item() == o.total(), (it, out.item(), o.total())
        np.testing.assert_array_equal(r.debug_state()["leaves"], o.leaves()[:cap])
        _cmp_sample(r, o, 512, 400 + it)


@pytest.mark.parametrize("capacity", [1024, 1088, 65536, 69632])
def test_top_level_computed_and_stored(capacity):
    """The top level's entries with children are computed by the readers when there are at
    most 16 of them (replay.hip kTopComputed; the one-launch update then leaves the stored
    top alone) and read when there are more: 1024 / 65536 slots have 16, 1088 / 69632 have
    17.  Both paths: draws, probabilities and the sampling mass bit-exact against the
    oracle after one-launch priority updates (a total that read a stale top would differ)."""
    import ctypes
    from acme_amd._lib import lib
    rng = np.random.default_rng(capacity)
    r = _native(capacity, [4], True)
    o = OracleTable(capacity, True, 0.6, 1234)
    pr = rng.uniform(0.1, 2.0, capacity)
    r.insert([np.zeros((capacity, 1), np.int32)], pr)
    o.insert(pr)
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    for it in range(3):
        keys = rng.integers(0, capacity, 512).astype(np.uint64)
        newp = rng.uniform(0.0, 3.0, 512)
        r.update_priorities(torch.as_tensor(keys.view(np.int64)).cuda().view(torch.uint64),
                            torch.as_tensor(newp).cuda())
        o.update(keys, newp)
        _cmp_sample(r, o, 512, 300 + it)
        assert lib().acme_replay_total(r._h, ctypes.c_void_p(out.data_ptr()), None) == 0
        torch.cuda.synchronize()
        assert out.item() == o.total(), (it, out.item(), o.total())


@pytest.mark.parametrize("prefetch", [0, 1, 4])
def test_prefetched_dataset_draw_order(prefetch):
    """make_reverb_dataset(prefetch_size=P): batch k is drawn (Philox counter k) after the
    priority updates of steps < k - P and before the later ones, as Reverb's prefetched
    samples; replayed exactly by the oracle in that order."""
    from acme_amd import replay, specs
    from acme_amd.adders import reverb as adders
    from acme_amd.datasets import make_reverb_dataset
    cap, B = 5000, 64
    env_spec = specs.EnvironmentSpec(
        observations=specs.Array((24,), np.float32),
        actions=specs.BoundedArray((6,), np.float32, -1.0, 1.0),
        rewards=specs.Array((), np.float32), discounts=specs.BoundedArray((), np.float32, 0, 1))
    table = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Prioritized(0.6),
                         replay.selectors.Fifo(), cap, replay.rate_limiters.MinSize(1),
                         signature=adders.NStepTransitionAdder.signature(env_spec), seed=1234,
                         device=torch.device("cuda"))
    table.native.fill_synthetic(cap, layout=1, num_actions=1, seed=0)
    server = replay.Server([table])
    client = replay.Client(server)
    it = iter(make_reverb_dataset(server, batch_size=B, prefetch_size=prefetch))
    o = OracleTable(cap, True, 0.6, 1234)
    o.insert(np.ones(cap))
    rng = np.random.default_rng(prefetch)
    issued, expect = 0, {}
    for k in range(8):
        s = next(it)
        while issued <= k + prefetch:
            expect[issued] = o.sample(B, issued)
            issued += 1
        keys = s.info.key.cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(keys, expect[k]["keys"])
        np.testing.assert_array_equal(s.info.probability.cpu().numpy(),
                                      expect[k]["probabilities"])
        newp = rng.uniform(0.0, 3.0, B)
        client.update_priorities(adders.DEFAULT_PRIORITY_TABLE, s.info.key,
                                 torch.as_tensor(newp).cuda())
        o.update(keys, newp)


@pytest.mark.parametrize("fields", [[28224, 4, 4, 4, 28224], [28224, 4, 4], [2048, 1040, 8],
                                    [96, 24, 4, 4, 96], [1024, 4, 1024], [3072, 12, 3072]])
def test_gather_kernels_bit_identical(fields):
    """The gather kernels (acme_tune_set GATH: 0 = transition pair / pieces default, 1 =
    row-per-workgroup, 2 = wave pieces) copy exactly the sampled rows."""
    from acme_amd._lib import lib
    rng = np.random.default_rng(len(fields) * 31 + fields[0])
    cap, n, B = 700, 900, 333
    data = [rng.integers(0, 256, (n, b), dtype=np.uint8) for b in fields]
    pr = rng.uniform(0.1, 2.0, n)
    outs = {}
    for gv in (0, 1, 2):
        lib().acme_tune_set(b"GATH", gv)  # read once, at the table's creation
        try:
            r = _native(cap, fields, True)
        finally:
            lib().acme_tune_set(b"GATH", 0)
        r.insert(data, pr)
        s = r.sample(B, 4)
        keys = s["keys"].cpu().numpy().view(np.int64)
        o = [torch.full((B, b), 7, dtype=torch.uint8, device="cuda") for b in fields]
        r.gather(s["slots"], o)
        outs[gv] = [x.cpu().numpy() for x in o]
    for f, b in enumerate(fields):
        np.testing.assert_array_equal(outs[0][f], data[f][keys])
        np.testing.assert_array_equal(outs[1][f], outs[0][f])
        np.testing.assert_array_equal(outs[2][f], outs[0][f])


def _pipe_buffers(r, B, fields):
    import ctypes
    info = r.alloc_sample_info(B)
    outs = [torch.zeros(B, b, dtype=torch.uint8, device="cuda") for b in fields]
    ptrs = (ctypes.c_void_p * len(outs))(*[x.data_ptr() for x in outs])
    raw = [info[k].data_ptr() for k in ("slots", "keys", "probabilities", "table_size",
                                          "priorities")]
    return info, outs, ptrs, raw


@pytest.mark.parametrize("prioritized", [True, False])
@pytest.mark.parametrize("fields", [[28224, 4, 4, 4, 28224], [2048, 4, 2048], [96, 24, 4, 4, 96]])
def test_pipelined_sample_gather(prioritized, fields):
    """acme_replay_sample_gather_pipe (round 6): batch k's rows are copied by call k + 1's
    launch (or a flush); every batch equals the oracle's draw of its step counter and the
    rows of its keys.  Three buffer sets in rotation, a batch-size change mid-stream, and
    an insert between a draw and its copy (the commit issues the pending copy first, so the
    batch still gets the rows of its drawn keys, not the new items')."""
    import ctypes
    from acme_amd._lib import lib
    L = lib()
    rng = np.random.default_rng(9)
    cap, n = 3000, 3000
    data = [rng.integers(0, 256, (n, b), dtype=np.uint8) for b in fields]
    pr = rng.uniform(0.0, 2.0, n)
    o = OracleTable(cap, prioritized, 0.6, 1234)
    o.insert(pr)
    r = _native(cap, fields, prioritized)
    r.insert(data, pr)
    pid = ctypes.c_int32()
    assert L.acme_replay_pipe_open(r.handle, ctypes.byref(pid)) == 0
    st = torch.cuda.Stream()
    sets = [_pipe_buffers(r, 300, fields) for _ in range(3)]
    plan = [(0, 257, 11), (1, 257, 12), (2, 300, 13), (0, 64, 14), (1, 257, 15)]

    def check(k):
        s, B, step = plan[k]
        info, outs = sets[s][0], sets[s][1]
        ref = o.sample(B, step)
        for key in ("slots", "probabilities", "table_size", "priorities"):
            np.testing.assert_array_equal(info[key][:B].cpu().numpy(), ref[key])
        keys = info["keys"][:B].cpu().numpy().view(np.int64)
        for f in range(len(fields)):
            np.testing.assert_array_equal(outs[f][:B].cpu().numpy(), data[f][keys % cap])

    with torch.cuda.stream(st):
        for k, (s, B, step) in enumerate(plan):
            _, _, ptrs, raw = sets[s]
            assert L.acme_replay_sample_gather_pipe(r.handle, pid.value, B, step, *raw, ptrs,
                                                    ctypes.c_void_p(st.cuda_stream)) == 0
            if k > 0:
                st.synchronize()
                check(k - 1)
        # An insert while the last batch's copy is pending: overwrite every slot.
        new = [rng.integers(0, 256, (cap, b), dtype=np.uint8) for b in fields]
        r.insert(new, rng.uniform(0.1, 1.0, cap))
        torch.cuda.synchronize()
        check(len(plan) - 1)
        assert L.acme_replay_pipe_flush(r.handle, pid.value) == 0  # nothing pending: no-op
    assert L.acme_replay_pipe_close(r.handle, pid.value) == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("prioritized", [True, False])
@pytest.mark.parametrize("fields", [[28224, 4, 4, 4, 28224], [2048, 4, 2048],
                                    [96, 24, 4, 4, 96], [1020, 8]])
def test_fused_sample_gather_matches_two_launches(prioritized, fields):
    """acme_replay_sample_gather's fused kernels (the transition layout: draw + row copy in
    one workgroup; rows of small fields: draw + copy per wave, e.g. D4PG's control
    transitions) against the sampling kernel + gather (SGF=1) and the oracle's draw."""
    import ctypes
    from acme_amd._lib import lib
    rng = np.random.default_rng(5)
    cap, n, B = 3000, 3500, 257
    data = [rng.integers(0, 256, (n, b), dtype=np.uint8) for b in fields]
    pr = rng.uniform(0.0, 2.0, n)
    o = OracleTable(cap, prioritized, 0.6, 1234)
    o.insert(pr)
    L = lib()
    res = {}
    for sgf in (0, 1):
        L.acme_tune_set(b"SGF", sgf)  # read once, at the table's creation
        try:
            r = _native(cap, fields, prioritized)
        finally:
            L.acme_tune_set(b"SGF", 0)
        r.insert(data, pr)
        info = r.alloc_sample_info(B)
        outs = [torch.zeros(B, b, dtype=torch.uint8, device="cuda") for b in fields]
        ptrs = (ctypes.c_void_p * len(outs))(*[x.data_ptr() for x in outs])
        raw = [info[k].data_ptr() for k in ("slots", "keys", "probabilities", "table_size",
                                              "priorities")]
        assert L.acme_replay_sample_gather(r.handle, B, 77, *raw, ptrs, None) == 0
        torch.cuda.synchronize()
        res[sgf] = ({k: v.cpu().numpy() for k, v in info.items()},
                    [x.cpu().numpy() for x in outs])
    ref = o.sample(B, 77)
    for k in ("slots", "probabilities", "table_size", "priorities"):
        np.testing.assert_array_equal(res[0][0][k], ref[k])
        np.testing.assert_array_equal(res[1][0][k], ref[k])
    keys = res[0][0]["keys"].view(np.int64)
    for f in range(len(fields)):
        np.testing.assert_array_equal(res[0][1][f], data[f][keys])
        np.testing.assert_array_equal(res[1][1][f], res[0][1][f])
