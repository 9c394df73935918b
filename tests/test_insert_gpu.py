"""Actor-side insert path: pinned staging ring + side-stream hipMemcpyAsync (north star;
SURVEY §8(f) row 1).  Replaces Writer.append + create_item, one item per environment step
(acme/adders/reverb/transition.py:119-165; acme/agents/agent.py:78-89).

Checked: inserts through the staging chunks (zero-copy stage/commit, packed host insert,
over-capacity inserts, device rows) leave the table bit-identical to the C oracle; and with
an actor thread inserting while the learner thread samples through a prefetching dataset
and writes priorities back (no host synchronisation anywhere), every gathered row is the
row of the key the sampler reported for it (an insert never lands under a queued gather, and
a sample never sees a slot before its copy).
"""

import threading

import numpy as np
import pytest
import torch

from tests._oracle import OracleTable

pytestmark = pytest.mark.gpu


def _native(capacity, fields, prioritized=True, alpha=0.6, seed=1234):
    from acme_amd.native import NativeReplay
    return NativeReplay(capacity, fields, prioritized=prioritized, priority_exponent=alpha,
                        seed=seed)


def _cmp(r, o, batch, step):
    g = {k: v.cpu().numpy() for k, v in r.sample(batch, step).items()}
    ref = o.sample(batch, step)
    np.testing.assert_array_equal(g["slots"], ref["slots"])
    np.testing.assert_array_equal(g["keys"].view(np.uint64), ref["keys"])
    np.testing.assert_array_equal(g["probabilities"], ref["probabilities"])
    np.testing.assert_array_equal(g["priorities"], ref["priorities"])
    return g


def test_stage_commit_bit_exact_and_rows():
    rng = np.random.default_rng(0)
    cap = 5000
    r = _native(cap, [64, 4])
    o = OracleTable(cap, True, 0.6, 1234)
    chunk = r.stage_capacity()
    assert chunk >= 1
    total, rows = 0, {}
    for n in (1, 7, 300, 2999, 4000):  # ring wrap-around inside one chunk and across chunks
        pr = rng.uniform(0.0, 3.0, n)
        done = 0
        while done < n:
            m = min(chunk, n - done)
            bufs = r.stage(m)
            payload = rng.integers(0, 256, (m, 64), dtype=np.uint8)
            bufs[0][:] = payload
            bufs[1][:] = np.arange(total + done, total + done + m, dtype=np.int32).view(
                np.uint8).reshape(m, 4)
            keys = r.commit(m, pr[done:done + m])
            np.testing.assert_array_equal(keys, np.arange(total + done, total + done + m))
            for k, p in zip(keys, payload):
                rows[int(k)] = p
            done += m
        o.insert(pr)
        total += n
        _cmp(r, o, 512, total)
    np.testing.assert_array_equal(r.debug_state()["leaves"], o.leaves()[:cap])
    s = r.sample(256, 99)
    outs = [torch.empty(256, 64, dtype=torch.uint8, device="cuda"),
            torch.empty(256, dtype=torch.int32, device="cuda")]
    r.gather(s["slots"], outs)
    keys = s["keys"].cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(outs[1].cpu().numpy(), keys.astype(np.int32))
    np.testing.assert_array_equal(outs[0].cpu().numpy(), np.stack([rows[int(k)] for k in keys]))


def test_commit_fewer_than_staged_and_errors():
    r = _native(100, [8])
    bufs = r.stage(10)
    bufs[0][:] = 7
    with pytest.raises(ValueError):
        r.stage(1)  # previous chunk not committed
    keys = r.commit(4, np.ones(4))
    np.testing.assert_array_equal(keys, np.arange(4))
    assert r.size() == 4
    with pytest.raises(ValueError):
        r.commit(1)  # nothing staged
    with pytest.raises(ValueError):
        r.stage(r.stage_capacity() + 1)
    r.stage(2)
    with pytest.raises(ValueError):
        r.commit(1, np.array([-1.0]))  # negative priority
    r.stage(2)  # the failed commit released its chunk
    r.commit(0)


@pytest.mark.parametrize("n", [1, 1000, 25_000])
def test_packed_host_insert_over_capacity(n):
    """acme_replay_insert with host rows: packed into pinned chunks (several per call when n
    exceeds a chunk), only the last `capacity` items land, keys still count every item."""
    rng = np.random.default_rng(n)
    cap = 7000
    r = _native(cap, [2048, 4])
    o = OracleTable(cap, True, 0.6, 1234)
    assert r.stage_capacity() < 25_000
    all_obs = []
    for rep in range(2):
        pr = rng.uniform(0.0, 2.0, n)
        obs = rng.integers(0, 256, (n, 2048), dtype=np.uint8)
        all_obs.append(obs)
        keys = r.insert([obs, np.arange(rep * n, rep * n + n, dtype=np.int32)], pr)
        first = rep * n
        np.testing.assert_array_equal(keys, np.arange(first, first + n))
        o.insert(pr)
        _cmp(r, o, 256, rep)
    s = r.sample(128, 5)
    outs = [torch.empty(128, 2048, dtype=torch.uint8, device="cuda"),
            torch.empty(128, dtype=torch.int32, device="cuda")]
    r.gather(s["slots"], outs)
    k = s["keys"].cpu().numpy().view(np.int64)
    assert (k >= 2 * n - cap).all()  # only the last `capacity` items live
    np.testing.assert_array_equal(outs[1].cpu().numpy(), k)
    np.testing.assert_array_equal(outs[0].cpu().numpy(), np.concatenate(all_obs)[k])


def test_device_rows_insert_matches_host_insert():
    rng = np.random.default_rng(4)
    cap, n = 3000, 4500
    pr = rng.uniform(0.0, 2.0, n)
    obs = rng.integers(0, 256, (n, 256), dtype=np.uint8)
    a, b = _native(cap, [256]), _native(cap, [256])
    a.insert([obs], pr)
    b.insert([torch.as_tensor(obs).cuda()], pr)
    for step in range(3):
        ga = {k: v.cpu().numpy() for k, v in a.sample(512, step).items()}
        gb = {k: v.cpu().numpy() for k, v in b.sample(512, step).items()}
        for k in ga:
            np.testing.assert_array_equal(ga[k], gb[k])
    sa, sb = a.debug_state(), b.debug_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k])


@pytest.mark.parametrize("width", [16, 256])
def test_concurrent_actor_inserts_with_prefetching_learner(width):
    """An actor thread writes items (payload = its key) through Table.insert / flush while
    the learner thread draws prefetched batches and writes priorities back, with no host
    synchronisation: every gathered row carries the key the sampler reported for it.
    width 256 (1 KiB rows: the transition layout) runs the pipelined draws, whose pending
    row copies each commit issues before it lands (acme_replay_sample_gather_pipe)."""
    from acme_amd import replay, specs
    from acme_amd.adders import reverb as adders
    from acme_amd.datasets import make_reverb_dataset
    cap, B = 4096, 256
    sig = (specs.Array((width,), np.int32), specs.Array((), np.int32),
           specs.Array((), np.float32), specs.Array((), np.float32),
           specs.Array((width,), np.int32))
    table = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Prioritized(0.6),
                         replay.selectors.Fifo(), cap, replay.rate_limiters.MinSize(1),
                         signature=sig, seed=5, device=torch.device("cuda"), flush_every=64)
    next_key = [0]

    def item(k):
        row = np.full(width, k, np.int32)
        return (row, np.int32(k % 18), np.float32(k), np.float32(0.5), row + 1)

    def insert_some(n, rng):
        for _ in range(n):
            table.insert(item(next_key[0]), float(rng.uniform(0.1, 2.0)))
            next_key[0] += 1

    rng0 = np.random.default_rng(0)
    insert_some(cap, rng0)
    table.flush()
    server = replay.Server([table])
    client = replay.Client(server)
    it = iter(make_reverb_dataset(server, batch_size=B, prefetch_size=4))
    stop = threading.Event()
    errors = []

    def actor():
        rng = np.random.default_rng(1)
        try:
            while not stop.is_set() and next_key[0] < 60 * cap:
                insert_some(32, rng)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = threading.Thread(target=actor)
    th.start()
    seen = []
    try:
        for step in range(120):
            s = next(it)
            client.update_priorities(adders.DEFAULT_PRIORITY_TABLE, s.info.key,
                                     torch.rand(B, dtype=torch.float64, device="cuda") + 0.1)
            # Device-side check, no host sync in the loop: row payload == reported key.
            k = s.info.key.view(torch.int64)
            o_tm1, a, r_t, d_t, o_t = s.data
            ok = ((o_tm1 == k[:, None].to(torch.int32)).all(1) &
                  (o_t == (k[:, None] + 1).to(torch.int32)).all(1) &
                  (r_t == k.to(torch.float32)))
            seen.append((ok.all(), k.max()))
    finally:
        stop.set()
        th.join()
    assert not errors, errors
    torch.cuda.synchronize()
    assert all(bool(ok) for ok, _ in seen)
    inserted = next_key[0]
    assert inserted > 2 * cap, "the actor thread did not overlap the learner"
    # Later batches see newer items (inserts become visible without a host sync).
    assert int(seen[-1][1]) > cap
