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
