"""The HIP path reproduces the committed §8(c) fixtures (tests/golden/make_parity_goldens.py)
through the C ABI.  Bars as tests/test_dqn_gpu.py: loss / TD / priorities / q rtol 1e-5;
parameters after Adam within lr of the f64 trajectory and 98% within 1e-5 relative (Adam's
first step is sign descent, so elements whose gradient is at the fp32 noise floor may move
by up to lr either way); sampler bit-exact."""

import os

import numpy as np
import pytest
import torch

from tests.golden import make_parity_goldens as G

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KEYS = ("o_tm1", "a_tm1", "r_t", "d_t", "o_t", "probabilities")


def _load(name):
    return dict(np.load(os.path.join(HERE, name), allow_pickle=False))


def _dev(b):
    return [torch.as_tensor(np.ascontiguousarray(b[k])).cuda() for k in KEYS]


class _GPUTable:
    """NativeReplay behind the OracleTable interface of the fixture script."""

    def __init__(self, capacity, alpha, seed):
        from acme_amd.native import NativeReplay
        self.r = NativeReplay(capacity, [4], prioritized=True, priority_exponent=alpha,
                              seed=seed)

    def insert(self, priorities):
        n = len(priorities)
        self.r.insert([np.arange(n, dtype=np.int32)], np.asarray(priorities, np.float64))

    def update(self, keys, priorities):
        k = torch.as_tensor(np.asarray(keys, np.uint64).view(np.int64)).view(torch.uint64)
        self.r.update_priorities(k.cuda(), torch.as_tensor(priorities).cuda())

    def sample(self, batch, step):
        out = self.r.sample(batch, step)
        torch.cuda.synchronize()
        res = {k: v.cpu().numpy() for k, v in out.items() if k != "keys"}
        res["keys"] = out["keys"].view(torch.int64).cpu().numpy().view(np.uint64)
        return res


def test_sampler_fixture_bit_exact():
    z = _load("sampler_1k.npz")
    c = G.SAMPLER
    draws = G.run_sampler(lambda: _GPUTable(c["capacity"], c["alpha"], c["seed"]))
    for i, d in enumerate(draws):
        for k in ("slots", "keys", "probabilities", "table_size", "priorities"):
            np.testing.assert_array_equal(d[k], z[f"out/{i}/{k}"], err_msg=f"draw {i} {k}")


def _check_params(got, ref, lr, name):
    err = np.abs(got.astype(np.float64) - ref)
    assert err.max() <= lr + 1e-6, (name, float(err.max()))
    frac = np.mean(err <= 1e-5 * np.abs(ref) + 1e-7)
    assert frac >= 0.98, (name, frac)


def test_cartpole_fixture():
    from acme_amd.native import NativeDQN
    z = _load("dqn_cartpole_b32.npz")
    net = G.cartpole_net()
    names = [n for n, _ in net.tensor_shapes()]
    d = NativeDQN(network="mlp", num_actions=2, max_batch=32, obs_dtype="float32", obs_dim=4,
                  hidden=(50, 50), target_update_period=2)
    d.set_params({k: z[f"in/params/{k}"] for k in names},
                 {k: z[f"in/target/{k}"] for k in names})
    q = torch.empty(32, 2, device="cuda")
    for i in range(3):
        b = {k: z[f"in/{i}/{k}"] for k in KEYS}
        d.step(*_dev(b), q_tm1=q)
        torch.cuda.synchronize()
        np.testing.assert_allclose(d.loss.item(), z[f"out/{i}/loss"], rtol=1e-5)
        np.testing.assert_allclose(d.td_error[:32].cpu().numpy(), z[f"out/{i}/td_error"],
                                   rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(d.priorities[:32].cpu().numpy(), z[f"out/{i}/priorities"],
                                   rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(q.cpu().numpy(), z[f"out/{i}/q_tm1"], rtol=1e-5, atol=1e-6)
        if i == 0:
            g = d.get_params("grads")
            for k in names:
                ref = z[f"out/0/grad/{k}"]
                bound = 1e-4 * np.abs(ref) + 2e-5 * np.abs(ref).max() + 1e-30
                assert (np.abs(g[k] - ref) <= bound).all(), k
        got = d.get_params("params")
        tgt = d.get_params("target")
        for k in names:
            _check_params(got[k], z[f"out/{i}/params/{k}"], 1e-3, k)
            _check_params(tgt[k], z[f"out/{i}/target/{k}"], 1e-3, "target " + k)
        assert d.num_steps == i + 1


def test_nature_fixture_three_steps():
    """DQNAtariNetwork, B = 4, three free-running steps with target copies after steps 0
    and 2, against the f64 trajectory's losses, TD errors, q values and parameter
    fingerprints."""
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    z = _load("dqn_nature_b4.npz")
    net = DQNAtariNetwork(18)
    p, t = net.init(1), net.init(2)
    assert G.sha(*[p[k] for k in sorted(p)]) == str(z["in/params_sha"])
    B = G.NATURE_B
    d = NativeDQN(network="nature", num_actions=18, max_batch=B, obs_dtype="uint8",
                  target_update_period=2)
    d.set_params(p, t)
    q = torch.empty(B, 18, device="cuda")
    for i, b in enumerate(G.nature_batches()):
        assert G.sha(b["o_tm1"], b["o_t"]) == str(z[f"in/{i}/frames_sha"])
        d.step(*_dev(b), q_tm1=q)
        torch.cuda.synchronize()
        np.testing.assert_allclose(d.loss.item(), z[f"out/{i}/loss"], rtol=1e-5)
        np.testing.assert_allclose(d.td_error[:B].cpu().numpy(), z[f"out/{i}/td_error"],
                                   rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(d.priorities[:B].cpu().numpy(), z[f"out/{i}/priorities"],
                                   rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(q.cpu().numpy(), z[f"out/{i}/q_tm1"], rtol=1e-5, atol=1e-6)
        if i == 0:
            g = d.get_params("grads")
            for k in g:
                ref = z[f"out/0/grad/{k}/val"]
                got = g[k].reshape(-1)[z[f"out/0/grad/{k}/idx"]]
                bound = 1e-4 * np.abs(ref) + 2e-5 * np.abs(g[k]).max() + 1e-30
                assert (np.abs(got - ref) <= bound).all(), k
        for which in ("params", "target"):
            cur = d.get_params(which)
            for k, x in cur.items():
                ref = z[f"out/{i}/{which}/{k}/val"]
                _check_params(x.reshape(-1)[z[f"out/{i}/{which}/{k}/idx"]], ref, 1e-3,
                              f"step {i} {which} {k}")
        if i in (0, 2):  # post-update target copy (learning.py:157-161), bit-identical
            pa, ta = d.get_params("params"), d.get_params("target")
            for k in pa:
                np.testing.assert_array_equal(pa[k], ta[k])
