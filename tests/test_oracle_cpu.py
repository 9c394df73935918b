"""CPU checks of the oracles themselves (no GPU).

The replay oracle (oracle/replay_oracle.c) is pinned by the published Philox4x32-10
known-answer vectors (Random123 kat_vectors) and by the fdlibm accuracy of its log/exp.
The learner oracle (oracle/dqn_oracle.py) has no reference golden vectors (TF/trfl/Sonnet
are absent): it is cross-checked against an independent formulation —
torch autograd on CPU — for forward values and every gradient.
"""

import math

import numpy as np
import pytest
import torch

from oracle import dqn_oracle as O
from tests import _oracle


# ----------------------------------------------------------------------- replay oracle
@pytest.mark.parametrize("ctr,key,expect", [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
])
def test_philox_known_answers(ctr, key, expect):
    assert list(_oracle.philox(ctr, key)) == expect


def test_fdlibm_log_exp_accuracy():
    L = _oracle.load()
    rng = np.random.default_rng(0)
    for x in np.exp(rng.uniform(-700, 700, 5000)):
        assert abs(L.oracle_log(x) - math.log(x)) <= 2.3e-16 * max(abs(math.log(x)), 1e-300)
    for y in rng.uniform(-700, 700, 5000):
        assert abs(L.oracle_exp(y) - math.exp(y)) <= 2.3e-16 * math.exp(y)
    assert L.oracle_priority_weight(1.0, 0.6) == 1.0
    assert L.oracle_priority_weight(0.0, 0.6) == 0.0
    assert L.oracle_priority_weight(2.5, 1.0) == 2.5


def test_oracle_tree_distribution():
    """The restated sampler draws i with probability p_i^alpha / sum (chi-square)."""
    cap = 50
    pr = np.linspace(0.0, 3.0, cap)
    t = _oracle.OracleTable(cap, True, 0.6, 5)
    t.insert(pr)
    counts = np.zeros(cap)
    for step in range(200):
        s = t.sample(1000, step)
        counts += np.bincount(s["slots"], minlength=cap)
        w = pr ** 0.6
        np.testing.assert_allclose(s["probabilities"], (w / w.sum())[s["slots"]], rtol=1e-12)
    w = pr ** 0.6
    exp = w / w.sum() * counts.sum()
    assert counts[exp == 0].sum() == 0
    chi2 = (((counts - exp) ** 2)[exp > 0] / exp[exp > 0]).sum()
    assert chi2 < 90  # 48 dof


def test_oracle_fifo_and_updates():
    t = _oracle.OracleTable(10, True, 1.0, 0)
    t.insert(np.ones(15))  # keys 0..14, slots hold keys 5..14
    t.update(np.array([3, 7, 7], np.uint64), np.array([9.0, 2.0, 4.0]))  # 3 evicted; last wins
    leaves = t.leaves()[:10]
    assert leaves[7] == 4.0 and leaves.sum() == 13.0
    assert t.total() == 13.0


def test_u8_scaling_exact():
    """The conv1 loader's reciprocal + fma correction equals float32(x / 255.0)."""
    x = np.arange(256)
    xf = x.astype(np.float32)
    c = np.float32(1.0) / np.float32(255.0)
    q = xf * c
    # fma in float64 is exact for these products; round once to float32.
    r = (-(q.astype(np.float64)) * 255.0 + xf.astype(np.float64)).astype(np.float32)
    q2 = (r.astype(np.float64) * np.float64(c) + q.astype(np.float64)).astype(np.float32)
    np.testing.assert_array_equal(q2, (x / 255.0).astype(np.float32))


# ----------------------------------------------------------------------- learner oracle
def _torch_nature_q(params, o, A):
    """Independent formulation with torch.nn.functional (NCHW conv, explicit SAME pads)."""
    x = torch.as_tensor((o / 255.0).astype(np.float32).astype(np.float64)).permute(0, 3, 1, 2)
    t = {k: torch.as_tensor(v.astype(np.float64), dtype=torch.float64).requires_grad_(True)
         for k, v in params.items()}
    for name, s, (pt, pl, pb, pr) in O.CONVS:
        w = t[name + "/w"].permute(3, 2, 0, 1)  # HWIO -> OIHW
        x = torch.nn.functional.pad(x, (pl, pr, pt, pb))
        x = torch.relu(torch.nn.functional.conv2d(x, w, t[name + "/b"], stride=s))
    flat = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)  # NHWC flatten order
    h = torch.relu(flat @ t["duelling_q_network/hidden/w"] + t["duelling_q_network/hidden/b"])
    v = h[:, :512] @ t["duelling_q_network/mlp/linear_1/w"] + t["duelling_q_network/mlp/linear_1/b"]
    adv = h[:, 512:] @ t["duelling_q_network/mlp_1/linear_1/w"] + \
        t["duelling_q_network/mlp_1/linear_1/b"]
    return v + (adv - adv.mean(dim=-1, keepdim=True)), t


def test_nature_oracle_matches_torch_autograd():
    from acme_amd.networks import DQNAtariNetwork
    net = DQNAtariNetwork(6)
    rng = np.random.default_rng(0)
    params = net.init(seed=3)
    # Smaller hidden layer values keep the test fast; shapes are the real ones.
    B = 3
    batch = dict(o_tm1=rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8),
                 a_tm1=np.array([0, 5, 2], np.int32), r_t=np.array([0.5, -2.0, 1.0], np.float32),
                 d_t=np.array([0.96, 0.0, 0.96], np.float32),
                 o_t=rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8),
                 probabilities=np.array([1e-3, 2e-4, 5e-4]))
    target = net.init(seed=4)
    cfg = O.DQNConfig(num_actions=6)
    out, grads = O.dqn_loss_and_grads(cfg, params, target, batch, np.float64)
    q, t = _torch_nature_q(params, batch["o_tm1"], 6)
    np.testing.assert_allclose(q.detach().numpy(), out["q_tm1"], rtol=1e-10, atol=1e-12)
    # Loss built from the oracle's (stop-gradient) targets and weights.
    tgt = torch.as_tensor(out["td_error"] + out["q_tm1"][np.arange(B), batch["a_tm1"]])
    qa = q[torch.arange(B), torch.as_tensor(batch["a_tm1"], dtype=torch.long)]
    td = tgt - qa
    ax = td.abs()
    quad = torch.clamp(ax, max=1.0)
    loss = ((0.5 * quad ** 2 + (ax - quad)) * torch.as_tensor(out["importance_weights"])).mean()
    np.testing.assert_allclose(loss.item(), out["loss"], rtol=1e-12)
    loss.backward()
    for k, g in grads.items():
        np.testing.assert_allclose(g, t[k].grad.numpy(), rtol=1e-8, atol=1e-12, err_msg=k)


def test_mlp_oracle_matches_torch_autograd():
    from acme_amd.networks import MLP
    net = MLP(4, [50, 50], 2)
    rng = np.random.default_rng(1)
    params = net.init(seed=0)
    B = 16
    batch = dict(o_tm1=rng.standard_normal((B, 4)).astype(np.float32),
                 a_tm1=rng.integers(0, 2, B).astype(np.int32),
                 r_t=(rng.standard_normal(B) * 2).astype(np.float32),
                 d_t=np.full(B, 0.96, np.float32),
                 o_t=rng.standard_normal((B, 4)).astype(np.float32),
                 probabilities=rng.uniform(1e-3, 1e-2, B))
    cfg = O.DQNConfig(num_actions=2, network="mlp", obs_dim=4, hidden=(50, 50))
    out, grads = O.dqn_loss_and_grads(cfg, params, params, batch, np.float64)
    t = {k: torch.as_tensor(v.astype(np.float64)).requires_grad_(True) for k, v in params.items()}
    x = torch.as_tensor(batch["o_tm1"].astype(np.float64))
    for i in range(3):
        x = x @ t[f"mlp/linear_{i}/w"] + t[f"mlp/linear_{i}/b"]
        if i < 2:
            x = torch.relu(x)
    tgt = torch.as_tensor(out["td_error"] + out["q_tm1"][np.arange(B), batch["a_tm1"]])
    td = tgt - x[torch.arange(B), torch.as_tensor(batch["a_tm1"], dtype=torch.long)]
    ax = td.abs()
    quad = torch.clamp(ax, max=1.0)
    loss = ((0.5 * quad ** 2 + (ax - quad)) * torch.as_tensor(out["importance_weights"])).mean()
    np.testing.assert_allclose(loss.item(), out["loss"], rtol=1e-12)
    loss.backward()
    for k, g in grads.items():
        np.testing.assert_allclose(g, t[k].grad.numpy(), rtol=1e-9, atol=1e-14, err_msg=k)


def test_double_q_target_semantics():
    """trfl.double_qlearning: argmax of the SELECTOR (first max), value from the TARGET."""
    from acme_amd.networks import MLP
    net = MLP(2, [], 3)
    p = {"mlp/linear_0/w": np.eye(2, 3, dtype=np.float32), "mlp/linear_0/b": np.zeros(3, np.float32)}
    tg = {"mlp/linear_0/w": np.array([[0, 0, 5], [0, 7, 0]], np.float32),
          "mlp/linear_0/b": np.zeros(3, np.float32)}
    batch = dict(o_tm1=np.array([[1.0, 0.0]], np.float32), a_tm1=np.array([0], np.int32),
                 r_t=np.array([3.0], np.float32), d_t=np.array([0.5], np.float32),
                 o_t=np.array([[2.0, 2.0]], np.float32), probabilities=np.array([1.0]))
    cfg = O.DQNConfig(num_actions=3, network="mlp", obs_dim=2, hidden=(), discount=1.0)
    out, _ = O.dqn_loss_and_grads(cfg, p, tg, batch, np.float64)
    # selector q(o_t) = [2, 2, 0] -> first max = action 0 -> target value q_t[0] = 0;
    # reward 3 is clipped to 1; q_tm1[a=0] = 1 -> td = 1 + 0.5 * 0 - 1 = 0.
    assert out["td_error"][0] == 0.0
    del net


def test_adam_matches_kingma_ba():
    rng = np.random.default_rng(0)
    p, g = rng.standard_normal(100).astype(np.float32), rng.standard_normal(100).astype(np.float32)
    m = np.zeros(100, np.float32)
    v = np.zeros(100, np.float32)
    p1, m1, v1 = O.adam_update(p, g, m, v, 1, 1e-3)
    # Step 1: m_hat = g, v_hat = g^2 -> update = lr * g / (|g| + eps).
    np.testing.assert_allclose(p1, p - 1e-3 * g / (np.abs(g) + 1e-8), rtol=2e-6, atol=1e-9)
