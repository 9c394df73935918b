"""The torch-CPU restatement used as bench.py's CPU baseline (oracle/dqn_torch.py, SURVEY
§8(d)) equals the numpy oracle's TF DQN step (float64) to float32 accuracy: loss, |td|
priorities, and the parameters after one Adam step and the step-0 target copy."""

import numpy as np
import torch

from oracle import dqn_oracle as O
from oracle.dqn_torch import TorchDQN


def test_torch_cpu_step_matches_numpy_oracle():
    from acme_amd.networks import DQNAtariNetwork
    torch.set_num_threads(4)
    rng = np.random.default_rng(0)
    B, A = 6, 18
    net = DQNAtariNetwork(A)
    p = net.init(1)
    batch = dict(o_tm1=rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8),
                 a_tm1=rng.integers(0, A, B).astype(np.int32),
                 r_t=(1.5 * rng.standard_normal(B)).astype(np.float32),
                 d_t=np.where(rng.random(B) < 0.3, 0, 0.99 ** 4).astype(np.float32),
                 o_t=rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8),
                 probabilities=rng.uniform(1e-6, 1e-3, B))
    z = {k: np.zeros_like(v) for k, v in p.items()}
    state = dict(params=p, target={k: v.copy() for k, v in p.items()}, m=z, v=dict(z),
                 num_steps=0)
    out, _, new = O.dqn_step(O.DQNConfig(num_actions=A), state, batch, np.float64)
    t = TorchDQN(p, A)
    loss, prio = t.step(*(torch.from_numpy(batch[k]) for k in
                          ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")), batch["probabilities"])
    np.testing.assert_allclose(loss, out["loss"], rtol=1e-5)
    np.testing.assert_allclose(prio, out["priorities"], rtol=1e-4, atol=1e-6)
    for k in p:
        got = t.p[k].detach().numpy()
        np.testing.assert_allclose(got, new["params"][k], rtol=1e-5, atol=1e-3 + 1e-6)
        np.testing.assert_array_equal(t.t[k].numpy(), got)  # step-0 copy, post-update
    assert t.num_steps == 1
