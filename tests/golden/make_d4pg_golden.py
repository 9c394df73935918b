"""Generates tests/golden/d4pg_step_b8.npz: one D4PG learner step (B = 8, 24-dim
observations, 6-dim actions, 51 atoms on [-150, 150], reduced hidden widths) from the
float64 restatement oracle/d4pg_oracle.py (which tests/test_d4pg_oracle_cpu.py pins
against torch autograd).  The reference's own tests hold no D4PG values (SURVEY.md
§8(c)), so this fixture pins regressions of the restatement and is the common input of
the CPU and GPU parity tests.

    python -m tests.golden.make_d4pg_golden
"""

import os

import numpy as np

from oracle import d4pg_oracle as O

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "d4pg_step_b8.npz")


def golden_cfg():
    return O.D4PGConfig(obs_dim=24, act_dim=6, policy_sizes=(32, 32, 32),
                        critic_sizes=(64, 64, 32), num_atoms=51, vmin=-150.0, vmax=150.0,
                        target_update_period=100)


def make_inputs(cfg, B=8, seed=0):
    rng = np.random.default_rng(seed)
    z = {}
    for which in ("params", "target"):
        for name, shape in O.d4pg_tensor_shapes(cfg):
            if name.endswith("/scale"):
                v = 1.0 + 0.1 * rng.standard_normal(shape)
            elif name.endswith("/b") or name.endswith("/offset"):
                v = 0.1 * rng.standard_normal(shape)
            else:
                v = rng.standard_normal(shape) / np.sqrt(shape[0])
            z[f"in/{which}/{name}"] = v.astype(np.float32)
    # Config-3 shaped batch: o ~ N(0,1), a ~ U[-1,1], r ~ U[0,5],
    # d = 0.99^4 with a terminal.
    z["in/o_tm1"] = rng.standard_normal((B, cfg.obs_dim)).astype(np.float32)
    z["in/a_tm1"] = rng.uniform(-1, 1, (B, cfg.act_dim)).astype(np.float32)
    z["in/r_t"] = rng.uniform(0, 5, B).astype(np.float32)
    d = np.full(B, 0.99 ** 4, np.float32)
    d[3] = 0.0
    z["in/d_t"] = d
    z["in/o_t"] = rng.standard_normal((B, cfg.obs_dim)).astype(np.float32)
    return z


def unpack(cfg, z):
    params = {n: z[f"in/params/{n}"] for n, _ in O.d4pg_tensor_shapes(cfg)}
    target = {n: z[f"in/target/{n}"] for n, _ in O.d4pg_tensor_shapes(cfg)}
    batch = {k: z[f"in/{k}"] for k in ("o_tm1", "a_tm1", "r_t", "d_t", "o_t")}
    return params, target, batch


def compute(cfg, z):
    params, target, batch = unpack(cfg, z)
    zeros = {k: np.zeros_like(v) for k, v in params.items()}
    # num_steps = 1: no start-of-step target copy, Adam t = 2.
    state = dict(params=params, target=target, m=zeros, v=dict(zeros), num_steps=1)
    out, raw, new = O.d4pg_step(cfg, state, batch, np.float64)
    res = {"critic_loss": np.float64(out["critic_loss"]),
           "policy_loss": np.float64(out["policy_loss"]),
           "q_tm1": out["q_tm1"], "q_t": out["q_t"], "dqda": out["dqda"],
           "dpg_a": out["dpg_a"], "a_target": out["a_target"],
           "norms": np.asarray(out["norms"], np.float64)}
    for k, g in raw.items():
        res["grad/" + k] = g
    for k, p in new["params"].items():
        res["new/" + k] = p
    return res


def main():
    cfg = golden_cfg()
    z = make_inputs(cfg)
    res = compute(cfg, z)
    z.update({"out/" + k: v for k, v in res.items()})
    np.savez_compressed(OUT, **z)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes)")


if __name__ == "__main__":
    main()
