"""Generates the SURVEY.md §8(c) parity fixtures from the CPU restatements in oracle/.

The reference's own tests hold no learner, V-trace or sampler values (SURVEY.md §8(c):
parity is unpinned at the trfl / Sonnet / Reverb boundary), so these fixtures pin the
restatements against drift and are the common inputs of the CPU tests
(tests/test_golden_cpu.py: the oracle reproduces them) and the GPU tests
(tests/test_golden_gpu.py: the HIP path reproduces them through the C ABI).

    python -m tests.golden.make_parity_goldens

Fixtures (all small; large tensors are stored as fingerprints, see `fingerprint`):
  dqn_cartpole_b32.npz   DQN TF learner (agents/tf/dqn/learning.py:112-161) on the
                         CartPole MLP [50, 50] (examples/bsuite/run_dqn.py:46-49), B = 32,
                         3 steps with target_update_period 2 (copies after steps 0 and 2).
  dqn_nature_b4.npz      the same learner on DQNAtariNetwork (18 actions), uint8 frames,
                         B = 4, 3 steps, target_update_period 2.  Parameters come from the
                         seeded initialiser and the frames from a seeded generator; both are
                         checked against stored SHA-256 digests before use.
  vtrace_t20_b4.npz      trfl.vtrace_from_importance_weights (agents/tf/impala/
                         learning.py:133-139), T = 20, B = 4, with rho > 1 and terminals.
  sampler_1k.npz         prioritized(0.6) table of capacity 1000 (FIFO over 1100 inserts,
                         zero priorities included): 3 draws of 64, then 64 priority updates
                         (duplicates, an evicted key), then 3 more draws.
"""

import hashlib
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
NATURE_STEPS = 3
NATURE_B = 4
SAMPLE_IDX = 256  # elements per tensor kept in a fingerprint


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def fingerprint(name: str, x: np.ndarray):
    """(indices, values, sum, abs-sum) of a tensor: a fixed pseudo-random subset of its
    elements (seeded by the tensor name) plus two f64 reductions."""
    flat = np.asarray(x).reshape(-1)
    seed = int(hashlib.sha256(name.encode()).hexdigest()[:8], 16)
    idx = np.random.default_rng(seed).choice(flat.size, min(SAMPLE_IDX, flat.size),
                                             replace=False)
    idx.sort()
    return idx.astype(np.int64), flat[idx].astype(np.float64), \
        np.float64(flat.astype(np.float64).sum()), np.float64(np.abs(flat.astype(np.float64)).sum())


# --------------------------------------------------------------------------- DQN
def cartpole_net():
    from acme_amd.networks import MLP
    return MLP(4, [50, 50], 2)


def cartpole_batches(B=32, steps=3, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(steps):
        out.append(dict(o_tm1=rng.standard_normal((B, 4)).astype(np.float32),
                        a_tm1=rng.integers(0, 2, B).astype(np.int32),
                        r_t=(1.5 * rng.standard_normal(B)).astype(np.float32),
                        d_t=np.where(rng.random(B) < 0.15, 0.0, 0.99 ** 4).astype(np.float32),
                        o_t=rng.standard_normal((B, 4)).astype(np.float32),
                        probabilities=rng.uniform(1e-5, 1e-3, B)))
    return out


def nature_batches(B=NATURE_B, steps=NATURE_STEPS, seed=7):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(steps):
        out.append(dict(o_tm1=rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8),
                        a_tm1=rng.integers(0, 18, B).astype(np.int32),
                        r_t=(1.5 * rng.standard_normal(B)).astype(np.float32),
                        d_t=np.where(rng.random(B) < 0.25, 0.0, 0.99 ** 4).astype(np.float32),
                        o_t=rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8),
                        probabilities=rng.uniform(1e-6, 1e-3, B)))
    return out


def run_dqn(cfg, params, target, batches):
    from oracle import dqn_oracle as O
    state = dict(params=params, target=target,
                 m={k: np.zeros_like(v) for k, v in params.items()},
                 v={k: np.zeros_like(v) for k, v in params.items()}, num_steps=0)
    outs, grads0, states = [], None, []
    for i, b in enumerate(batches):
        out, grads, state = O.dqn_step(cfg, state, b, np.float64)
        outs.append(out)
        states.append(state)
        if i == 0:
            grads0 = grads
    return outs, grads0, states


def make_cartpole():
    from oracle import dqn_oracle as O
    net = cartpole_net()
    cfg = O.DQNConfig(num_actions=2, network="mlp", obs_dim=4, hidden=(50, 50),
                      target_update_period=2)
    p, t = net.init(1), net.init(2)
    batches = cartpole_batches()
    outs, g0, states = run_dqn(cfg, p, t, batches)
    z = {}
    for k in p:
        z[f"in/params/{k}"], z[f"in/target/{k}"] = p[k], t[k]
    for i, b in enumerate(batches):
        for k, v in b.items():
            z[f"in/{i}/{k}"] = v
        z[f"out/{i}/loss"] = np.float64(outs[i]["loss"])
        for k in ("td_error", "priorities", "q_tm1"):
            z[f"out/{i}/{k}"] = outs[i][k]
        for k in p:
            for which in ("params", "target", "m", "v"):
                z[f"out/{i}/{which}/{k}"] = states[i][which][k]
    for k, g in g0.items():
        z[f"out/0/grad/{k}"] = g
    path = os.path.join(HERE, "dqn_cartpole_b32.npz")
    np.savez_compressed(path, **z)
    return path


def make_nature():
    from acme_amd.networks import DQNAtariNetwork
    from oracle import dqn_oracle as O
    net = DQNAtariNetwork(18)
    cfg = O.DQNConfig(num_actions=18, target_update_period=2)
    p, t = net.init(1), net.init(2)
    batches = nature_batches()
    outs, g0, states = run_dqn(cfg, p, t, batches)
    z = {"in/params_sha": np.array(sha(*[p[k] for k in sorted(p)])),
         "in/target_sha": np.array(sha(*[t[k] for k in sorted(t)]))}
    for i, b in enumerate(batches):
        z[f"in/{i}/frames_sha"] = np.array(sha(b["o_tm1"], b["o_t"]))
        for k in ("a_tm1", "r_t", "d_t", "probabilities"):
            z[f"in/{i}/{k}"] = b[k]
        z[f"out/{i}/loss"] = np.float64(outs[i]["loss"])
        for k in ("td_error", "priorities", "q_tm1"):
            z[f"out/{i}/{k}"] = outs[i][k]
        for which in ("params", "target"):
            for k, x in states[i][which].items():
                idx, val, s, a = fingerprint(k, x)
                z[f"out/{i}/{which}/{k}/idx"] = idx
                z[f"out/{i}/{which}/{k}/val"] = val
                z[f"out/{i}/{which}/{k}/sum"] = s
                z[f"out/{i}/{which}/{k}/abssum"] = a
    for k, g in g0.items():
        idx, val, s, a = fingerprint(k, g)
        z[f"out/0/grad/{k}/idx"], z[f"out/0/grad/{k}/val"] = idx, val
        z[f"out/0/grad/{k}/sum"], z[f"out/0/grad/{k}/abssum"] = s, a
    path = os.path.join(HERE, "dqn_nature_b4.npz")
    np.savez_compressed(path, **z)
    return path


# --------------------------------------------------------------------------- V-trace
def vtrace_inputs(T=20, B=4, seed=3):
    rng = np.random.default_rng(seed)
    log_rhos = 0.8 * rng.standard_normal((T, B))  # both sides of the rho / c clip at 1
    discounts = np.where(rng.random((T, B)) < 0.1, 0.0, 0.99)
    rewards = 2.0 * rng.standard_normal((T, B))
    values = rng.standard_normal((T, B))
    bootstrap = rng.standard_normal(B)
    return log_rhos, discounts, rewards, values, bootstrap


def make_vtrace():
    from oracle import impala_oracle as O
    x = vtrace_inputs()
    vs, pg = O.vtrace(*x)
    names = ("log_rhos", "discounts", "rewards", "values", "bootstrap")
    z = {f"in/{n}": v for n, v in zip(names, x)}
    z["out/vs"], z["out/pg_advantages"] = vs, pg
    path = os.path.join(HERE, "vtrace_t20_b4.npz")
    np.savez_compressed(path, **z)
    return path


# --------------------------------------------------------------------------- sampler
SAMPLER = dict(capacity=1000, alpha=0.6, seed=1234, inserts=1100, batch=64)


def sampler_inputs():
    rng = np.random.default_rng(11)
    pr = rng.uniform(0.05, 3.0, SAMPLER["inserts"])
    pr[rng.choice(SAMPLER["inserts"], 40, replace=False)] = 0.0
    keys = rng.integers(100, SAMPLER["inserts"], 64).astype(np.uint64)
    keys[5] = keys[40] = 777          # duplicate key: the later update wins
    keys[9] = 3                       # evicted by FIFO (only keys >= 100 remain): ignored
    upd = rng.uniform(0.0, 4.0, 64)
    return pr, keys, upd


def run_sampler(table_factory):
    """Drives a table (oracle or GPU, same interface) through the fixture's script."""
    pr, keys, upd = sampler_inputs()
    t = table_factory()
    t.insert(pr)
    draws = [t.sample(SAMPLER["batch"], step) for step in range(3)]
    t.update(keys, upd)
    draws += [t.sample(SAMPLER["batch"], step) for step in range(3, 6)]
    return draws


def make_sampler():
    from tests._oracle import OracleTable
    draws = run_sampler(lambda: OracleTable(SAMPLER["capacity"], True, SAMPLER["alpha"],
                                            SAMPLER["seed"]))
    pr, keys, upd = sampler_inputs()
    z = {"in/priorities": pr, "in/update_keys": keys, "in/update_priorities": upd}
    for i, d in enumerate(draws):
        for k, v in d.items():
            z[f"out/{i}/{k}"] = v
    path = os.path.join(HERE, "sampler_1k.npz")
    np.savez_compressed(path, **z)
    return path


def main():
    for fn in (make_cartpole, make_nature, make_vtrace, make_sampler):
        path = fn()
        print(f"wrote {path} ({os.path.getsize(path)} bytes)")


if __name__ == "__main__":
    main()
