"""The bench's data-parallel DQN path (bench.py setup_dqn with WORLD_SIZE N, what
`bench.py --gpus N` runs on every rank) rehearsed on one GPU with N gloo ranks: N = 2 at
B = 32 per rank, and N = 8 (the 8-GPU node's rank count) at B = 16 per rank, so share
allocation, the 2 B cap per rank, the LAG = 2 mass snapshots and the ordering of the
per-step collectives run at the real rank count before the driver's first 8-GPU run.  The
N = 8 case runs 12 steps at prefetch 2 from skewed shard masses (rank 0's
initial priorities 30, the others 1 -- 7.7x the mass, so its proportional share of the
128-row global draw is 68 and the 2 B = 32 cap binds throughout), so every draw after the
first LAG gets unequal shares from the write-backs' mass snapshots.

Each rank builds exactly the bench's learner: a device-filled uint8 Atari shard
(fill_synthetic, priorities 1), make_reverb_dataset with prefetch, DQNLearner over
torch.distributed (global-probability shares, the IS normaliser's MIN all-reduce, the two
gradient buckets, the ranks' skip gate in the torso bucket).  Checked:
  * every draw bit-exact against the C oracle's global draw over the two shards (shares
    from the mass snapshot LAG draws earlier, each shard's own Philox stream), the oracle
    tables taking the learners' priority write-backs in the dataset's order (draw k is
    issued after the write-backs of steps < k - prefetch);
  * both replicas end with bit-identical parameters and no skipped step;
  * the replicas' parameters equal one learner stepping on the union batch with the
    reported probabilities, averaged over N * B (free-running, the suite's trajectory bar).
Reference: the only data-parallel learner of the reference, crr/recurrent_learning.py:346-358
(mean of the replicas' gradients, then the update); DQNLearner._step
(agents/tf/dqn/learning.py:112-168).
"""

import os
import socket
import sys
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SHARD = 1024
UNION_STEPS = 4  # the union-batch learner follows the replicas this far (free-running)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init_priority(WORLD, rank):
    return 30.0 if WORLD == 8 and rank == 0 else 1.0


def _worker(rank, WORLD, B, STEPS, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    import bench
    args = SimpleNamespace(batch=B, replay_size=WORLD * SHARD, num_actions=18, prefetch=2,
                           cpu_baseline_seconds=0.0)
    step, _, meta, _, _ = bench.setup_dqn(args, WORLD, rank, torch.device("cuda", 0))
    learner = step.__self__
    p_init = _init_priority(WORLD, rank)
    if p_init != 1.0:  # before the first draw (the dataset draws on the first step)
        keys = torch.arange(SHARD, dtype=torch.int64, device="cuda").view(torch.uint64)
        meta["_table"].native.update_priorities(keys, torch.full((SHARD,), p_init,
                                                                 dtype=torch.float64))
        torch.cuda.synchronize()
    records = []

    class _Rec:
        def __init__(self, it):
            self.it = it

        def __iter__(self):
            return self

        def __next__(self):
            s = next(self.it)
            d = s.data
            records.append(dict(keys=s.info.key.cpu().numpy().view(np.uint64).copy(),
                                probs=s.info.probability.cpu().numpy().copy(),
                                rows=[x.cpu().numpy().copy() for x in d[:5]]))
            return s

        def __getattr__(self, name):  # the dataset's events and frame copy
            return getattr(self.it, name)

    learner._iterator = _Rec(learner._iterator)
    prios = []
    union_params = None
    for i in range(STEPS):
        step()
        torch.cuda.synchronize()
        n = len(records[len(prios)]["keys"])
        prios.append(learner.native.priorities[:n].cpu().numpy().copy())
        if i + 1 == UNION_STEPS:
            union_params = learner.native.params.cpu().numpy()
    for rec, pr in zip(records, prios):
        rec["prios"] = pr
    q.put((rank, records, learner.native.params.cpu().numpy(), learner.native.guard_state(),
           union_params))
    dist.destroy_process_group()


@pytest.mark.parametrize("WORLD,B,STEPS", [(2, 32, 4), (8, 16, 12)])
def test_bench_data_parallel_path(WORLD, B, STEPS):
    from acme_amd.native import NativeDQN
    from acme_amd.networks import DQNAtariNetwork
    from acme_amd.replay.sharding import LAG, allocate_shares
    from tests._oracle import OracleTable
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, B, STEPS, port, q))
             for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        r, recs, params, guard, union_params = q.get(timeout=300)
        res[r] = (recs, params, guard, union_params)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(1, WORLD):
        np.testing.assert_array_equal(res[0][1], res[r][1])  # replicas identical
    for r in range(WORLD):
        assert res[r][2]["skipped"] == 0 and res[r][2]["applied"] == STEPS, res[r][2]
    # Draws: the bench's shards (priorities 1, seeds 1234 + rank) against the oracle.
    orc = []
    for r in range(WORLD):
        o = OracleTable(SHARD, True, 0.6, 1234 + r)
        o.insert(np.full(SHARD, _init_priority(WORLD, r)))
        orc.append(o)
    NB = WORLD * B
    P = 2  # the bench's prefetch (args.prefetch above)
    snaps, applied, all_shares = [], 0, []
    for k in range(STEPS):
        while applied < k - P:  # write-backs of steps < k - P precede draw k
            for r in range(WORLD):
                rec = res[r][0][applied]
                orc[r].update(rec["keys"].astype(np.int64), rec["prios"])
            applied += 1
        snaps.append([o.total() for o in orc])  # the mass snapshot after draw k
        shares = [B] * WORLD if k < LAG else allocate_shares(snaps[k - LAG], NB, cap=2 * B)
        all_shares.append(shares)
        for r in range(WORLD):
            rec = res[r][0][k]
            ref = orc[r].sample(shares[r], k)
            np.testing.assert_array_equal(rec["keys"], ref["keys"], err_msg=f"step {k} rank {r}")
            np.testing.assert_array_equal(rec["probs"], ref["probabilities"] * (shares[r] / NB))
    if WORLD == 8:  # the skewed masses: unequal shares, rank 0 at the 2 B cap
        late = all_shares[LAG:]
        assert all(sh[0] == 2 * B for sh in late), late
        assert all(min(sh) < B for sh in late) and all(sum(sh) == NB for sh in late), late
    # One learner on the union batches, mean over N * B (the bench's learner settings), for
    # the first UNION_STEPS steps.
    net = DQNAtariNetwork(18)
    d = NativeDQN(network="nature", num_actions=18, max_batch=2 * NB, obs_dtype="uint8",
                  discount=0.99, importance_sampling_exponent=0.2, learning_rate=1e-3,
                  target_update_period=100)
    d.set_params(net.init(0), net.init(1))
    for k in range(UNION_STEPS):
        cols = [np.concatenate([res[r][0][k]["rows"][c] for r in range(WORLD)]) for c in range(5)]
        probs = np.concatenate([res[r][0][k]["probs"] for r in range(WORLD)])
        dev = [torch.as_tensor(x).cuda().contiguous() for x in cols + [probs]]
        d.step(*dev)
    torch.cuda.synchronize()
    got = d.params.cpu().numpy()
    np.testing.assert_allclose(res[0][3], got, rtol=1e-5, atol=1e-3 + 1e-6)
    assert np.mean(np.abs(res[0][3] - got) <= 1e-5 * np.abs(got) + 1e-6) > 0.98
