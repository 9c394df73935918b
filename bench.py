#!/usr/bin/env python3
"""Learner throughput benchmark: sampled transitions/sec through DQN Learner.step().

Workload (BASELINE.json configs[1]): Nature-CNN DQN
(DQNAtariNetwork, 18 actions), synthetic uint8 [84, 84, 4] transitions in a 1,000,000-slot
GPU-resident prioritized replay (alpha 0.6, beta 0.2, n-step discount 0.99^4), batch 512
per GPU, Adam lr 1e-3, target period 100.  One "step" = prioritized sample + gather of the
(o_tm1, a, r, d, o_t) batch + the full learner step (3 Q forwards, double-Q TD, Huber,
f64 IS weights, backward, Adam, periodic target copy) + priority write-back — exactly the
work of DQNLearner._step (acme/agents/tf/dqn/learning.py:112-168) plus its iterator.

N > 1 (torchrun, one process per GPU): the 1M-slot replay is sharded 1/N per rank, every
rank draws its own 512 (weak scaling, global batch 512 N), the IS-weight normaliser is
all-reduced (MIN of probabilities) and the gradients are all-reduced (AVG) over RCCL
before Adam, so every replica applies the identical update.

Prints ONE JSON line on rank 0 (contract in the task statement / DESIGN.md §6).
"""

from __future__ import annotations

import argparse
import gc
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "learner transitions/sec (sample+step) at batch 512, 1/2/4/8 MI355X"
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 (spec)
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
OBS_BYTES = 84 * 84 * 4


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--workload", choices=("dqn", "d4pg", "impala", "impala_actors", "insert",
                                          "r2d2"),
                   default="dqn",
                   help="dqn: the headline config (BASELINE configs[1]); d4pg: configs[2]; "
                        "impala: configs[3] (learner side); impala_actors: configs[3] end to "
                        "end (--actors host actor threads feeding the device queue); insert: "
                        "host inserts into the configs[1] table while its learner steps")
    p.add_argument("--actors", type=int, default=64, help="impala_actors: environments / actors")
    p.add_argument("--actor-procs", type=int, default=12,
                   help="impala_actors: worker processes owning the environments and their "
                        "adders (ProcessActorPool; policy batched in this process); 0 = host "
                        "threads (--actor-threads)")
    p.add_argument("--actor-groups", type=int, default=1,
                   help="impala_actors with processes: environment groups whose policy steps "
                        "alternate with the other groups' environment steps")
    p.add_argument("--actor-threads", type=int, default=2,
                   help="impala_actors with --actor-procs 0: host threads stepping the "
                        "environments in batches (VectorActorPool); 0 = one thread per actor "
                        "(ActorPool)")
    p.add_argument("--batch", type=int, default=0, help="default 512 (dqn) / 256 (d4pg)")
    p.add_argument("--replay-size", type=int, default=1_000_000)
    p.add_argument("--num-actions", type=int, default=18)
    p.add_argument("--prefetch", type=int, default=4,
                   help="dataset prefetch_size (DQN; the reference DQN agent's default is 4)")
    p.add_argument("--settle-seconds", type=float, default=0.5,
                   help="after the --warmup steps, further untimed steps until this much warm-up "
                        "time has passed (the GPU's clocks ramp over the first ~20 ms of load); "
                        "the count is reported as settle_steps")
    p.add_argument("--no-profile", action="store_true", help="skip the profiled pass")
    p.add_argument("--profile-steps", type=int, default=50,
                   help="steps of the separate, untimed section-profiler pass")
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-staged", action="store_true",
                   help="dqn: skip the dp_staged_ms_per_step pass (kernel traces of the fused step)")
    return p.parse_args()


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(batch: int, num_actions: int, seconds: float):
    """SURVEY §8(d)'s CPU baseline: the build's float32 torch-CPU restatement of the TF
    DQN step (oracle/dqn_torch.py: F.conv2d + autograd + Sonnet Adam) fed by the C oracle's
    prioritized sum tree over 1,000,000 slots (draw, gather, step, priority write-back),
    timed on the host cores: all of them (torch.set_num_threads), then one thread.  The
    frames of the 1M slots would be 56 GB of host memory, so slot s reads frame pair
    s mod 16,384 of a host pool (the tree, draws and priorities are the full 1M-slot ones).
    Sample: at least 200 timed steps with all threads, more if `seconds`
    allows, after one warm-up step; one thread: a bounded sample of `seconds` / 2 (at least
    1 step)."""
    from oracle.dqn_torch import TorchDQN
    from tests._oracle import OracleTable
    from acme_amd.networks import DQNAtariNetwork
    rng = np.random.default_rng(0)
    pool, cap = 16384, 1_000_000
    obs = torch.from_numpy(rng.integers(0, 256, (pool, 84, 84, 4), dtype=np.uint8))
    nxt = torch.from_numpy(rng.integers(0, 256, (pool, 84, 84, 4), dtype=np.uint8))
    act = torch.from_numpy(rng.integers(0, num_actions, pool).astype(np.int32))
    rew = torch.from_numpy(rng.standard_normal(pool).astype(np.float32))
    dis = torch.from_numpy(np.where(rng.random(pool) < 0.01, 0,
                                    np.float32(0.99) ** 4).astype(np.float32))
    table = OracleTable(cap, True, 0.6, 1234)
    table.insert(np.ones(cap))
    learner = TorchDQN(DQNAtariNetwork(num_actions).init(0), num_actions)
    draw = [0]

    def one():
        s = table.sample(batch, draw[0])
        draw[0] += 1
        k = torch.from_numpy(s["slots"] % pool)
        _, prio = learner.step(obs[k], act[k], rew[k], dis[k], nxt[k], s["probabilities"])
        table.update(s["keys"], prio)

    def timed(threads, budget, least, cap=float("inf")):
        torch.set_num_threads(threads)
        one()  # warm-up (page faults, oneDNN primitive creation)
        t0 = time.perf_counter()
        n, shown = 0, t0
        while (n < least or time.perf_counter() - t0 < budget) and time.perf_counter() - t0 < cap:
            one()
            n += 1
            if time.perf_counter() - shown > 15.0:  # a progress line (a silent minute reads as hung)
                shown = time.perf_counter()
                print(f"[bench] cpu baseline: {threads} threads, {n} steps in "
                      f"{shown - t0:.0f} s", file=sys.stderr, flush=True)
        return batch * n / (time.perf_counter() - t0), n

    # Three thread counts (SURVEY §8(d) times the reference CPU learner on the host cores of
    # the same box): every visible core (sched_getaffinity; the box's OMP_NUM_THREADS, 16, is
    # ignored), 16 threads and 1 thread.  On the GPU box 256 cores are visible but the box's
    # CPU share is 16 (round 5: 256 threads ran 29 transitions/s, 9 steps in 150 s, against
    # 2,603/s on 16 threads), so the all-cores sample is bounded (`seconds`, at least 1 step)
    # and the 16-thread one takes the >= 200 timed steps; `value` is the fastest of the three
    # and `cores` its thread count, with all three reported.
    cores = len(os.sched_getaffinity(0))
    print(f"[bench] cpu baseline: {cores} visible cores, then 16 threads, then 1", file=sys.stderr,
          flush=True)
    prev = torch.get_num_threads()
    try:
        v_all, n_all = timed(cores, seconds, 1, cap=seconds)
        t16 = min(16, cores)
        v_16, n_16 = timed(t16, seconds, 200, cap=150.0)
        v_one, n_one = timed(1, seconds / 2, 1)
    finally:
        torch.set_num_threads(prev)
    best = max((v_all, cores), (v_16, t16), (v_one, 1))
    return dict(value=round(best[0], 2), unit="transitions/s", cores=best[1], kind="port",
                value_all_cores=round(v_all, 2), visible_cores=cores,
                value_16threads=round(v_16, 2), value_1thread=round(v_one, 2),
                sample=(f"float32 torch-CPU restatement of the TF DQN step (oracle/dqn_torch.py) "
                        f"+ C sum-tree oracle over 1,000,000 slots (frames from a {pool}-slot "
                        f"host pool), batch {batch}: {n_16} timed steps on {t16} threads, {n_all} "
                        f"on all {cores} visible cores, {n_one} on 1 thread; value = the fastest; "
                        f"{cpu_model()}"))


def d4pg_cpu_baseline(batch: int, seconds: float):
    """The numpy D4PG oracle (oracle/d4pg_oracle.py, float32): a 16,384-slot host replay drawn
    uniformly, batch 256, config-3 networks, timed at three BLAS thread counts as the DQN
    baseline is (every visible core on a bounded sample of `seconds`, at least 1 step; 16
    threads for at least 200 timed steps, capped at 150 s; 1 thread for `seconds` / 2), after
    one warm-up step each; `value` is the fastest and `cores` its thread count."""
    from oracle import d4pg_oracle as O
    from acme_amd.networks import DistributionalCritic, LayerNormMLPPolicy
    from threadpoolctl import threadpool_limits
    rng = np.random.default_rng(0)
    cap = 16384
    obs = rng.standard_normal((cap, 24)).astype(np.float32)
    nxt = rng.standard_normal((cap, 24)).astype(np.float32)
    act = rng.uniform(-1, 1, (cap, 6)).astype(np.float32)
    rew = rng.uniform(0, 5, cap).astype(np.float32)
    dis = np.where(rng.random(cap) < 0.001, 0, np.float32(0.99) ** 4).astype(np.float32)
    cfg = O.D4PGConfig()
    p = dict(LayerNormMLPPolicy(24, 6).init(0))
    p.update(DistributionalCritic(24, 6).init(1))
    z = {k: np.zeros_like(v) for k, v in p.items()}
    state = [dict(params=p, target={k: v.copy() for k, v in p.items()}, m=z, v=dict(z),
                  num_steps=0)]

    def one():
        k = rng.integers(0, cap, batch)
        b = dict(o_tm1=obs[k], a_tm1=act[k], r_t=rew[k], d_t=dis[k], o_t=nxt[k])
        state[0] = O.d4pg_step(cfg, state[0], b, np.float32)[2]

    def timed(threads, budget, least, limit=float("inf")):
        with threadpool_limits(threads):
            one()  # warm-up
            t0 = time.perf_counter()
            n = 0
            while (n < least or time.perf_counter() - t0 < budget) and \
                    time.perf_counter() - t0 < limit:
                one()
                n += 1
            return batch * n / (time.perf_counter() - t0), n

    cores = len(os.sched_getaffinity(0))
    v_all, n_all = timed(cores, seconds, 1, limit=seconds)
    t16 = min(16, cores)
    v_16, n_16 = timed(t16, seconds, 200, limit=150.0)
    v_one, n_one = timed(1, seconds / 2, 1)
    best = max((v_all, cores), (v_16, t16), (v_one, 1))
    return dict(value=round(best[0], 2), unit="transitions/s", cores=best[1], kind="port",
                value_all_cores=round(v_all, 2), visible_cores=cores,
                value_16threads=round(v_16, 2), value_1thread=round(v_one, 2),
                sample=(f"numpy float32 oracle (oracle/d4pg_oracle.py), batch {batch}, uniform "
                        f"draws from a {cap}-slot host replay: {n_16} timed steps on {t16} BLAS "
                        f"threads, {n_all} on all {cores} visible cores, {n_one} on 1 thread; "
                        f"value = the fastest; {cpu_model()}"))


def setup_dqn(args, world, rank, dev):
    from acme_amd import replay, specs
    from acme_amd.adders import reverb as adders
    from acme_amd.agents.dqn import DQNLearner
    from acme_amd.datasets import make_reverb_dataset
    from acme_amd.networks import DQNAtariNetwork
    from acme_amd.utils import counting, loggers
    # The measured path is the drop-in one: GPU replay Table (Reverb replacement) ->
    # make_reverb_dataset iterator -> DQNLearner.step() -> update_priorities.
    B, A = args.batch or 512, args.num_actions
    shard = -(-args.replay_size // world)
    env_spec = specs.EnvironmentSpec(
        observations=specs.Array((84, 84, 4), np.uint8), actions=specs.DiscreteArray(A, np.int32),
        rewards=specs.Array((), np.float32), discounts=specs.BoundedArray((), np.float32, 0, 1))
    table = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Prioritized(0.6),
                         replay.selectors.Fifo(), shard, replay.rate_limiters.MinSize(1),
                         signature=adders.NStepTransitionAdder.signature(env_spec),
                         seed=1234 + rank, device=dev)
    assert [f.row_bytes for f in table.fields] == [OBS_BYTES, 4, 4, 4, OBS_BYTES]
    table.native.fill_synthetic(shard, layout=0, num_actions=A, seed=rank)
    server = replay.Server([table])
    # prefetch_size as the reference DQN agent (agents/tf/dqn/agent.py:50): batch k+4 is
    # sampled and gathered on the dataset's stream while step k runs.
    dataset = make_reverb_dataset(server, batch_size=B, prefetch_size=args.prefetch)
    net = DQNAtariNetwork(A)
    learner = DQNLearner(net, net, discount=0.99, importance_sampling_exponent=0.2,
                         learning_rate=1e-3, target_update_period=100, dataset=dataset,
                         replay_client=replay.Client(server), counter=counting.Counter(),
                         logger=loggers.NoOpLogger(), seed=0, device=dev,
                         reduce_logged_loss=False,
                         # timing-only builds (tools/, e.g. -DWS_EXP) compute garbage: skip
                         on_plane_overflow=os.environ.get("ACME_BENCH_ON_OVERFLOW", "reissue"))
    meta = dict(
        # The arithmetic: every GEMM operand as two scaled f16 planes (22-23 significant
        # bits, per-tensor power-of-two scale), three MFMA terms per product, f32
        # accumulation (csrc/gemm_p3.h); f32 everywhere else.
        metric=METRIC, dtype="f32 (2xf16 split planes, 3 MFMA terms)",
        data="synthetic (device-generated uint8 Atari-shape transitions, random-init "
             "Nature-CNN weights)",
        config={"workload": "dqn_nature_cnn_prioritized_replay (BASELINE configs[1])",
                "global_batch": B * world, "batch_per_gpu": B,
                "replay_slots": args.replay_size, "replay_slots_per_gpu": shard,
                "obs": "uint8[84,84,4]", "num_actions": A,
                "sampler": "prioritized(alpha=0.6), IS beta=0.2", "prefetch_size": args.prefetch,
                "parallelism": f"dp{world}"})
    meta["_table"] = table
    meta["_set_staged"] = lambda on: setattr(learner, "_staged", bool(on))
    # Adam against SURVEY §8(d)'s algorithmic bytes (7 x 4 B per parameter: p, m, v read and
    # written, g read) beside the kernel's design bytes (also the parameter planes it writes
    # and the conv weight gradients' split-K slabs it reduces), VERDICT r5 item 4.
    meta["_adam_survey_bytes"] = 28.0 * sum(int(np.prod(s)) for _, s in net.tensor_shapes())

    def guard():  # synchronises: read outside the timed window
        g = learner.native.guard_state()
        return dict(applied=g["applied"], skipped=g["skipped"],
                    reissued=learner._reissued,  # noqa: SLF001
                    verdict_timeouts=g["verdict_timeouts"])
    meta["_guard"] = guard
    return (learner.step, B, meta, lambda: float(learner.native.loss.item()),
            lambda: cpu_baseline(B, A, args.cpu_baseline_seconds))


def insert_bench(args, dev):
    """Actor-side insert path (north star: pinned hipMemcpyAsync on a side stream) into the
    1M-slot table of the headline config while the DQN learner steps.  Three measurements:
    learner steps alone; the same steps with a host thread stepping the reference DQN agent's
    NStepTransitionAdder (n_step 5, agents/tf/dqn/agent.py:57,103-108: one adder.add per
    environment step, one item each, through the table's native n-step writer) at the
    reference's ratio of one insert per 32 sampled items; and with a host thread committing
    whole staged chunks (the native stage/commit path, bulk).  Inserts/s counts items added
    inside the timed window of learner steps.  The environment's timesteps are pre-built
    (its own cost is not the insert path's)."""
    import threading
    from acme_amd import dm_env, replay as rp
    from acme_amd.adders import reverb as adders
    step, B, meta, _, _ = setup_dqn(args, 1, 0, dev)
    table = meta["_table"]
    nat = table.native
    rng = np.random.default_rng(0)
    pool = 512
    obs = rng.integers(0, 256, (pool, 84, 84, 4), dtype=np.uint8)
    acts = [np.int32(i % 18) for i in range(pool)]
    steps_ts = [dm_env.transition(np.float32(0.5), obs[i], np.float32(0.99)) for i in range(pool)]
    adder = adders.NStepTransitionAdder(rp.Client(rp.Server([table])), n_step=5, discount=0.99)
    adder.add_first(dm_env.restart(obs[0]))
    rows = [obs.reshape(pool, -1), np.arange(pool, dtype=np.int32).view(np.uint8).reshape(pool, 4),
            np.full(pool, 0.5, np.float32).view(np.uint8).reshape(pool, 4),
            np.full(pool, 0.99 ** 4, np.float32).view(np.uint8).reshape(pool, 4),
            np.roll(obs.reshape(pool, -1), -5, axis=0)]

    done = [0]

    def timed_steps(n):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            step()
            done[0] += 1
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    def with_inserter(body):
        count, stop = [0], threading.Event()

        def run():
            while not stop.is_set():
                count[0] += body()
        th = threading.Thread(target=run, daemon=True)
        th.start()
        try:
            time.sleep(0.2)  # the inserter reaches its steady state
            c0 = count[0]
            dt = timed_steps(args.steps)
            c1 = count[0]
        finally:
            stop.set()
            th.join()
        nat.sync_inserts()
        return dt, (c1 - c0) / dt

    env_t = [0]

    def adder_body(n=64):
        for _ in range(n):
            t = env_t[0] % pool
            adder.add(acts[t], steps_ts[t])
            env_t[0] += 1
        return n

    # The reference agent's ratio: one insert per samples_per_insert = 32 sampled items
    # (agents/tf/dqn/agent.py:52, agents/agent.py:45-89), i.e. B / 32 items per step.
    per_step = B // 32
    issued = [0]

    def paced_adder_body():
        if issued[0] >= (done[0] + 1) * per_step:
            time.sleep(50e-6)
            return 0
        issued[0] += adder_body(per_step)
        return per_step

    chunk = min(nat.stage_capacity(), pool)

    def bulk_body():
        bufs = nat.stage(chunk)
        for b, src in zip(bufs, rows):
            np.copyto(b, src[:chunk])
        nat.commit(chunk, None)
        return chunk

    for _ in range(args.warmup):
        step()
    t_alone = timed_steps(args.steps)
    issued[0] = done[0] * per_step
    t_paced, r_paced = with_inserter(paced_adder_body)
    t_bulk, r_bulk = with_inserter(bulk_body)
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 1.0:
        n += adder_body()
    table.flush()
    r_adder = n / (time.perf_counter() - t0)
    assert adder._fast, "the adder did not take the native writer path"  # noqa: SLF001
    # Bulk inserts with no learner running: the host + PCIe ceiling of the path.
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 2.0:
        n += bulk_body()
    nat.sync_inserts()
    r_solo = n / (time.perf_counter() - t0)
    item_bytes = sum(f.row_bytes for f in table.fields)
    out = {
        "metric": "host->HBM inserts/s into the 1M-slot prioritized table (pinned staging ring, "
                  "async upload to a device mirror, one-launch landing on the side stream) "
                  "while the DQN learner steps",
        "value": round(r_bulk, 1), "unit": "items/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "higher_is_better": True, "vs_baseline": None,
        "dtype": "u8", "data": "synthetic uint8 Atari transitions (56,460 B per item)",
        "config": {"workload": "dqn_insert (BASELINE configs[1] table + learner)",
                   "item_bytes": item_bytes, "staging_chunk_items": nat.stage_capacity(),
                   "batch": B},
        "inserts": {
            "bulk_items_per_s_concurrent": round(r_bulk, 1),
            "bulk_items_per_s_alone": round(r_solo, 1),
            "bulk_GB_per_s_alone": round(r_solo * item_bytes / 1e9, 2),
            "adder_items_per_s_alone": round(r_adder, 1),
            "adder_items_per_s_paced": round(r_paced, 1),
            "learner_ms_per_step_alone": round(1e3 * t_alone / args.steps, 4),
            "learner_ms_per_step_with_paced_adder_inserts": round(1e3 * t_paced / args.steps, 4),
            "learner_ms_per_step_with_bulk_inserts": round(1e3 * t_bulk / args.steps, 4),
            "reference_rate_needed_items_per_s": round(
                B / 32.0 / (t_alone / args.steps), 1),  # samples_per_insert = 32
            # The paced adder is held to B / 32 items per learner step, so its rate follows
            # the learner: the ratio it reached inside the window (the reference's 32).
            "paced_samples_per_insert": round(B * args.steps / max(r_paced * t_paced, 1e-9), 2),
        },
    }
    print(json.dumps(out))


def setup_d4pg(args, world, rank, dev):
    from acme_amd import replay, specs
    from acme_amd.adders import reverb as adders
    from acme_amd.agents.d4pg import D4PGLearner
    from acme_amd.datasets import make_reverb_dataset
    from acme_amd.networks import make_d4pg_networks
    from acme_amd.utils import counting, loggers
    if world > 1:
        raise SystemExit("the D4PG workload is single-GPU (BASELINE configs[2])")
    B = args.batch or 256
    env_spec = specs.EnvironmentSpec(
        observations=specs.Array((24,), np.float32),
        actions=specs.BoundedArray((6,), np.float32, -1.0, 1.0),
        rewards=specs.Array((), np.float32), discounts=specs.BoundedArray((), np.float32, 0, 1))
    table = replay.Table(adders.DEFAULT_PRIORITY_TABLE, replay.selectors.Uniform(),
                         replay.selectors.Fifo(), args.replay_size,
                         replay.rate_limiters.MinSize(1),
                         signature=adders.NStepTransitionAdder.signature(env_spec), seed=4321,
                         device=dev)
    table.native.fill_synthetic(args.replay_size, layout=1, num_actions=1, seed=rank)
    server = replay.Server([table])
    nets = make_d4pg_networks(24, env_spec.actions)
    learner = D4PGLearner(nets["policy"], nets["critic"], nets["policy"], nets["critic"],
                          discount=0.99, target_update_period=100,
                          dataset=make_reverb_dataset(server, batch_size=B),
                          counter=counting.Counter(), logger=loggers.NoOpLogger(), device=dev)
    meta = dict(
        metric="learner transitions/sec (sample+step) at batch 256, D4PG control shape",
        dtype="f32",
        data="synthetic (device-generated 24-dim control-shape transitions, random-init "
             "D4PG networks)",
        config={"workload": "d4pg_control_uniform_replay (BASELINE configs[2])",
                "global_batch": B, "batch_per_gpu": B, "replay_slots": args.replay_size,
                "obs": "f32[24]", "act": "f32[6]", "atoms": 51,
                "policy": "LayerNormMLP(256,256,256)+tanh", "critic": "LayerNormMLP(512,512,256)+51",
                "sampler": "uniform", "parallelism": "dp1"})
    return (learner.step, B, meta, lambda: float(learner.native.critic_loss.item()),
            lambda: d4pg_cpu_baseline(B, args.cpu_baseline_seconds))


def impala_cpu_baseline(B: int, T: int, seconds: float):
    """The numpy IMPALA oracle (oracle/impala_oracle.py, float32) on a bounded sample: the
    same B x T Atari sequences, as many full learner steps as fit in `seconds` (at least 2;
    the first is a warm-up)."""
    from oracle import impala_oracle as O
    from acme_amd.networks import IMPALAAtariNetwork
    threads = len(os.sched_getaffinity(0))  # every visible host core
    try:
        from threadpoolctl import threadpool_limits
        ctx = threadpool_limits(threads)
    except ImportError:  # pragma: no cover
        ctx = None
    rng = np.random.default_rng(0)
    A, H = 18, 256
    batch = dict(obs=rng.integers(0, 256, (B, T, 84, 84, 4), dtype=np.uint8),
                 prev_action=rng.integers(0, A, (B, T)).astype(np.int32),
                 prev_reward=rng.standard_normal((B, T)).astype(np.float32),
                 action=rng.integers(0, A, (B, T)).astype(np.int32),
                 reward=rng.standard_normal((B, T)).astype(np.float32),
                 discount=np.full((B, T), 0.99, np.float32),
                 behaviour_logits=rng.standard_normal((B, T, A)).astype(np.float32),
                 h0=np.zeros((B, H), np.float32), c0=np.zeros((B, H), np.float32))
    cfg = O.IMPALAConfig(num_actions=A)
    p = IMPALAAtariNetwork(A).init(0)
    z = {k: np.zeros_like(v) for k, v in p.items()}
    state = dict(params=p, m=z, v=dict(z), num_steps=0)
    state = O.impala_step(cfg, state, batch, np.float32)[2]
    t0 = time.perf_counter()
    n = 0
    while n < 2 or time.perf_counter() - t0 < seconds:
        state = O.impala_step(cfg, state, batch, np.float32)[2]
        n += 1
    dt = time.perf_counter() - t0
    if ctx is not None and hasattr(ctx, "unregister"):
        ctx.unregister()
    return dict(value=round(B * T * n / dt, 2), unit="frames/s", cores=threads, kind="port",
                sample=(f"numpy float32 oracle (oracle/impala_oracle.py), {n} timed steps of "
                        f"B={B} x T={T} Atari sequences, {threads} BLAS threads, {cpu_model()}"))


def setup_impala(args, world, rank, dev):
    """BASELINE configs[3]: IMPALAAtariNetwork (LSTM 256, 18 actions), batch 16 sequences
    of T = 20 frames.  The queue is a device-resident pool of 4 batches of synthetic
    sequences (what 64 actors would have enqueued); each step consumes the next batch."""
    from acme_amd.native import NativeIMPALA
    from acme_amd.networks import IMPALAAtariNetwork
    if world > 1:
        raise SystemExit("the IMPALA workload is single-GPU (BASELINE configs[3])")
    B, T, A, H = args.batch or 16, 20, 18, 256
    pool = 4
    g = torch.Generator(device=dev).manual_seed(rank)
    obs = torch.randint(0, 256, (pool, B, T, 84, 84, 4), dtype=torch.uint8, device=dev, generator=g)
    ia = lambda: torch.randint(0, A, (pool, B, T), dtype=torch.int32, device=dev, generator=g)  # noqa
    fl = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa
    prev_a, act = ia(), ia()
    prev_r, rew = fl(pool, B, T), fl(pool, B, T)
    disc = torch.where(torch.rand(pool, B, T, device=dev, generator=g) < 0.01, 0.0, 0.99)
    mu = fl(pool, B, T, A)
    state = 0.1 * fl(pool, B, T, 2, H)
    net = IMPALAAtariNetwork(A)
    n = NativeIMPALA(num_actions=A, max_batch=B, max_sequence_length=T, lstm_size=H,
                     head_size=256, entropy_cost=0.01, baseline_cost=0.5, learning_rate=1e-3,
                     device=dev)
    n.set_params(net.init(0))
    it = [0]

    def step():
        i = it[0] % pool
        it[0] += 1
        n.step(obs[i], prev_a[i], prev_r[i], act[i], rew[i], disc[i], mu[i], state[i][:, 0, 0],
               state[i][:, 0, 1])

    meta = dict(
        metric="learner frames/sec (B=16 sequences x T=20) IMPALA Atari, 1 MI355X",
        unit="frames/s", dtype="f32 (torso and W_i: 2xf16 split planes, 3 MFMA terms)",
        # The one-launch LSTM unroll is a sequential latency chain, not an MFMA roofline: it
        # is reported per timestep against a kernel boundary (below), and the roofline
        # object names the dominant MFMA kernel among the others.
        _roofline_exclude=("impala_lstm_fwd", "impala_lstm_bwd"), _lstm_T=T,
        data="synthetic (device-generated uint8 Atari sequences in a device-resident queue "
             "pool, random-init IMPALAAtariNetwork)",
        config={"workload": "impala_atari_lstm_vtrace (BASELINE configs[3])",
                "batch_sequences": B, "sequence_length": T, "frames_per_step": B * T,
                "obs": "uint8[84,84,4]", "num_actions": A, "lstm": H, "parallelism": "dp1"})
    return (step, B * T, meta, lambda: float(n.metrics[0].item()),
            lambda: impala_cpu_baseline(B, T, args.cpu_baseline_seconds))


def r2d2_cpu_baseline(B: int, T: int, burn_in: int, seconds: float):
    """The numpy R2D2 oracle (oracle/r2d2_oracle.py, float32) on a bounded sample: B
    sequences of the workload's T = burn-in + trace + 1 Atari frames, as many full learner
    steps as fit in `seconds` (at least 2; the first is a warm-up)."""
    from oracle import r2d2_oracle as O
    threads = len(os.sched_getaffinity(0))  # every visible host core
    try:
        from threadpoolctl import threadpool_limits
        ctx = threadpool_limits(threads)
    except ImportError:  # pragma: no cover
        ctx = None
    rng = np.random.default_rng(0)
    A, H = 18, 512
    batch = dict(obs=rng.integers(0, 256, (B, T, 84, 84, 4), dtype=np.uint8),
                 prev_action=rng.integers(0, A, (B, T)).astype(np.int32),
                 prev_reward=rng.standard_normal((B, T)).astype(np.float32),
                 action=rng.integers(0, A, (B, T)).astype(np.int32),
                 reward=rng.standard_normal((B, T)).astype(np.float32),
                 discount=np.full((B, T), 1.0, np.float32),
                 h0=np.zeros((B, H), np.float32), c0=np.zeros((B, H), np.float32),
                 probabilities=np.full(B, 1e-4))
    cfg = O.R2D2Config(num_actions=A, burn_in_length=burn_in)
    from acme_amd.networks import R2D2AtariNetwork
    p = R2D2AtariNetwork(A).init(0)
    z = {k: np.zeros_like(v) for k, v in p.items()}
    state = dict(params=p, target=dict(p), m=z, v=dict(z), num_steps=0)
    state = O.r2d2_step(cfg, state, batch, np.float32)[2]
    t0 = time.perf_counter()
    n = 0
    while n < 2 or time.perf_counter() - t0 < seconds:
        state = O.r2d2_step(cfg, state, batch, np.float32)[2]
        n += 1
    dt = time.perf_counter() - t0
    if ctx is not None and hasattr(ctx, "unregister"):
        ctx.unregister()
    return dict(value=round(B * n / dt, 3), unit="sequences/s", cores=threads, kind="port",
                sample=(f"numpy float32 oracle (oracle/r2d2_oracle.py), {n} timed steps of "
                        f"B={B} x T={T} Atari sequences (burn-in {burn_in}), {threads} BLAS "
                        f"threads, {cpu_model()}"))


def setup_r2d2(args, world, rank, dev):
    """R2D2 widening: R2D2AtariNetwork (LSTM 512, duelling [512], 18
    actions), batch 32 sequences (the agent's default, agents/tf/r2d2/agent.py:55) of
    burn-in 40 + trace 80 + 1 = 121 frames (the R2D2 paper's Atari setting), n = 5.
    Synthetic sequences from a device-resident pool of 2 batches; each step consumes the
    next one and writes its priorities to a device buffer."""
    from acme_amd.native import NativeR2D2
    from acme_amd.networks import R2D2AtariNetwork
    if world > 1:
        raise SystemExit("the R2D2 workload is single-GPU")
    B, BI, TR, A, H = args.batch or 32, 40, 80, 18, 512
    T = BI + TR + 1
    pool = 2
    g = torch.Generator(device=dev).manual_seed(rank)
    obs = torch.randint(0, 256, (pool, B, T, 84, 84, 4), dtype=torch.uint8, device=dev, generator=g)
    ia = lambda: torch.randint(0, A, (pool, B, T), dtype=torch.int32, device=dev, generator=g)  # noqa
    fl = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa
    prev_a, act = ia(), ia()
    prev_r, rew = fl(pool, B, T), fl(pool, B, T)
    disc = torch.where(torch.rand(pool, B, T, device=dev, generator=g) < 0.01, 0.0, 1.0)
    state = 0.1 * fl(pool, B, T, 2, H)
    probs = (torch.rand(pool, B, device=dev, generator=g, dtype=torch.float64) + 0.5) * 1e-5
    net = R2D2AtariNetwork(A)
    n = NativeR2D2(num_actions=A, max_batch=B, max_sequence_length=T, burn_in_length=BI,
                   device=dev)
    n.set_params(net.init(0), net.init(1))
    it = [0]

    def step():
        i = it[0] % pool
        it[0] += 1
        n.step(obs[i], prev_a[i], prev_r[i], act[i], rew[i], disc[i], probs[i],
               state[i][:, 0, 0], state[i][:, 0, 1])

    meta = dict(
        metric=f"learner sequences/sec (B={B} x T={T}, burn-in {BI}) R2D2 Atari, 1 MI355X",
        unit="sequences/s",
        dtype="f32 (torso and W_i: 2xf16 split planes, 3 MFMA terms; LSTM: f32 one-launch unroll; head: f32 MFMA)",
        _roofline_exclude=("r2d2_lstm_fwd", "r2d2_lstm_bwd"),
        _lstm_T={"r2d2_lstm_fwd": T, "r2d2_lstm_bwd": T - BI},
        data="synthetic (device-generated uint8 Atari sequences in a device-resident pool, "
             "random-init R2D2AtariNetwork)",
        config={"workload": "r2d2_atari_lstm_transformed_nstep (SURVEY §8(f) widening)",
                "batch_sequences": B, "sequence_length": T, "burn_in": BI, "n_step": 5,
                "frames_per_step": B * T, "obs": "uint8[84,84,4]", "num_actions": A,
                "lstm": H, "parallelism": "dp1"})
    return (step, B, meta, lambda: float(n.loss[0].item()),
            lambda: r2d2_cpu_baseline(2, T, BI, args.cpu_baseline_seconds))


IMPALA_T, IMPALA_A, IMPALA_H = 20, 18, 256


def impala_actor_signature():
    """The configs[3] queue signature (CPU only: the actor processes need it before the
    parent touches the GPU)."""
    from acme_amd import specs
    from acme_amd.adders import reverb as adders
    from acme_amd.environments.atari_like import AtariLike
    from acme_amd.networks import LSTMState
    from acme_amd.wrappers import ObservationActionRewardWrapper
    spec = specs.make_environment_spec(ObservationActionRewardWrapper(AtariLike(seed=0)))
    H, A = IMPALA_H, IMPALA_A
    extra = {"core_state": LSTMState(specs.Array((H,), np.float32), specs.Array((H,), np.float32)),
             "logits": specs.Array((A,), np.float32)}
    return spec, adders.SequenceAdder.signature(spec, extras_spec=extra)


def start_actor_processes(args):
    """ProcessActorPool for impala_actors, started before anything touches the GPU."""
    from acme_amd.agents.impala.process_actors import (ProcessActorPool, atari_like_oar,
                                                       sequence_fields)
    from acme_amd.networks import IMPALAAtariNetwork
    _, sig = impala_actor_signature()
    net = IMPALAAtariNetwork(IMPALA_A)
    pool = ProcessActorPool(atari_like_oar, sequence_fields(sig, IMPALA_T), (84, 84, 4),
                            IMPALA_A, IMPALA_H, net.initial_state, num_actors=args.actors,
                            processes=args.actor_procs, groups=args.actor_groups,
                            sequence_length=IMPALA_T,
                            period=IMPALA_T)
    pool.start()
    return pool


def impala_actors_bench(args, dev, pool=None):
    """BASELINE configs[3] end to end: `--actors` host threads, each an Atari-shaped
    environment (acme_amd.environments.AtariLike), an IMPALAActor and a SequenceAdder
    (T = 20, period 20) writing into the device queue table; their policy calls are batched
    into GPU network steps on the learner's current parameters (agents/impala/actors.py);
    the learner (B = 16 sequences) steps whenever the queue holds a batch
    (agents/tf/impala/agent.py:117-120).  Reports learned frames/s (B x T per learner step)
    over `--steps` learner steps after `--warmup`, and the actors' environment steps/s."""
    from acme_amd import replay, specs
    from acme_amd.adders import reverb as adders
    from acme_amd.agents.impala import IMPALALearner
    from acme_amd.agents.impala.actors import ActorPool, BatchedPolicy, VectorActorPool
    from acme_amd.datasets import make_reverb_dataset
    from acme_amd.environments.atari_like import AtariLike
    from acme_amd.networks import IMPALAAtariNetwork, LSTMState
    from acme_amd.utils import loggers
    from acme_amd.wrappers import ObservationActionRewardWrapper
    B, T, A, H = args.batch or 16, 20, 18, 256
    env0 = ObservationActionRewardWrapper(AtariLike(seed=0))
    spec = specs.make_environment_spec(env0)
    extra = {"core_state": LSTMState(specs.Array((H,), np.float32), specs.Array((H,), np.float32)),
             "logits": specs.Array((A,), np.float32)}
    queue = replay.Table.queue(adders.DEFAULT_PRIORITY_TABLE, max_size=4 * B * 8,
                               signature=adders.SequenceAdder.signature(spec, extras_spec=extra),
                               device=dev)
    server = replay.Server([queue])
    net = IMPALAAtariNetwork(A)
    learner = IMPALALearner(spec, net, make_reverb_dataset(server, batch_size=B,
                                                           sequence_length=T),
                            learning_rate=1e-3, entropy_cost=0.01, baseline_cost=0.5,
                            logger=loggers.NoOpLogger(), batch_size=B, sequence_length=T,
                            device=dev)
    make_env = lambda i: ObservationActionRewardWrapper(AtariLike(seed=1 + i))  # noqa: E731
    make_adder = lambda i: adders.SequenceAdder(replay.Client(server), sequence_length=T,  # noqa: E731
                                                period=T)
    # The environment's own cost per step (what an actor pays before any policy or adder).
    e, t0 = make_env(999), time.perf_counter()
    e.reset()
    for k in range(2000):
        ts = e.step(np.int32(k % A))
        if ts.last():
            e.reset()
    env_us = 1e6 * (time.perf_counter() - t0) / 2000
    if pool is not None:
        return impala_process_actors(args, dev, pool, queue, learner, B, T, A, H, env_us)
    if args.actor_threads > 0:  # K environments per host thread, one policy call per K steps
        th = args.actor_threads
        per = min(-(-args.actors // th), 16)  # the native policy's batch limit (LDS) at LSTM 256
        policy = None
        pool = VectorActorPool(make_env, make_adder, lambda t: learner.actor_policy(max_rows=per),
                               net.initial_state, num_actors=args.actors, threads=th,
                               max_rows=per)
    else:  # one host thread per actor (IMPALAActor), policy calls batched by a server thread
        policy = BatchedPolicy(learner.actor_policy(max_rows=16), max_rows=16)
        pool = ActorPool(make_env, make_adder, policy, net.initial_state, num_actors=args.actors)
    pool.start()
    try:
        def learn(n):
            done = 0
            while done < n:
                if pool.errors:
                    raise pool.errors[0]
                if queue.can_sample(B):
                    learner.step()
                    done += 1
                else:
                    time.sleep(0.0005)
        learn(args.warmup)
        torch.cuda.synchronize(dev)
        s0, t0 = pool.env_steps, time.perf_counter()
        learn(args.steps)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        env_rate = (pool.env_steps - s0) / dt
    finally:
        pool.stop(timeout=5)
        if policy is not None:
            policy.close()
    out = {
        "metric": "IMPALA learned frames/sec (B=16 x T=20 per step) with host actors feeding "
                  "the device queue, 1 MI355X",
        "value": round(B * T * args.steps / dt, 1), "unit": "frames/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic Atari-shaped environment (acme_amd.environments.AtariLike), "
                "random-init IMPALAAtariNetwork",
        "config": {"workload": "impala_actor_learner (BASELINE configs[3])", "actors": args.actors,
                   "batch_sequences": B, "sequence_length": T, "sequence_period": T,
                   "obs": "uint8[84,84,4]", "num_actions": A, "lstm": H},
        "actors": {"env_steps_per_s": round(env_rate, 1), "env_us_per_step": round(env_us, 2),
                   "host_threads": args.actor_threads if policy is None else args.actors,
                   "policy_batches": policy.batches if policy else None,
                   "mean_policy_rows": (round(policy.rows / max(policy.batches, 1), 2)
                                        if policy else min(-(-args.actors // args.actor_threads),
                                                           16))},
    }
    print(json.dumps(out))


def impala_process_actors(args, dev, pool, queue, learner, B, T, A, H, env_us):
    """impala_actors with the environments and adders in worker processes (ProcessActorPool):
    a driver thread of this process runs the batched policy over one group of environments
    while the workers step the other, and hands the workers' finished sequences to the
    device queue in native inserts; the learner steps on this thread whenever the queue
    holds a batch."""
    import threading
    queue.set_sequence_length(T)
    fields = [(f.shape, f.dtype, f.nbytes, f.row_bytes) for f in queue.fields]
    if fields != pool._fields:  # noqa: SLF001
        raise RuntimeError("actor rings and the queue table disagree on the item layout")
    G = args.actor_groups
    rows = args.actors // G
    policy = [learner.pipelined_policy(rows) for _ in range(G)]  # one per group
    pool.register_pinned()
    stop, errors = threading.Event(), []

    def drive():
        try:
            pool.run(policy, queue.insert_rows, ticks=1 << 40, should_stop=stop.is_set)
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    th = threading.Thread(target=drive, daemon=True)
    th.start()
    try:
        def learn(n):
            done = 0
            while done < n:
                if errors:
                    raise errors[0]
                if queue.can_sample(B):
                    learner.step()
                    done += 1
                else:
                    time.sleep(0.0002)
        learn(args.warmup)
        torch.cuda.synchronize(dev)
        s0, t0 = pool.env_steps, time.perf_counter()
        learn(args.steps)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        env_rate = (pool.env_steps - s0) / dt
    finally:
        stop.set()
        th.join(60)
        pool.close()
    out = {
        "metric": "IMPALA learned frames/sec (B=16 x T=20 per step) with host actors feeding "
                  "the device queue, 1 MI355X",
        "value": round(B * T * args.steps / dt, 1), "unit": "frames/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic Atari-shaped environment (acme_amd.environments.AtariLike), "
                "random-init IMPALAAtariNetwork",
        "config": {"workload": "impala_actor_learner (BASELINE configs[3])", "actors": args.actors,
                   "batch_sequences": B, "sequence_length": T, "sequence_period": T,
                   "obs": "uint8[84,84,4]", "num_actions": A, "lstm": H},
        "actors": {"env_steps_per_s": round(env_rate, 1), "env_us_per_step": round(env_us, 2),
                   "actor_processes": args.actor_procs, "policy_rows": rows, "groups": G,
                   "items_inserted": pool.items,
                   "driver_us_per_act": {k[:-2]: round(1e6 * v / max(pool.stats["acts"], 1), 1)
                                         for k, v in pool.stats.items() if k.endswith("_s")}},
    }
    print(json.dumps(out))


def merge_launch_sections(sections, name, other, labels):
    """One record for a kernel profiled as two sections (the DQN fc_fwd: the online launch,
    256 blocks over the whole chip, and the target launch, 128 blocks by design, DESIGN.md
    4.1): summed time and FLOPs under `name`, each launch kept under "per_launch"."""
    a = next((r for r in sections if r["name"] == name), None)
    b = next((r for r in sections if r["name"] == other), None)
    if a is None or b is None or a.get("bound") != "mfma" or b.get("bound") != "mfma":
        return
    parts = []
    for lab, r in zip(labels, (a, b)):
        parts.append(dict(launch=lab, launches=r["launches"], avg_us=r["avg_us"],
                          achieved=r["achieved"], frac=r["frac"]))
    fl = sum(r["achieved"] * 1e12 * r["avg_us"] * 1e-6 * r["launches"] for r in (a, b))
    ms = a["total_ms"] + b["total_ms"]
    n = a["launches"] + b["launches"]
    tf = fl / (ms * 1e-3) / 1e12
    a.update(launches=n, avg_us=round(1e3 * ms / n, 2), total_ms=round(ms, 3),
             achieved=round(tf, 2), frac=round(tf / a["peak"], 4), per_launch=parts)
    sections.remove(b)


def pmc_traffic(workload: str, section: str):
    """HBM bytes per launch of `section` from the newest committed PMC summary
    (profiles/<round>/pmc_traffic_<workload>.json, written by tools/pmc_traffic.py from
    separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench); (None, source) when the
    newest summary does not hold the section (an older round's bytes would describe an older
    kernel), (None, None) without a summary."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"pmc_traffic_{workload}.json")))
    if not paths:
        return None, None
    path = paths[-1]
    try:
        with open(path) as f:
            k = json.load(f)["kernels"].get(section)
    except (OSError, ValueError, KeyError):
        k = None
    return (int(k["bytes"]) if k else None), os.path.relpath(path, ROOT)


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` run without a launcher: start N ranks with torch.distributed.run
    (one process per GPU, rendezvous on 127.0.0.1) as a child process, before this process
    touches the GPU, and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        if "WORLD_SIZE" not in os.environ and args.gpus > 1:
            sys.exit(spawn_ranks(args.gpus))
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    pool = None
    if args.workload == "impala_actors" and args.actor_procs > 0 and world == 1:
        pool = start_actor_processes(args)  # before this process touches the GPU
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # One rank per GPU.  More ranks than visible GPUs (a rehearsal on a one-GPU box) share
    # devices round-robin; ACME_DIST_BACKEND=gloo selects gloo for such a rehearsal, since
    # RCCL rejects two ranks on one device.  The driver's runs use RCCL ("nccl").
    ngpu = torch.cuda.device_count()
    local = local % max(ngpu, 1)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        backend = os.environ.get("ACME_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        dist = None
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from acme_amd import _lib
    L = _lib.lib()
    if args.workload in ("insert", "impala_actors"):
        if world > 1:
            raise SystemExit(f"the {args.workload} workload is single-GPU")
        if args.workload == "insert":
            insert_bench(args, dev)
        else:
            impala_actors_bench(args, dev, pool)
        return
    t_fill = time.perf_counter()
    setup = {"dqn": setup_dqn, "d4pg": setup_d4pg, "impala": setup_impala,
             "r2d2": setup_r2d2}[args.workload]
    step, B, meta, loss_fn, cpu_fn = setup(args, world, rank, dev)
    torch.cuda.synchronize(dev)
    t_fill = time.perf_counter() - t_fill

    gc.collect()  # before the warm-up: no host pause between the settling steps and the window
    tw = time.perf_counter()
    for i in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # Settling: a short warm-up (the driver's default is 5 steps, ~3 ms) leaves the first
    # timed steps on ramping clocks (20 steps after 5 warm-up steps measured 0.577 ms against
    # 0.542 ms over 100 steps after 20).  Untimed steps continue until --settle-seconds of
    # warm-up have passed; the count is the same on every rank (from the slowest rank's warm-up
    # rate), since every step issues collectives.
    settle = 0
    if args.settle_seconds > 0 and args.steps > 0:
        spent = time.perf_counter() - tw
        per = spent / max(args.warmup, 1)
        if world > 1:
            t = torch.tensor([spent, per], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            spent, per = float(t[0].item()), float(t[1].item())
        if spent < args.settle_seconds:
            settle = min(int((args.settle_seconds - spent) / max(per, 1e-4)) + 1, 5000)
        for i in range(settle):
            step()
        torch.cuda.synchronize(dev)
    # The host issues a step in about half the GPU's step time, so a host pause early in a
    # short timed window (the driver times 20 steps) stalls the GPU directly: Python's cyclic
    # garbage collector ran before the warm-up (a collection right before the window
    # idled the GPU long enough to drop its clocks: 20 timed steps 0.53 -> 0.58 ms) and is
    # paused inside the window (nothing is skipped; the steps make no cyclic garbage).
    g0 = meta["_guard"]() if "_guard" in meta else None
    gc.disable()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    # The step guard over the timed window: updates applied, steps the
    # device skipped (plane overflow) and steps the learner re-issued; a skipped-and-re-issued
    # step inside the window costs time the line would otherwise hide.  Read after the window
    # (the re-issue of a step skipped in its last two calls happens when the learner settles).
    guard = None
    if g0 is not None:
        g1 = meta["_guard"]()
        guard = {k: g1[k] - g0[k] for k in g1}
        guard["window_steps"] = args.steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # The N = 1 point of a scaling curve: a data-parallel rank runs the learner's stages with
    # the collectives between them (DQNLearner._staged_step); the same stages on one GPU with
    # the collectives left out, timed like the line above (separately, after it).
    staged_ms = None
    if "_set_staged" in meta and world == 1 and args.steps > 0 and not args.no_staged:
        meta["_set_staged"](True)
        for i in range(min(args.warmup, 10)):
            step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        staged_ms = 1e3 * (time.perf_counter() - t0) / args.steps
        meta["_set_staged"](False)
    # Per-kernel durations come from a separate pass with the in-library section profiler
    # (HIP event pairs on the launch stream), so its event records stay out of the timed
    # region above.
    if not args.no_profile and args.profile_steps > 0:
        torch.cuda.synchronize(dev)  # prefetched batches land before profiling starts
        L.acme_profile_reset()
        _lib.set_profiling(True)
        for i in range(args.profile_steps):
            step()
        torch.cuda.synchronize(dev)
        _lib.set_profiling(False)
    loss = loss_fn()

    sections = []
    for i in range(L.acme_profile_num_sections()):
        import ctypes
        nm, ms, cnt = ctypes.c_char_p(), ctypes.c_double(), ctypes.c_int64()
        fl, by = ctypes.c_double(), ctypes.c_double()
        _lib.check(L.acme_profile_query(i, ctypes.byref(nm), ctypes.byref(ms), ctypes.byref(cnt),
                                        ctypes.byref(fl), ctypes.byref(by)))
        if cnt.value == 0:
            continue
        avg_ms = ms.value / cnt.value
        rec = dict(name=nm.value.decode(), launches=int(cnt.value), avg_us=round(1e3 * avg_ms, 2),
                   total_ms=round(ms.value, 3))
        if fl.value > 0:
            # Peak of the arithmetic path the section ran on (f32 MFMA, or the exact
            # f16-plane engine at the f16 dense peak / MFMA terms per product).
            pk = ctypes.c_double()
            _lib.check(L.acme_profile_query_peak(i, ctypes.byref(pk)))
            peak = pk.value if pk.value > 0 else FP32_MFMA_PEAK_TFLOPS
            tf = fl.value / cnt.value / (avg_ms * 1e-3) / 1e12
            rec.update(bound="mfma", achieved=round(tf, 2), unit="TFLOP/s", peak=round(peak, 1),
                       frac=round(tf / peak, 4))
        elif by.value > 0:
            gbs = by.value / cnt.value / (avg_ms * 1e-3) / 1e9
            rec.update(bound="hbm", achieved=round(gbs, 1), unit="GB/s",
                       frac=round(gbs / HBM_PEAK_GBS, 4))
            if rec["name"] == "adam" and "_adam_survey_bytes" in meta:
                sb = meta["_adam_survey_bytes"]
                rec.update(design_bytes=round(by.value / cnt.value), survey_bytes=round(sb),
                           frac_survey_bytes=round(sb / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
        sections.append(rec)
    merge_launch_sections(sections, "fc_fwd", "fc_fwd_target", ("online", "target"))
    sections.sort(key=lambda r: -r["total_ms"])
    # Sum of the profiled kernel durations per step: ms_per_step minus this is launch gaps
    # and host time the GPU waited on.
    busy = (sum(r["total_ms"] for r in sections) / args.profile_steps
            if sections and args.profile_steps > 0 else None)

    ms_per_step = 1e3 * elapsed / args.steps
    value = world * B * args.steps / elapsed
    roofline = None
    mfma = [s for s in sections if s.get("bound") == "mfma"
            and s["name"] not in meta.get("_roofline_exclude", ())]
    if mfma:
        dom = mfma[0]
        traffic, src = pmc_traffic(args.workload, dom["name"])
        roofline = dict(bound="mfma", kernel=dom["name"], achieved=dom["achieved"],
                        peak=dom["peak"], unit="TFLOP/s", frac=dom["frac"],
                        traffic=traffic, traffic_unit="bytes/launch", traffic_source=src,
                        avg_us=dom["avg_us"])
        if "per_launch" in dom:
            roofline["per_launch"] = dom["per_launch"]
    if rank == 0:
        for s in sections:
            print(f"[bench] {s['name']:16s} {s['launches']:6d} x {s['avg_us']:9.2f} us  "
                  f"{s.get('achieved', '')} {s.get('unit', '')} (peak {s.get('peak', '-')}) "
                  f"frac={s.get('frac', '')}",
                  file=sys.stderr)
        print(f"[bench] replay fill {t_fill:.1f}s, final loss {loss:.5f}", file=sys.stderr)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_fn()
    if rank == 0:
        out = {
            "metric": meta["metric"], "value": round(value, 1),
            "unit": meta.get("unit", "transitions/s"),
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "settle_steps": settle,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": meta["dtype"], "data": meta["data"],
            "config": meta["config"],
            "roofline": roofline,
            "cpu_baseline": cpu,
            "gpu_busy_ms_per_step": None if busy is None else round(busy, 4),
            "dp_staged_ms_per_step": None if staged_ms is None else round(staged_ms, 4),
            "kernels": sections,
        }
        if guard is not None:
            out["step_guard"] = guard
        if "_lstm_T" in meta:
            # The LSTM unroll per timestep (one launch each way) against a dependent kernel
            # boundary on MI355X (1.45 us between trivial kernels, MI355X_MICROARCH.md
            # "boundary"), the floor of one launch per timestep before any work.
            # (R2D2: the BPTT launch covers the T - burn-in trained steps.)
            lstm = {s["name"]: s for s in sections if s["name"] in meta["_roofline_exclude"]}
            T = meta["_lstm_T"]
            steps_of = (lambda k: T[k]) if isinstance(T, dict) else (lambda k: T)
            out["lstm"] = {k.replace("impala_", "").replace("r2d2_", ""): {
                "us_per_launch": v["avg_us"], "timesteps": steps_of(k),
                "us_per_timestep": round(v["avg_us"] / steps_of(k), 3)} for k, v in lstm.items()}
            out["lstm"]["boundary_us"] = 1.45
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
