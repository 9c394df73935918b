"""Actor processes for BASELINE configs[3] (64 CPU actors feeding one GPU IMPALA learner).

The reference runs every actor as its own program (acme/agents/tf/impala/acting.py:32-95:
environment, TF policy, SequenceAdder writing into the Reverb queue; agent.py:111-120 steps
the learner while the queue holds a batch).  Python threads in one process cap that at a
few tens of thousands of environment steps per second (the GIL: every environment step and
adder call is Python).  Here:

- `processes` worker processes own the environments and their SequenceAdders.  They never
  touch the GPU and are started (spawn) before anything in the parent does, so no process
  that initialised the GPU forks or execs.
- The policy runs in the learner's process, batched: one network step per group of
  environments on the GPU (the learner's parameter snapshot), actions sampled there.
- Environments are split into `groups` (default 2): while the workers step one group's
  environments with the actions just posted, the parent runs the policy for the other group,
  so policy latency and environment time overlap.
- Observations, actions and the adders' extras (the step's logits, the LSTM state before
  it) travel through shared memory; the workers' adders write finished sequence items
  straight into per-worker shared-memory rings laid out as the queue table's rows (field-
  major, row padding zero), and the parent hands each drained range to the table in one
  native insert (`QueueTable.insert_rows`).
- Hand-offs are counters in shared memory polled with short sleeps (a pipe round trip costs
  more than a tick's budget).

Per environment the behaviour is IMPALAActor's with a SequenceAdder (`tests/
test_process_actors_cpu.py` compares the items with the reference actor's): the state reset
at episode starts (the policy is called with the initial state), a ~ Categorical(logits of
the step), extras {'logits', 'core_state'} of the step.
"""

from __future__ import annotations

import multiprocessing as mp
import time
from multiprocessing import shared_memory
from typing import Callable, List, Optional, Sequence

import numpy as np

from acme_amd.networks import LSTMState

_SLEEP = 0.0  # polls yield the CPU without sleeping: a timed sleep costs ~60 us on Linux


def _views(shm, specs):
    """Numpy views of one shared-memory block: specs = [(name, shape, dtype)]."""
    out, off = {}, 0
    for name, shape, dt in specs:
        dt = np.dtype(dt)
        n = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
        out[name] = np.ndarray(shape, dt, buffer=shm.buf, offset=off)
        off += (n + 63) // 64 * 64
    return out


def _nbytes(specs):
    return sum((int(np.prod(s, dtype=np.int64)) * np.dtype(d).itemsize + 63) // 64 * 64
               for _, s, d in specs)


def _state_specs(N, obs_shape, A, H, P, G):
    return [("obs", (N,) + tuple(obs_shape), np.uint8), ("prev_a", (N,), np.int32),
            ("prev_r", (N,), np.float32), ("first", (N,), np.uint8),
            ("action", (N,), np.int32), ("logits", (N, A), np.float32),
            ("core_h", (N, H), np.float32), ("core_c", (N, H), np.float32),
            ("go", (P, G), np.int64), ("done", (P, G), np.int64), ("steps", (P,), np.int64),
            ("stop", (1,), np.int64), ("error", (P,), np.int64)]


def _ring_specs(fields, M):
    return [(f"f{i}", (M, rb), np.uint8) for i, (_, _, _, rb) in enumerate(fields)] + \
           [("head", (1,), np.int64), ("tail", (1,), np.int64)]


class _RingTable:
    """The worker-side table: T-step items packed into a shared-memory ring, one step's
    leaves at a time (typed views of the ring rows: no stacking, one copy per leaf)."""

    def __init__(self, ring, fields, M, stop):
        self._ring, self._fields, self._M, self._stop = ring, fields, M, stop
        self._typed = [ring[f"f{i}"][:, :nb].view(dt).reshape((M,) + shape)
                       for i, (shape, dt, nb, _) in enumerate(fields)]
        self._checked = False

    def insert_steps(self, steps) -> None:
        """steps: the item's T steps, each its flattened leaves."""
        head, tail = self._ring["head"], self._ring["tail"]
        while head[0] - tail[0] >= self._M:  # full: the parent drains every tick
            if self._stop[0]:
                raise SystemExit
            time.sleep(_SLEEP)
        if not self._checked:  # the layout, once per writer process
            for leaves in steps:
                if len(leaves) != len(self._fields):
                    raise ValueError(f"step has {len(leaves)} leaves, ring expects "
                                     f"{len(self._fields)}")
                for i, (leaf, (shape, _, _, _)) in enumerate(zip(leaves, self._fields)):
                    if np.shape(leaf) != shape[1:] or len(steps) != shape[0]:
                        raise ValueError(f"leaf {i}: step shape {np.shape(leaf)} x "
                                         f"{len(steps)}, ring expects {shape}")
            self._checked = True
        slot = int(head[0] % self._M)
        for t, leaves in enumerate(steps):
            for typed, leaf in zip(self._typed, leaves):
                typed[slot, t] = leaf
        head[0] += 1  # publish (the parent reads head after the rows are written)


class _RingWriter:
    """Reverb Writer surface over the ring: append(step) keeps the step's flattened leaves,
    create_item(table, num_timesteps, priority) packs the last num_timesteps steps."""

    def __init__(self, table: _RingTable, max_sequence_length: int):
        import collections
        self._table = table
        self._hist = collections.deque(maxlen=max_sequence_length)

    def append(self, data) -> None:
        from acme_amd.utils import tree
        self._hist.append(tree.flatten(data))

    def create_item(self, table: str, num_timesteps: int, priority: float) -> None:
        if num_timesteps < 1 or num_timesteps > len(self._hist):
            raise ValueError(f"num_timesteps={num_timesteps} but only {len(self._hist)} "
                             "steps are available")
        self._table.insert_steps(list(self._hist)[len(self._hist) - num_timesteps:])

    def flush(self) -> None:
        pass

    def close(self) -> None:
        pass


class _RingClient:
    """The adders' client in a worker (uniform priorities: the queue ignores them)."""

    def __init__(self, table: _RingTable):
        self._table = table

    def writer(self, max_sequence_length: int, delta_encoded: bool = False,
               chunk_length: Optional[int] = None) -> _RingWriter:
        return _RingWriter(self._table, max_sequence_length)


def atari_like_oar(i: int, seed: int = 1, **kw):
    """Environment i of the harness: AtariLike (seed + i) under ObservationActionReward."""
    from acme_amd.environments.atari_like import AtariLike
    from acme_amd.wrappers import ObservationActionRewardWrapper
    return ObservationActionRewardWrapper(AtariLike(seed=seed + i, **kw))


def sequence_fields(signature, T: int):
    """The stored rows of T-step items of a per-timestep signature, as a Table fixes them
    at its first sequence item: [(shape, dtype, nbytes, row_bytes)] in leaf order."""
    from acme_amd.replay import _layout_from_signature, _row_bytes
    return [((T,) + f.shape, f.dtype, T * f.nbytes, _row_bytes(T * f.nbytes, f.dtype.itemsize))
            for f in _layout_from_signature(signature)]


def _attach(name):
    # Spawned children share the parent's resource tracker (a set of names), so attaching
    # registers nothing new; the parent unlinks the block in close().
    return shared_memory.SharedMemory(name=name)


def _worker(w, env_ids, env_factory, state_name, ring_name, meta):
    from acme_amd.adders import reverb as adders
    N, obs_shape, A, H, P, G, T, period, fields, M = meta
    st_shm = _attach(state_name)
    rg_shm = _attach(ring_name)
    S = _views(st_shm, _state_specs(N, obs_shape, A, H, P, G))
    R = _views(rg_shm, _ring_specs(fields, M))
    try:
        ring = _RingTable(R, fields, M, S["stop"])
        envs = {i: env_factory(i) for i in env_ids}
        adder = {i: adders.SequenceAdder(_RingClient(ring), sequence_length=T, period=period)
                 for i in env_ids}
        by_group = [[i for i in env_ids if i * G // N == g] for g in range(G)]

        def publish(i, ts):
            S["obs"][i] = ts.observation.observation
            S["prev_a"][i] = ts.observation.action
            S["prev_r"][i] = ts.observation.reward

        for i in env_ids:
            ts = envs[i].reset()
            adder[i].add_first(ts)
            publish(i, ts)
            S["first"][i] = 1
        S["done"][w, :] = 0  # every group's first observations are ready
        while True:
            for g in range(G):
                while S["go"][w, g] <= S["done"][w, g]:
                    if S["stop"][0]:
                        return
                    time.sleep(_SLEEP)
                for i in by_group[g]:
                    a = np.int32(S["action"][i])
                    nt = envs[i].step(a)
                    adder[i].add(a, nt, {"logits": S["logits"][i].copy(),
                                         "core_state": LSTMState(S["core_h"][i].copy(),
                                                                 S["core_c"][i].copy())})
                    first = 0
                    if nt.last():
                        nt = envs[i].reset()
                        adder[i].add_first(nt)
                        first = 1
                    publish(i, nt)
                    S["first"][i] = first
                S["steps"][w] += len(by_group[g])
                S["done"][w, g] += 1
    except SystemExit:
        pass
    except BaseException:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        S["error"][w] = 1
    finally:
        del S, R
        st_shm.close()
        rg_shm.close()


class ProcessActorPool:
    """`num_actors` environments (env_factory(i), picklable) in `processes` worker processes,
    each with a SequenceAdder (sequence_length T, period), policy batched in this process.

    policy_step(obs [n, ...] u8, prev_a [n], prev_r [n], h [n, H], c [n, H]) -> (logits, v,
    h, c) numpy, on at most num_actors / groups rows; sink(fields, n) receives drained items
    as per-field uint8 row arrays (e.g. QueueTable.insert_rows); `fields` describes the
    stored rows: [(shape, dtype, nbytes, row_bytes)] in the item's leaf order.

    start() spawns the workers: call it before the parent initialises the GPU.  run(n)
    steps every environment n times from the calling thread (a driver thread of the learner
    process, say); stop() ends the workers."""

    def __init__(self, env_factory: Callable, fields: Sequence, obs_shape, num_actions: int,
                 lstm_size: int, initial_state: Callable, num_actors: int = 64,
                 processes: int = 8, groups: int = 2, sequence_length: int = 20,
                 period: int = 20, ring_items: int = 16, seed: int = 0):
        N, P, G = int(num_actors), max(1, min(int(processes), int(num_actors))), int(groups)
        if N % G or (N // G) < 1:
            raise ValueError(f"num_actors {N} must split into {G} groups")
        self._N, self._P, self._G = N, P, G
        self._A, self._H = int(num_actions), int(lstm_size)
        self._fields = [(tuple(s), np.dtype(d), int(nb), int(rb)) for s, d, nb, rb in fields]
        self._M = int(ring_items)
        self._obs_shape = tuple(obs_shape)
        self._env_factory = env_factory
        self._meta = (N, self._obs_shape, self._A, self._H, P, G, int(sequence_length),
                      int(period), self._fields, self._M)
        ss = _state_specs(N, self._obs_shape, self._A, self._H, P, G)
        self._st_shm = shared_memory.SharedMemory(create=True, size=_nbytes(ss))
        self.S = _views(self._st_shm, ss)
        for v in self.S.values():
            v[...] = 0
        self.S["done"][...] = -1  # not ready
        rs = _ring_specs(self._fields, self._M)
        self._rg_shm = [shared_memory.SharedMemory(create=True, size=_nbytes(rs))
                        for _ in range(P)]
        self.R = [_views(s, rs) for s in self._rg_shm]
        for r in self.R:
            for v in r.values():
                v[...] = 0
        # Environment i belongs to group i * G // N (contiguous rows per group) and to worker
        # i % P (every worker steps a share of every group).
        self._groups = [np.arange(g * N // G, (g + 1) * N // G) for g in range(G)]
        self._env_ids = [[i for i in range(N) if i % P == w] for w in range(P)]
        s0 = initial_state(1)
        self._h0, self._c0 = np.asarray(s0.hidden[0], np.float32), np.asarray(s0.cell[0], np.float32)
        st = initial_state(N)
        self._h = np.array(st.hidden, np.float32)
        self._c = np.array(st.cell, np.float32)
        self._rng = np.random.default_rng(seed)
        self._procs: List[mp.Process] = []
        self._policy = None
        self._sink = None
        self.items = 0
        # Seconds of the driver thread spent in the policy, waiting for workers, draining.
        import threading
        self._drain_lock = threading.Lock()
        self.stats = {"wait_s": 0.0, "result_s": 0.0, "post_s": 0.0, "issue_s": 0.0,
                      "drain_s": 0.0, "acts": 0}

    # -- lifecycle
    def start(self) -> None:
        ctx = mp.get_context("spawn")
        self._procs = [ctx.Process(target=_worker, daemon=True,
                                   args=(w, self._env_ids[w], self._env_factory,
                                         self._st_shm.name, self._rg_shm[w].name, self._meta))
                       for w in range(self._P)]
        for p in self._procs:
            p.start()

    def stop(self, timeout: float = 10.0) -> None:
        self.S["stop"][0] = 1
        for p in self._procs:
            p.join(timeout)
            if p.is_alive():
                p.terminate()
        self._procs = []

    def register_pinned(self) -> None:
        """Page-locks the observation block (the policy's host-to-device copies then read it
        directly); call after the parent has initialised the GPU."""
        import ctypes
        from acme_amd._lib import check, lib
        if getattr(self, "_pinned", None):
            return
        obs = self.S["obs"]
        p = obs.ctypes.data
        check(lib().acme_host_register(ctypes.c_void_p(p), obs.nbytes), "host register")
        self._pinned = p

    def _unregister(self) -> None:
        p = getattr(self, "_pinned", None)
        if p:
            import ctypes
            from acme_amd._lib import lib
            lib().acme_host_unregister(ctypes.c_void_p(p))
            self._pinned = None

    @property
    def obs_pinned(self) -> bool:
        return bool(getattr(self, "_pinned", None))

    def close(self) -> None:
        if self._procs:
            self.stop()
        self._unregister()
        for s in [self._st_shm] + self._rg_shm:
            try:
                s.close()
                s.unlink()
            except FileNotFoundError:
                pass

    @property
    def env_steps(self) -> int:
        return int(self.S["steps"].sum())

    def _check(self) -> None:
        err = getattr(self, "_drain_error", None)
        if err is not None:  # the drain thread's failure, re-raised on the driver
            raise RuntimeError(f"the queue drain thread failed: {err!r}") from err
        if self.S["error"].any():
            raise RuntimeError(f"actor worker(s) {np.nonzero(self.S['error'])[0].tolist()} failed")
        for w, p in enumerate(self._procs):
            if not p.is_alive() and not self.S["stop"][0]:
                raise RuntimeError(f"actor worker {w} exited ({p.exitcode})")

    # -- one group's policy step
    def _wait_group(self, g: int, timeout: float = 60.0) -> None:
        S, deadline = self.S, time.time() + timeout
        while (S["done"][:, g] < S["go"][:, g]).any():
            if getattr(self, "_drain_error", None) is not None:
                self._check()
            self.drain(block=False)  # a worker whose ring is full waits for it
            if time.time() > deadline:
                self._check()
                raise RuntimeError("actor workers did not finish their environment steps")
            time.sleep(_SLEEP)

    def _slice(self, g: int) -> slice:
        rows = self._groups[g]
        return slice(int(rows[0]), int(rows[-1]) + 1)

    def _issue(self, g: int, policy) -> None:
        """Group g's policy inputs (its environments' current observations; the initial
        state where an episode starts, as IMPALAActor) handed to an issue/result policy."""
        S, sl = self.S, self._slice(g)
        first = S["first"][sl].astype(bool)
        h, c = self._h[sl], self._c[sl]
        h[first], c[first] = self._h0, self._c0
        if self.obs_pinned:
            policy.issue(S["obs"][sl], S["prev_a"][sl], S["prev_r"][sl], h, c,
                         observation_pinned=True)
        else:
            policy.issue(S["obs"][sl], S["prev_a"][sl], S["prev_r"][sl], h, c)

    def _finish(self, g: int, out) -> None:
        """Samples group g's actions from the policy outputs and posts them."""
        S, sl = self.S, self._slice(g)
        logits, _, h_new, c_new = out
        logits = np.asarray(logits, np.float32)
        rows = self._groups[g]
        z = logits - logits.max(axis=1, keepdims=True)
        cdf = np.cumsum(np.exp(z), axis=1)
        u = self._rng.random(len(rows)) * cdf[:, -1]
        actions = np.minimum((cdf < u[:, None]).sum(axis=1), logits.shape[1] - 1)
        S["action"][sl] = actions
        S["logits"][sl] = logits
        S["core_h"][sl] = self._h[sl]  # the state the step's action was taken from
        S["core_c"][sl] = self._c[sl]
        self._h[sl], self._c[sl] = h_new, c_new
        S["go"][:, g] += 1

    def _act(self, g: int) -> None:
        S, rows = self.S, self._groups[g]
        sl = slice(int(rows[0]), int(rows[-1]) + 1)
        first = S["first"][sl].astype(bool)
        h, c = self._h[sl], self._c[sl]
        h[first], c[first] = self._h0, self._c0  # IMPALAActor: initial state at episode start
        logits, _, h_new, c_new = self._policy(S["obs"][sl], S["prev_a"][sl], S["prev_r"][sl],
                                               h, c)
        logits = np.asarray(logits, np.float32)
        z = logits - logits.max(axis=1, keepdims=True)
        cdf = np.cumsum(np.exp(z), axis=1)
        u = self._rng.random(len(rows)) * cdf[:, -1]
        actions = np.minimum((cdf < u[:, None]).sum(axis=1), logits.shape[1] - 1)
        S["action"][sl] = actions
        S["logits"][sl] = logits
        S["core_h"][sl] = h  # the state the step's action was taken from
        S["core_c"][sl] = c
        self._h[sl], self._c[sl] = h_new, c_new
        S["go"][:, g] += 1

    def drain(self, block: bool = True) -> int:
        """Hands every finished item of every worker's ring to the sink; returns the count
        (0 without waiting when another thread is draining and block is False)."""
        if not self._drain_lock.acquire(blocking=block):
            return 0
        try:
            return self._drain()
        finally:
            self._drain_lock.release()

    def _drain(self) -> int:
        n_all = 0
        for r in self.R:
            head, tail = int(r["head"][0]), int(r["tail"][0])
            while tail < head:
                s = tail % self._M
                n = min(head - tail, self._M - s)
                self._sink([r[f"f{i}"][s:s + n] for i in range(len(self._fields))], n)
                tail += n
                r["tail"][0] = tail
                n_all += n
        self.items += n_all
        return n_all

    def run(self, policy_step, sink: Callable, ticks: int,
            should_stop: Optional[Callable[[], bool]] = None) -> None:
        """`ticks` policy steps of every group (each environment steps `ticks` times).
        policy_step: a callable, or a list of one issue/result object per group (e.g.
        IMPALALearner.pipelined_policy), whose calls are kept in flight: group g's network
        step is issued as soon as its environments have stepped and collected after the
        next group's is issued, so the GPU time overlaps the driver's waits."""
        if isinstance(policy_step, (list, tuple)):
            return self._run_pipelined(list(policy_step), sink, ticks, should_stop)
        self._policy, self._sink = policy_step, sink
        S = self.S
        if (S["done"] < 0).any():
            deadline = time.time() + 120.0
            while (S["done"] < 0).any():
                self._check()
                if time.time() > deadline:
                    raise RuntimeError("actor workers did not start")
                time.sleep(1e-3)
        st = self.stats
        for _ in range(int(ticks)):
            for g in range(self._G):
                t0 = time.perf_counter()
                self._wait_group(g)
                t1 = time.perf_counter()
                self.drain()
                t2 = time.perf_counter()
                self._act(g)
                t3 = time.perf_counter()
                st["wait_s"] += t1 - t0
                st["drain_s"] += t2 - t1
                st["issue_s"] += t3 - t2
                st["acts"] += 1
            if should_stop is not None and should_stop():
                break
        for g in range(self._G):  # the last posted actions are stepped
            self._wait_group(g)
        self.drain()

    def _wait_started(self) -> None:
        S = self.S
        deadline = time.time() + 120.0
        while (S["done"] < 0).any():
            self._check()
            if time.time() > deadline:
                raise RuntimeError("actor workers did not start")
            time.sleep(1e-3)

    def _run_pipelined(self, policies, sink, ticks, should_stop) -> None:
        if len(policies) != self._G:
            raise ValueError(f"{len(policies)} policies for {self._G} groups")
        import threading
        self._sink = sink
        self._wait_started()
        st = self.stats
        pending = None
        # Items are inserted by a thread of their own (the native insert copies outside the
        # GIL), so the driver only posts actions and issues policy steps.
        drained = threading.Event()
        self._drain_error = None

        def drainer():
            try:
                while not drained.is_set():
                    if not self.drain():
                        time.sleep(2e-4)
            except BaseException as e:  # noqa: BLE001 - handed to the driver thread
                self._drain_error = e

        dth = threading.Thread(target=drainer, daemon=True)
        dth.start()
        for _ in range(int(ticks)):
            for g in range(self._G):
                t0 = time.perf_counter()
                self._wait_group(g)
                t1 = time.perf_counter()
                # The workers are idle now: post the previous group's actions first (its
                # network step ran while they stepped group g), then issue group g's.
                t2 = t1
                if pending is not None:
                    out = policies[pending].result()
                    t2 = time.perf_counter()
                    self._finish(pending, out)
                t3 = time.perf_counter()
                self._issue(g, policies[g])
                pending = g
                t4 = time.perf_counter()
                t5 = t4
                for k, v in (("wait_s", t1 - t0), ("result_s", t2 - t1), ("post_s", t3 - t2),
                             ("issue_s", t4 - t3), ("drain_s", t5 - t4)):
                    st[k] += v
                st["acts"] += 1
            if should_stop is not None and should_stop():
                break
        if pending is not None:
            self._finish(pending, policies[pending].result())
        for g in range(self._G):
            self._wait_group(g)
        drained.set()
        dth.join()
        self._check()
        self.drain()
