"""Actor harness of BASELINE configs[3]: many CPU actors feeding one GPU IMPALA learner.

The reference runs each actor as its own program (acme/agents/tf/impala/acting.py:32-95:
per-actor TF policy, VariableClient, SequenceAdder into the Reverb queue) and the learner
steps while the queue holds a batch (agents/tf/impala/agent.py:111-120).  Here N host
threads each run an environment, an IMPALAActor and a SequenceAdder into the device
QueueTable; their policy calls go through one BatchedPolicy, which collects the pending
requests of all actors and runs them as one GPU network step (acme_impala_policy_step on
the learner's current parameters, in chunks of the learner's max batch).  The actors see
the learner's latest parameters at every step (the reference's VariableClient refreshes
every `update_period` steps; a fresher policy is the limit of that).

VectorActorPool runs the same per-environment actor semantics with K environments per host
thread and one policy call per K steps: a thread per actor pays two GIL hand-offs per
environment step (request, reply), which caps the thread pool at ~3k steps/s whatever the
environment costs.
"""

from __future__ import annotations

import threading
import time
from typing import Callable, List, Optional

import numpy as np

from acme_amd.agents.impala.acting import IMPALAActor
from acme_amd.networks import LSTMState


class BatchedPolicy:
    """Serves IMPALAActor.policy_step calls of many threads as batched GPU steps."""

    def __init__(self, policy_step: Callable, max_rows: int, max_wait_s: float = 0.002):
        self._step = policy_step  # (obs, prev_a, prev_r, h, c) numpy -> numpy (rows <= max_rows)
        self._max_rows = int(max_rows)
        self._max_wait = float(max_wait_s)
        self._cv = threading.Condition()
        self._pending: List[list] = []
        self._active = 0
        self._stop = False
        self.batches = 0
        self.rows = 0
        self._thread = threading.Thread(target=self._serve, daemon=True)
        self._thread.start()

    def register(self) -> None:
        with self._cv:
            self._active += 1

    def unregister(self) -> None:
        with self._cv:
            self._active -= 1
            self._cv.notify_all()

    def __call__(self, obs, prev_a, prev_r, h, c):
        req = [obs, prev_a, prev_r, h, c, None, threading.Event()]
        with self._cv:
            self._pending.append(req)
            self._cv.notify_all()
        req[6].wait()
        if isinstance(req[5], BaseException):
            raise req[5]
        return req[5]

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._thread.join()

    def _serve(self) -> None:
        while True:
            with self._cv:
                while not self._pending and not self._stop:
                    self._cv.wait(0.05)
                if self._stop and not self._pending:
                    return
                # Wait (briefly) for every active actor to queue its request.
                deadline = time.time() + self._max_wait
                while len(self._pending) < self._active and not self._stop:
                    left = deadline - time.time()
                    if left <= 0:
                        break
                    self._cv.wait(left)
                batch, self._pending = self._pending, []
            try:
                for i in range(0, len(batch), self._max_rows):
                    part = batch[i:i + self._max_rows]
                    cat = [np.concatenate([r[k] for r in part]) for k in range(5)]
                    lg, v, h, c = self._step(*cat)
                    for j, r in enumerate(part):
                        r[5] = (lg[j:j + 1], v[j:j + 1], h[j:j + 1], c[j:j + 1])
                    self.batches += 1
                    self.rows += len(part)
            except BaseException as e:  # noqa: BLE001  (handed to the callers)
                for r in batch:
                    if r[5] is None:
                        r[5] = e
            for r in batch:
                r[6].set()


class ActorPool:
    """N actor threads: environment (make_env(i)), IMPALAActor and SequenceAdder each, one
    shared BatchedPolicy.  start() / stop(); env_steps counts every environment step."""

    def __init__(self, make_env: Callable[[int], object], make_adder: Callable[[int], object],
                 policy: BatchedPolicy, initial_state: Callable, num_actors: int = 64,
                 seed: int = 0):
        self._make_env = make_env
        self._make_adder = make_adder
        self._policy = policy
        self._initial_state = initial_state
        self._n = int(num_actors)
        self._seed = int(seed)
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self._steps = [0] * self._n
        self.errors: List[BaseException] = []

    @property
    def env_steps(self) -> int:
        return sum(self._steps)

    def _run(self, i: int) -> None:
        self._policy.register()
        try:
            env = self._make_env(i)
            actor = IMPALAActor(self._policy, self._initial_state, self._make_adder(i),
                                seed=self._seed + i)
            ts = env.reset()
            actor.observe_first(ts)
            while not self._stop.is_set():
                a = actor.select_action(ts.observation)
                ts = env.step(a)
                actor.observe(a, ts)
                self._steps[i] += 1
                if ts.last():
                    ts = env.reset()
                    actor.observe_first(ts)
        except BaseException as e:  # noqa: BLE001
            if not self._stop.is_set():
                self.errors.append(e)
        finally:
            self._policy.unregister()

    def start(self) -> None:
        self._threads = [threading.Thread(target=self._run, args=(i,), daemon=True)
                         for i in range(self._n)]
        for t in self._threads:
            t.start()

    def stop(self, timeout: Optional[float] = 30.0) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout)


class VectorActor:
    """K environments stepped by one host thread with one batched policy call per step:
    per environment exactly IMPALAActor's behaviour (acme/agents/tf/impala/acting.py:
    a ~ Categorical(logits) of the step, the LSTM state carried across steps and reset at
    episode starts, {'logits', 'core_state'} of the step handed to the adder as extras)."""

    def __init__(self, envs: List[object], adders: List[object], policy_step: Callable,
                 initial_state: Callable, seed: int = 0, max_rows: Optional[int] = None):
        self._envs = envs
        self._rows = int(max_rows) if max_rows else len(envs)  # rows per policy call
        self._adders = adders
        self._policy = policy_step
        self._K = len(envs)
        self._rng = np.random.default_rng(seed)
        s0 = initial_state(1)
        self._h0, self._c0 = s0.hidden[0].copy(), s0.cell[0].copy()
        st = initial_state(self._K)
        self._h, self._c = st.hidden.copy(), st.cell.copy()
        self._ts = [None] * self._K
        self.steps = 0

    def start(self) -> None:
        for i, (env, adder) in enumerate(zip(self._envs, self._adders)):
            ts = env.reset()
            adder.add_first(ts)
            self._ts[i] = ts
            self._h[i], self._c[i] = self._h0, self._c0

    def step(self) -> None:
        K, ts = self._K, self._ts
        obs = np.stack([t.observation.observation for t in ts])
        prev_a = np.array([t.observation.action for t in ts], np.int32)
        prev_r = np.array([t.observation.reward for t in ts], np.float32)
        if self._rows >= K:
            logits, _, h, c = self._policy(obs, prev_a, prev_r, self._h, self._c)
        else:
            parts = [self._policy(obs[j:j + self._rows], prev_a[j:j + self._rows],
                                  prev_r[j:j + self._rows], self._h[j:j + self._rows],
                                  self._c[j:j + self._rows]) for j in range(0, K, self._rows)]
            logits, h, c = (np.concatenate([q[k] for q in parts]) for k in (0, 2, 3))
        z = logits - logits.max(axis=1, keepdims=True)
        p = np.exp(z)
        cdf = np.cumsum(p, axis=1)
        u = self._rng.random(K) * cdf[:, -1]
        actions = np.minimum((cdf < u[:, None]).sum(axis=1), logits.shape[1] - 1).astype(np.int32)
        prev_h, prev_c = self._h, self._c
        self._h, self._c = np.array(h, np.float32), np.array(c, np.float32)
        for i in range(K):
            a = actions[i]
            nt = self._envs[i].step(a)
            self._adders[i].add(a, nt, {"logits": logits[i],
                                        "core_state": LSTMState(prev_h[i], prev_c[i])})
            if nt.last():
                nt = self._envs[i].reset()
                self._adders[i].add_first(nt)
                self._h[i], self._c[i] = self._h0, self._c0
            ts[i] = nt
        self.steps += K


class VectorActorPool:
    """`num_actors` environments over `threads` host threads (VectorActor each); each thread
    calls its own policy (make_policy(t): e.g. learner.actor_policy(max_rows), one network
    and stream per thread) on at most `max_rows` environments at a time.  start() / stop();
    env_steps counts every environment step."""

    def __init__(self, make_env: Callable[[int], object], make_adder: Callable[[int], object],
                 make_policy: Callable[[int], Callable], initial_state: Callable,
                 num_actors: int = 64, threads: int = 2, seed: int = 0,
                 max_rows: Optional[int] = None):
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self.errors: List[BaseException] = []
        threads = max(1, min(int(threads), int(num_actors)))
        split = np.array_split(np.arange(int(num_actors)), threads)
        self._actors = [VectorActor([make_env(int(i)) for i in ids],
                                    [make_adder(int(i)) for i in ids], make_policy(t),
                                    initial_state, seed=seed + t, max_rows=max_rows)
                        for t, ids in enumerate(split)]

    @property
    def env_steps(self) -> int:
        return sum(a.steps for a in self._actors)

    def _run(self, actor: VectorActor) -> None:
        try:
            actor.start()
            while not self._stop.is_set():
                actor.step()
        except BaseException as e:  # noqa: BLE001
            if not self._stop.is_set():
                self.errors.append(e)

    def start(self) -> None:
        self._threads = [threading.Thread(target=self._run, args=(a,), daemon=True)
                         for a in self._actors]
        for t in self._threads:
            t.start()

    def stop(self, timeout: Optional[float] = 30.0) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout)
