"""IMPALALearner — drop-in for acme/agents/tf/impala/learning.py:36-180.

Same constructor (environment_spec, network, dataset, learning_rate, discount=0.99,
entropy_cost=0., baseline_cost=1., max_abs_reward=None, max_gradient_norm=None,
counter=None, logger=None) and `step()` contract.  One call takes a [B, T] batch of
sequences from the dataset (Step(observation=OAR(...), action, reward, discount,
start_of_episode, extras={'core_state': LSTMState, 'logits'})) and runs the whole step on
the GPU (acme_impala_step): torso over all B*T frames, OAR projection, LSTM unroll from
core_state[:, 0], policy/value head, V-trace, losses, BPTT, global-norm clip, Adam.

A step whose f16 planes overflowed, or whose one-launch LSTM unroll timed out, applies no
update (the device's step guard, as DQNLearner's): the learner sees the count lazily, logs
`skipped_steps` and recalibrates the plane scales before its next step (or raises
FloatingPointError with on_plane_overflow="raise").
"""

from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from acme_amd import core
from acme_amd.native import NativeIMPALA
from acme_amd.utils import counting, loggers


def _state_parts(core_state):
    if isinstance(core_state, dict):
        return core_state["hidden"], core_state["cell"]
    hidden, cell = core_state
    return hidden, cell


def _policy_engine(net: NativeIMPALA, rows: int) -> None:
    """Actor-side networks of 64+ rows run the Atari torso on the plane engine (the learner's
    f32-equivalent f16 planes): the 64-row policy step's f32 torso took 366 us."""
    if net.torso == "atari" and rows >= 64:
        net.set_policy_planes(True)


class IMPALALearner(core.Learner, core.Saveable):

    def __init__(self, environment_spec, network, dataset, learning_rate: float,
                 discount: float = 0.99, entropy_cost: float = 0., baseline_cost: float = 1.,
                 max_abs_reward: Optional[float] = None,
                 max_gradient_norm: Optional[float] = None,
                 counter: Optional[counting.Counter] = None,
                 logger: Optional[loggers.Logger] = None, batch_size: Optional[int] = None,
                 sequence_length: Optional[int] = None, seed: int = 0, device=None,
                 semantics: str = "tf", adam=None, on_plane_overflow: str = "skip"):
        if on_plane_overflow not in ("skip", "raise"):
            raise ValueError("on_plane_overflow must be 'skip' or 'raise'")
        self._on_overflow = on_plane_overflow
        self._skips_seen = 0
        self._env_spec = environment_spec
        self._network = network
        self._iterator = iter(dataset)
        B = batch_size or getattr(dataset, "batch_size", None) or 16
        T = sequence_length or getattr(dataset, "sequence_length", None) or 20
        self._native = NativeIMPALA(
            num_actions=network.num_actions, max_batch=B, max_sequence_length=T,
            torso=network.torso, obs_dim=network.obs_dim, lstm_size=network.lstm_size,
            head_size=network.head_size, discount=discount, entropy_cost=entropy_cost,
            baseline_cost=baseline_cost, max_abs_reward=max_abs_reward,
            max_gradient_norm=max_gradient_norm, learning_rate=learning_rate, semantics=semantics,
            device=device, **({} if adam is None else dict(
                adam_beta1=adam.beta1, adam_beta2=adam.beta2, adam_epsilon=adam.epsilon)))
        self._native.set_params(network.init(seed))
        self._counter = counter or counting.Counter()
        self._logger = logger or loggers.TerminalLogger("learner", time_delta=1.)
        self._timestamp = None
        m = self._native.metrics
        self._metric_views = {"loss": m[0], "critic_loss": m[1], "entropy_loss": m[2],
                              "policy_gradient_loss": m[3]}
        # Parameter snapshots for actor networks (actor_policy): allocated on first use.
        self._snap = None

    def _check_guard(self) -> int:
        n = self._native.skipped_steps  # pinned host word: no synchronisation
        if n != self._skips_seen:
            self._skips_seen = n
            if self._on_overflow == "raise":
                raise FloatingPointError(f"IMPALA learner: {n} step(s) skipped (f16 plane "
                                         "overflow or LSTM unroll timeout)")
            self._native.params_changed()
        return n

    def step(self):
        skipped = self._check_guard()
        sample = next(self._iterator)
        data = sample.data
        obs = data.observation
        if not hasattr(obs, "observation"):
            raise ValueError("IMPALAAtariNetwork takes OAR observations "
                             "(wrap the environment in ObservationActionRewardWrapper)")
        dt = torch.uint8 if self._network.torso == "atari" else torch.float32
        c = lambda x, t: x.to(t).contiguous()  # noqa: E731
        B, T = int(data.action.shape[0]), int(data.action.shape[1])
        hidden, cell = _state_parts(data.extras["core_state"])
        self._native.step(c(obs.observation.reshape((B, T, -1)) if dt == torch.float32
                            else obs.observation, dt),
                          c(obs.action.reshape(B, T), torch.int32),
                          c(obs.reward.reshape(B, T), torch.float32),
                          c(data.action.reshape(B, T), torch.int32),
                          c(data.reward.reshape(B, T), torch.float32),
                          c(data.discount.reshape(B, T), torch.float32),
                          c(data.extras["logits"], torch.float32),
                          hidden.to(torch.float32)[:, 0], cell.to(torch.float32)[:, 0])
        if self._snap is not None:
            self._publish_snapshot()
        now = time.time()
        elapsed = now - self._timestamp if self._timestamp else 0
        self._timestamp = now
        result = dict(self._metric_views)
        if skipped:
            result["skipped_steps"] = skipped
        result.update(self._counter.increment(steps=1, walltime=elapsed))
        self._logger.write(result)

    def policy_step(self, observation, prev_action, prev_reward, hidden, cell):
        """Batched network step for actors (numpy in, numpy out)."""
        n = self._native
        dt = torch.uint8 if self._network.torso == "atari" else torch.float32
        dev = n.device
        t = lambda x, d: torch.as_tensor(np.asarray(x)).to(dev, d)  # noqa: E731
        rows = int(np.asarray(prev_action).shape[0])
        lg, v, h, c = n.policy_step(t(observation, dt).reshape(rows, -1),
                                    t(prev_action, torch.int32), t(prev_reward, torch.float32),
                                    t(hidden, torch.float32), t(cell, torch.float32))
        return lg.cpu().numpy(), v.cpu().numpy(), h.cpu().numpy(), c.cpu().numpy()

    # -- actor-side parameter snapshots (the reference's VariableClient hands actors a whole
    # set of weights; an actor forward reading the learner's buffer while Adam rewrites it
    # in place could mix two updates).  Two snapshot buffers: after each step the learner's
    # stream copies the parameters into the one not published last (first waiting for every
    # actor read of it that was issued), records an event and publishes it; an actor step
    # waits for the published snapshot's event, reads it, and records its own read event.
    def _ensure_snapshots(self) -> None:
        if self._snap is None:
            n = self._native
            self._snap_lock = threading.Lock()
            self._snap_buf = [n.params.clone(), n.params.clone()]
            self._snap_ready = [torch.cuda.Event(), torch.cuda.Event()]
            self._snap_reads = [{}, {}]  # per buffer: the last read event of each stream
            for e in self._snap_ready:
                e.record(torch.cuda.current_stream(n.device))
            self._snap = 0  # the published buffer

    def _publish_snapshot(self) -> None:
        n = self._native
        cur = torch.cuda.current_stream(n.device)
        with self._snap_lock:
            j = self._snap ^ 1
            reads, self._snap_reads[j] = self._snap_reads[j], {}
        for ev in reads.values():
            cur.wait_event(ev)
        self._snap_buf[j].copy_(n.params)
        self._snap_ready[j].record(cur)
        with self._snap_lock:
            self._snap = j

    def actor_policy(self, max_rows: int = 16):
        """A policy_step for actor threads that does not share the learner's workspace: two
        native networks bound to the learner's two parameter snapshots, on the thread's own
        stream (actor inference overlaps learner steps; each actor step reads the latest
        published snapshot, a whole set of weights, as a VariableClient refreshed every
        step would)."""
        n = self._native
        self._ensure_snapshots()
        nets = [NativeIMPALA(num_actions=n.num_actions, max_batch=int(max_rows),
                             max_sequence_length=2, torso=n.torso, obs_dim=n.obs_dim,
                             lstm_size=n.lstm_size, head_size=self._network.head_size,
                             device=n.device, shared_params=buf) for buf in self._snap_buf]
        for net in nets:
            _policy_engine(net, max_rows)
        stream = torch.cuda.Stream(device=n.device)
        dt = torch.uint8 if self._network.torso == "atari" else torch.float32
        dev = n.device

        def step(observation, prev_action, prev_reward, hidden, cell):
            t = lambda x, d: torch.as_tensor(np.asarray(x)).to(dev, d, non_blocking=True)  # noqa
            rows = int(np.asarray(prev_action).shape[0])
            with self._snap_lock:
                j = self._snap
                stream.wait_event(self._snap_ready[j])
            with torch.cuda.stream(stream):
                lg, v, h, c = nets[j].policy_step(t(observation, dt).reshape(rows, -1),
                                                  t(prev_action, torch.int32),
                                                  t(prev_reward, torch.float32),
                                                  t(hidden, torch.float32),
                                                  t(cell, torch.float32), stream=stream)
                done = torch.cuda.Event()
                done.record(stream)
                with self._snap_lock:
                    self._snap_reads[j][id(stream)] = done  # later reads on a stream wait
                                                            # for the earlier ones
                out = [x.cpu().numpy() for x in (lg, v, h, c)]
            return tuple(out)

        step.native = nets  # keeps the networks alive with the closure
        return step

    def pipelined_policy(self, max_rows: int):
        """actor_policy as two halves for a driver that keeps several policy calls in flight
        (ProcessActorPool): issue(obs, prev_a, prev_r, h, c) stages the numpy inputs in pinned
        memory and issues the copies, the network step and the copies back on this policy's
        own stream without waiting; result() waits for them and returns (logits, v, h, c)."""
        return _PipelinedPolicy(self, int(max_rows))

    def get_variables(self, names: List[str]) -> List[Dict[str, np.ndarray]]:
        return [self._native.get_params("params")]

    @property
    def native(self) -> NativeIMPALA:
        return self._native

    @property
    def num_steps(self) -> int:
        return self._native.num_steps

    @property
    def state(self) -> Dict:
        return self.save()

    def save(self) -> Dict:
        n = self._native
        return {"network": n.get_params("params"),
                "optimizer": {"m": n.get_params("m"), "v": n.get_params("v"),
                              "step": n.applied_steps},
                "num_steps": n.num_steps,
                # f16 plane scales: a resumed run is bit-identical to an uninterrupted one.
                "plane_scales": n.scale_state()}

    def restore(self, state: Dict):
        n = self._native
        n.set_params(state["network"])
        for buf, src in ((n.m, state["optimizer"]["m"]), (n.v, state["optimizer"]["v"])):
            for k, t in n.views(buf).items():
                t.copy_(torch.as_tensor(np.asarray(src[k], np.float32)).view(t.shape))
        n.num_steps = int(state["num_steps"])
        n.applied_steps = int(state["optimizer"].get("step", state["num_steps"]))
        if "plane_scales" in state:
            n.set_scale_state(state["plane_scales"])
        if self._snap is not None:  # actors act with the restored weights from now on
            self._publish_snapshot()


class _PipelinedPolicy:
    """IMPALALearner.pipelined_policy: two networks bound to the learner's parameter
    snapshots (as actor_policy), one high-priority stream, and packed transfer blocks: the
    small inputs (previous actions and rewards, LSTM state) go to the device in one copy and
    the outputs (logits, values, LSTM state) come back in one, next to the observation copy
    (straight from page-locked memory when the caller has it there)."""

    def __init__(self, learner: "IMPALALearner", rows: int):
        n = learner._native  # noqa: SLF001
        learner._ensure_snapshots()  # noqa: SLF001
        self._l = learner
        self._nets = [NativeIMPALA(num_actions=n.num_actions, max_batch=rows,
                                   max_sequence_length=2, torso=n.torso, obs_dim=n.obs_dim,
                                   lstm_size=n.lstm_size,
                                   head_size=learner._network.head_size,  # noqa: SLF001
                                   device=n.device, shared_params=buf)
                      for buf in learner._snap_buf]  # noqa: SLF001
        for net in self._nets:
            _policy_engine(net, rows)
        try:  # the actors' policy ahead of the learner's kernels where both are queued
            self._stream = torch.cuda.Stream(device=n.device, priority=-1)
        except (RuntimeError, TypeError):
            self._stream = torch.cuda.Stream(device=n.device)
        A, H, dev = n.num_actions, n.lstm_size, n.device
        net = learner._network  # noqa: SLF001
        F = 84 * 84 * 4 if net.torso == "atari" else net.obs_dim
        odt = torch.uint8 if net.torso == "atari" else torch.float32
        self._rows, self._A, self._H = rows, A, H
        self._pin_obs = torch.empty((rows, F), dtype=odt, pin_memory=True)
        self._dev_obs = torch.empty((rows, F), dtype=odt, device=dev)
        # Small inputs, 4-byte words: prev_a [rows] (int32 bits), prev_r [rows], h, c [rows, H].
        self._nin = rows * (2 + 2 * H)
        self._pin_in = torch.empty(self._nin, dtype=torch.float32, pin_memory=True)
        self._dev_in = torch.empty(self._nin, dtype=torch.float32, device=dev)
        # Outputs: logits [rows, A], values [rows], h, c [rows, H].
        self._nout = rows * (A + 1 + 2 * H)
        self._pin_out = torch.empty(self._nout, dtype=torch.float32, pin_memory=True)
        self._dev_out = torch.empty(self._nout, dtype=torch.float32, device=dev)
        self._done = torch.cuda.Event()
        self._n = 0

    def _in_views(self, buf, n):
        R, H = self._rows, self._H
        return (buf[:n].view(torch.int32), buf[R:R + n], buf[2 * R:2 * R + n * H].view(n, H),
                buf[2 * R + R * H:2 * R + R * H + n * H].view(n, H))

    def _out_views(self, buf, n):
        R, A, H = self._rows, self._A, self._H
        o1, o2, o3 = R * A, R * A + R, R * A + R + R * H
        return (buf[:n * A].view(n, A), buf[o1:o1 + n], buf[o2:o2 + n * H].view(n, H),
                buf[o3:o3 + n * H].view(n, H))

    def issue(self, observation, prev_action, prev_reward, hidden, cell,
              observation_pinned: bool = False) -> None:
        """observation_pinned: the observation array lives in page-locked memory (e.g. a
        registered shared-memory block) and is copied to the device from there directly."""
        n = int(np.asarray(prev_action).shape[0])
        self._n = n
        pin = self._in_views(self._pin_in, n)
        for dst, x in zip(pin, (prev_action, prev_reward, hidden, cell)):
            dst.numpy()[...] = np.asarray(x).reshape(dst.shape)
        if observation_pinned:
            obs_src = torch.from_numpy(np.ascontiguousarray(observation).reshape(n, -1))
        else:
            np.copyto(self._pin_obs.numpy()[:n], np.asarray(observation).reshape(n, -1),
                      casting="unsafe")
            obs_src = self._pin_obs[:n]
        l, st = self._l, self._stream
        with l._snap_lock:  # noqa: SLF001
            j = l._snap  # noqa: SLF001
            st.wait_event(l._snap_ready[j])  # noqa: SLF001
        with torch.cuda.stream(st):
            self._dev_obs[:n].copy_(obs_src, non_blocking=True)
            self._dev_in.copy_(self._pin_in, non_blocking=True)
            outs = self._out_views(self._dev_out, n)
            self._nets[j].policy_step(self._dev_obs[:n], *self._in_views(self._dev_in, n),
                                      stream=st, out=outs)
            self._pin_out.copy_(self._dev_out, non_blocking=True)
            self._done.record(st)
            with l._snap_lock:  # noqa: SLF001
                l._snap_reads[j][id(st)] = self._done  # noqa: SLF001

    def result(self):
        self._done.synchronize()
        return tuple(x.numpy().copy() for x in self._out_views(self._pin_out, self._n))
