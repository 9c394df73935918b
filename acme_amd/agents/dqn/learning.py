"""DQNLearner — drop-in for acme/agents/tf/dqn/learning.py:35-199.

Same constructor arguments and `step()` contract: one call draws a batch from the
dataset iterator, runs the whole SGD step on the GPU (acme_dqn_step: three Q forwards,
double-Q n-step TD, Huber, f64 IS weights, backward, snt.Adam, post-step periodic target
copy), writes |td| priorities back to replay, increments the counter and logs.  Nothing
synchronises the host with the device: the loss is handed to the logger as a device
scalar and fetched only when a log line is actually emitted.

`network` / `target_network` are descriptors from acme_amd.networks (the reference
takes Sonnet modules); the target starts from its own initialisation, like the
reference's deepcopy + create_variables (agents/tf/dqn/agent.py:127-131).

Plane overflow (the uint8 Nature path runs its GEMMs on scaled f16 planes, csrc/gemm_p3.h):
a step in which some plane write overflowed f16 (a tensor's maximum grew more than ~2^8-fold
since the previous step, or fell more than ~2^7-fold) is skipped on the device: no
parameter, Adam moment or count, target or priority changes, and the end-of-step rescale
sets every scale from that step's true maxima.  The reference applies every step
(agents/tf/dqn/learning.py:147-161), so the learner RE-ISSUES a skipped step
(`on_plane_overflow="reissue"`, the default): the device holds every later step skipped
too (acme_dqn_set_reissue), and at the start of each step() call the learner reads the
verdict of the step issued two calls earlier (a pinned ring the device writes: no
synchronisation, and normally long decided, since the host runs at most two steps ahead).
On a skip it re-splits the parameter planes, recalibrates the scales and issues the held
batches again in their order, with the step counter of their first issue (so a due target
copy lands), before drawing the next batch; save(), state, get_variables() and q_values()
settle the last two steps the same way first.  So every step() call applies exactly one
update, in the reference's order, and a skip only costs the re-issued steps' time.
Re-issue needs the batches of the last two step() calls intact until the next draw: the
repo's own dataset iterators guarantee it (`holds_last_batches = 2`, their buffer rings);
with any other iterator the learner keeps its own copy of each held batch (one device copy
per step).  A write-back inside the step that timed out waiting for the step's verdict
(never expected; it would leave a step applied without its priorities) raises RuntimeError
when the learner next settles (save(), state, get_variables(), q_values()).
`"raise"` raises FloatingPointError instead; `"skip"` keeps the skip (the step's batch is
dropped, as before round 5).  `num_steps` (the target period) counts step() calls; Adam's
t counts applied updates.
"""

from __future__ import annotations

import collections
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from acme_amd import core
from acme_amd.adders import reverb as adders
from acme_amd.native import NativeDQN
from acme_amd.utils import counting, loggers

# Verdicts checked at step() call k: those of the steps issued up to call k - 2 (the
# dataset's buffer ring keeps the batches of calls k - 2 and k - 1 until call k draws).
_REISSUE_LAG = 2
_REISSUE_ATTEMPTS = 3


class DQNLearner(core.Learner, core.Saveable):

    def __init__(self, network, target_network, discount: float,
                 importance_sampling_exponent: float, learning_rate: float,
                 target_update_period: int, dataset, huber_loss_parameter: float = 1.0,
                 replay_client=None, counter: Optional[counting.Counter] = None,
                 logger: Optional[loggers.Logger] = None, checkpoint: bool = True,
                 max_abs_reward: float = 1.0, batch_size: Optional[int] = None, seed: int = 0,
                 device=None, data_parallel: bool = True, semantics: str = "tf",
                 target_seed: Optional[int] = None, adam=None,
                 reduce_logged_loss: bool = True, on_plane_overflow: str = "reissue"):
        if huber_loss_parameter < 0:
            raise ValueError("quadratic_linear_boundary must be >= 0.")
        if on_plane_overflow not in ("reissue", "skip", "raise"):
            raise ValueError("on_plane_overflow must be 'reissue', 'skip' or 'raise'")
        self._on_overflow = on_plane_overflow
        self._skips_seen = 0
        self._network = network
        self._iterator = iter(dataset)
        B = batch_size or getattr(dataset, "batch_size", None) or 256
        self._B = B
        import torch.distributed as _dist
        dp = (data_parallel and _dist.is_available() and _dist.is_initialized()
              and _dist.get_world_size() > 1)
        # A data-parallel rank takes its share of each global draw: up to 2 B rows
        # (acme_amd.replay.sharding), averaged over the nominal B.
        kw = dict(network=network.kind, num_actions=network.num_actions,
                  max_batch=2 * B if dp else B,
                  obs_dtype=network.obs_dtype, discount=discount,
                  importance_sampling_exponent=importance_sampling_exponent,
                  learning_rate=learning_rate, huber_loss_parameter=huber_loss_parameter,
                  target_update_period=target_update_period, max_abs_reward=max_abs_reward,
                  semantics=semantics, device=device)
        if adam is not None:
            kw.update(adam_beta1=adam.beta1, adam_beta2=adam.beta2, adam_epsilon=adam.epsilon)
        if network.kind == "mlp":
            kw.update(obs_dim=network.obs_dim, hidden=network.hidden)
        self._native = NativeDQN(**kw)
        self._native.set_params(network.init(seed), target_network.init(
            seed + 1 if target_seed is None else target_seed))
        self._replay_client = replay_client
        self._counter = counter or counting.Counter()
        self._logger = logger or loggers.TerminalLogger("learner", time_delta=1.0)
        self._timestamp = None
        self._obs_flat = int(np.prod(network.obs_shape))
        self._checkpoint = checkpoint
        self._log_loss = True
        # Data parallel: whether the logged loss is all-reduced to the global batch's.  Every
        # rank must make the same choice (a collective issued on some ranks only would pair
        # with a different collective on the others), so it is a constructor argument, never
        # derived from per-rank state such as the logger type.
        self._reduce_loss = bool(reduce_logged_loss)
        # Data parallelism (one process per GPU, torch.distributed over RCCL): each rank
        # samples its own batch from its replay shard; the IS-weight normaliser and the
        # gradients are reduced across ranks before Adam, so every replica applies the
        # update of the global batch (the mean-then-apply order of the reference's only
        # data-parallel learner, acme/agents/tf/crr/recurrent_learning.py:346-358).
        self._dist = None
        self._staged = False       # bench: the staged data-parallel path on one process
        self._comm_stream = None
        if data_parallel:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
                self._dist = dist
                for buf in (self._native.params, self._native.target):
                    dist.broadcast(buf, src=0)
                self._native.params_changed()
                self._gmin = torch.empty(1, dtype=torch.float64, device=self._native.device)
                self._grad_split = self._native.grad_split
                self._avg_op = (dist.ReduceOp.AVG if dist.get_backend() == "nccl" else None)
                # The ranks skip an overflowed step together: each rank's decision rides in
                # the torso gradient bucket's all-reduce.
                self._native.set_data_parallel_gate(True)
        self._skip_word = self._native.skip_word
        # Re-issue of skipped steps (the plane path): the last _REISSUE_LAG issued steps,
        # their batches held (sequence number of their verdict, step counter at issue).
        self._reissue = self._skip_word is not None and on_plane_overflow == "reissue"
        self._native.set_reissue(self._reissue)
        self._held = collections.deque(maxlen=_REISSUE_LAG)
        self._checked = self._native.verdicts_issued  # verdicts below this are settled
        self._reissued = 0
        # A foreign iterator may reuse its buffers on the next draw: hold copies then.
        self._copy_held = (self._reissue and getattr(self._iterator, "holds_last_batches", 0)
                           < _REISSUE_LAG)

    # ------------------------------------------------------------------ step
    def _prepare(self, x: torch.Tensor, dtype) -> torch.Tensor:
        if x.dtype != dtype:
            x = x.to(dtype)
        return x.contiguous()

    def _check_guard(self) -> int:
        """Skipped steps the device has reported so far (no synchronisation); on a new one,
        re-split the planes and recalibrate the scales before the next step, or raise."""
        if self._reissue:
            self._await_verdicts(settle=False)
            return self._reissued
        n = self._native.skipped_steps
        if n != self._skips_seen:
            self._skips_seen = n
            if self._on_overflow == "raise":
                raise FloatingPointError(
                    f"DQN learner: {n} step(s) skipped on f16 plane overflow (their updates "
                    "were not applied)")
            self._native.params_changed()
        return n

    def _await_verdicts(self, settle: bool) -> None:
        """Reads the verdicts not yet settled: those of all steps but the last
        _REISSUE_LAG - 1 issued (waiting for them: normally long decided), or with `settle`
        of every issued step (after a synchronisation); re-issues from the first skipped."""
        n = self._native
        if settle:
            torch.cuda.synchronize(n.device)
        upto = n.verdicts_issued - (0 if settle else _REISSUE_LAG - 1)
        deadline = None
        while self._checked < upto:
            v = n.step_verdict(self._checked)
            if v is None:  # not decided yet: the device is behind (rare)
                deadline = deadline or time.time() + 120.0
                if time.time() > deadline:
                    raise RuntimeError("DQN learner: step verdict not published within 120 s")
                time.sleep(0)
                continue
            if v:
                self._reissue_from(self._checked)
            else:
                self._checked += 1
        if settle and n.guard_state()["verdict_timeouts"]:
            raise RuntimeError("DQN learner: a priority write-back timed out waiting for its "
                               "step's verdict (the step's priorities were not written)")

    def _reissue_from(self, seq: int) -> None:
        """Step `seq` was skipped, and (sticky hold) every step issued after it: recalibrate
        and issue their held batches again, in order."""
        n = self._native
        if self._on_overflow == "raise":
            raise FloatingPointError(
                "DQN learner: a step was skipped on f16 plane overflow (its update was not "
                "applied)")
        for _ in range(_REISSUE_ATTEMPTS):
            torch.cuda.synchronize(n.device)
            pend = [e for e in self._held if e["seq"] >= seq]
            if not pend or pend[0]["seq"] != seq:
                raise RuntimeError(f"DQN learner: skipped step (verdict {seq}) is no longer held")
            n.params_changed()  # re-split the planes, recalibrate; clears the hold
            n.num_steps = pend[0]["num_steps"]
            for e in pend:
                self._issue(e)
                self._reissued += 1
            torch.cuda.synchronize(n.device)
            seq = next((e["seq"] for e in pend if n.step_verdict(e["seq"])), None)
            if seq is None:
                self._checked = n.verdicts_issued
                self._skips_seen = n.skipped_steps
                return
        raise FloatingPointError(
            f"DQN learner: a step was skipped {_REISSUE_ATTEMPTS} times on f16 plane overflow")

    def _issue(self, e: Dict) -> None:
        """Issues one held step (its batch, priority write-back and step counter)."""
        n = self._native
        e["seq"] = n.verdicts_issued
        e["num_steps"] = n.num_steps
        batch, fb, keys, B = e["batch"], e["fb"], e["keys"], e["B"]
        inputs_event = e.pop("inputs_event", None)  # only for the first issue
        upd = None
        if self._dist is None and not self._staged:
            # The priority write-back rides in the step (on the learner's second stream
            # beside the backward) when the client's table offers it.
            prep = getattr(self._replay_client, "prepare_priority_update", None)
            if prep is not None:
                upd = prep(adders.DEFAULT_PRIORITY_TABLE, keys)
            n.step(*batch, obs_f16=fb, priority_update=upd, inputs_event=inputs_event)
        else:
            self._staged_step(batch, fb, inputs_event)
        if self._replay_client is not None and upd is None:
            # Gated on the step's skip word: a skipped step writes no priority.
            kw = {"skip_word": self._skip_word} if self._skip_word else {}
            self._replay_client.update_priorities(table=adders.DEFAULT_PRIORITY_TABLE,
                                                  keys=keys, priorities=n.priorities[:B], **kw)

    def _settle(self) -> None:
        """Before the learner's state is read: every issued step decided, a skipped one
        re-issued."""
        if self._reissue:
            self._await_verdicts(settle=True)

    def step(self):
        skipped = self._check_guard()
        sample = next(self._iterator)
        o_tm1, a_tm1, r_t, d_t, o_t = sample.data[:5]
        keys, probs = sample.info[:2]
        B = int(a_tm1.shape[0])
        obs_dt = torch.uint8 if self._network.obs_dtype == "uint8" else torch.float32
        views = (o_tm1.reshape(B, self._obs_flat), a_tm1.reshape(B), r_t.reshape(B),
                 d_t.reshape(B), o_t.reshape(B, self._obs_flat), probs)
        batch = tuple(self._prepare(x, dt) for x, dt in zip(
            views, (obs_dt, torch.int32, torch.float32, torch.float32, obs_dt, torch.float64)))
        # The batch's ready event lets the learner start its target forward without waiting
        # for the previous step's tail, unless a conversion above produced new tensors on
        # this stream.
        inputs_event = getattr(self._iterator, "last_inputs_event", None)
        if any(b is not v for b, v in zip(batch, views)):
            inputs_event = None
        # The dataset's fused gather also wrote the exact f16 copy of [o_tm1; o_t] (uint8
        # tables; rows [0, B) and [B, 2B) of its buffer): the learner then skips its own
        # conversion (same bits).
        fb = getattr(self._iterator, "last_frames_f16", None)
        if fb is not None:
            fb = (fb[:2 * B] if obs_dt == torch.uint8 and fb.shape[0] >= 2 * B
                  and fb.shape[1] == self._obs_flat else None)
        if self._copy_held:
            batch = tuple(x.clone() for x in batch)
            keys = keys.clone()
            fb = None if fb is None else fb.clone()
        e = dict(batch=batch, fb=fb, keys=keys, B=B, inputs_event=inputs_event)
        self._issue(e)
        if self._reissue:
            self._held.append(e)
        now = time.time()
        elapsed = now - self._timestamp if self._timestamp else 0
        self._timestamp = now
        loss = self._native.loss
        if self._dist is not None and self._log_loss and self._reduce_loss:
            # The logged loss is the global batch's (SURVEY §8(e) collective 3): each rank's
            # loss is its share's sum over the nominal per-rank batch, so the mean over ranks.
            loss = loss.clone()
            if self._avg_op is not None:
                self._dist.all_reduce(loss, op=self._avg_op)
            else:
                self._dist.all_reduce(loss)
                loss.mul_(1.0 / self._dist.get_world_size())
        result = {"loss": loss} if self._log_loss else {}
        if skipped:
            result["skipped_steps"] = skipped
        result.update(self._counter.increment(steps=1, walltime=elapsed))
        self._logger.write(result)

    def _staged_step(self, batch, fb, inputs_event=None):
        """The data-parallel step: the learner's stages with the collectives between them.
        Gradient all-reduce in two buckets overlapped with the backward pass: the dense
        layers' gradients (the buffer's tail, ~99% of the bytes) are reduced on a collective
        stream as soon as the learner's second stream has produced them, while the torso
        backward runs on the compute stream.  Without a process group (bench's
        dp_staged_ms_per_step: the N = 1 point of a scaling curve) the same stages run with
        the collectives left out."""
        dist = self._dist
        n = self._native
        gmin = None
        if dist is not None:
            # The IS normaliser's all-reduce (8 bytes) runs beside the forwards: only the
            # loss (stage 4) reads it.
            gmin = self._gmin
            n.batch_min_probability(batch[5], gmin)
            work_min = dist.all_reduce(gmin, op=dist.ReduceOp.MIN, async_op=True)
        n.forward_backward_stage(2, *batch, mean_over=self._B, obs_f16=fb,
                                 inputs_event=inputs_event)
        if dist is not None:
            work_min.wait()
        n.forward_backward_stage(4, *batch, global_min_probability=gmin, mean_over=self._B,
                                 obs_f16=fb)
        if dist is not None:
            split = self._grad_split
            tail, head = n.grads[split:], n.grads[:split]
            op = self._avg_op if self._avg_op is not None else dist.ReduceOp.SUM
            if self._comm_stream is None:
                self._comm_stream = torch.cuda.Stream(device=n.device)
            cs = self._comm_stream
            cs.wait_stream(torch.cuda.current_stream(n.device))
            n.dense_grads_ready(cs)
            with torch.cuda.stream(cs):
                work = dist.all_reduce(tail, op=op, async_op=True)
        n.forward_backward_stage(1, *batch, global_min_probability=gmin, mean_over=self._B)
        if dist is not None:
            if split > 0:
                dist.all_reduce(head, op=op)
            work.wait()
            torch.cuda.current_stream(n.device).wait_stream(cs)
            if self._avg_op is None:  # gloo: sum, then scale
                n.grads.mul_(1.0 / dist.get_world_size())
        n.apply()

    # ------------------------------------------------------------------ variables
    def q_values(self, observations, use_target: bool = False) -> np.ndarray:
        self._settle()
        obs_dt = torch.uint8 if self._network.obs_dtype == "uint8" else torch.float32
        x = torch.as_tensor(np.asarray(observations)).to(self._native.device, obs_dt)
        x = x.reshape(x.shape[0], -1).contiguous()
        q = self._native.q_values(x, use_target).cpu().numpy()
        if self._skip_word and self._native.guard_state()["q_values_overflowed"]:
            # The forward overflowed its planes; its rescale set the scales from its maxima.
            q = self._native.q_values(x, use_target).cpu().numpy()
        return q

    def get_variables(self, names: List[str]) -> List[List[np.ndarray]]:
        # As the TF learner: one collection (the online trainable variables), names ignored.
        self._settle()
        sonnet = self._network.to_sonnet(self._native.get_params("params"))
        return [[sonnet[k] for k in sorted(sonnet)]]

    @property
    def num_steps(self) -> int:
        return self._native.num_steps

    @property
    def native(self) -> NativeDQN:
        return self._native

    @property
    def state(self) -> Dict:
        return self.save()

    def save(self) -> Dict:
        self._settle()
        n = self._native
        return {"network": n.get_params("params"), "target_network": n.get_params("target"),
                # Adam's t: the updates applied (step() calls minus skipped steps).
                "optimizer": {"m": n.get_params("m"), "v": n.get_params("v"),
                              "step": n.applied_steps},
                "num_steps": n.num_steps,
                # f16 plane scales (csrc/gemm_p3.h): restoring them keeps a resumed run
                # bit-identical to an uninterrupted one.
                "plane_scales": n.scale_state()}

    def restore(self, state: Dict):
        self._settle()
        self._held.clear()
        n = self._native
        n.set_params(state["network"], state["target_network"])
        for buf, src in ((n.m, state["optimizer"]["m"]), (n.v, state["optimizer"]["v"])):
            views = n.views(buf)
            for k, t in views.items():
                t.copy_(torch.as_tensor(np.asarray(src[k], np.float32)).view(t.shape))
        n.params_changed()
        if "plane_scales" in state:
            n.set_scale_state(state["plane_scales"])
        n.num_steps = int(state["num_steps"])
        n.applied_steps = int(state["optimizer"].get("step", state["num_steps"]))
        self._checked = n.verdicts_issued
