"""Thin owners of the native objects behind the drop-in API.

`NativeReplay` wraps an acme_replay (GPU table); `NativeDQN` wraps an acme_dqn learner and
owns its flat device buffers (params / target / grads / Adam m, v) as torch tensors so
that torch.distributed (RCCL) can all-reduce the gradient buffer in place.
"""

from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from acme_amd import _lib
from acme_amd._lib import check, lib, ptr, stream_ptr

SAMPLER_UNIFORM = 0
SAMPLER_PRIORITIZED = 1


class NativeReplay:
    """Device-resident FIFO table with a 64-ary sum-tree sampler (see csrc/replay.hip)."""

    def __init__(self, capacity: int, field_bytes: Sequence[int], prioritized: bool,
                 priority_exponent: float = 0.6, seed: int = 1234, device=None):
        _lib.require_gpu()
        if len(field_bytes) > _lib.MAX_FIELDS:
            raise ValueError(f"at most {_lib.MAX_FIELDS} flattened fields per item")
        cfg = _lib.ReplayConfig()
        cfg.capacity = int(capacity)
        cfg.sampler = SAMPLER_PRIORITIZED if prioritized else SAMPLER_UNIFORM
        cfg.num_fields = len(field_bytes)
        cfg.priority_exponent = float(priority_exponent)
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        for i, b in enumerate(field_bytes):
            cfg.field_bytes[i] = int(b)
        self.field_bytes = [int(b) for b in field_bytes]
        self.capacity = int(capacity)
        self.prioritized = prioritized
        self.priority_exponent = float(priority_exponent)
        self.seed = cfg.seed
        self.device = torch.device(device or "cuda")
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().acme_replay_create(ctypes.byref(cfg), ctypes.byref(h)), "replay create")
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().acme_replay_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self._h = None

    @property
    def handle(self):
        return self._h

    def size(self) -> int:
        return int(lib().acme_replay_size(self._h))

    def nstep_writer(self, n_step: int, discount: float, obs_bytes: int, action_bytes: int,
                     rows_per_chunk: int = 64) -> "NativeNStepWriter":
        return NativeNStepWriter(self, n_step, discount, obs_bytes, action_bytes, rows_per_chunk)

    def insert(self, fields: Sequence, priorities: Optional[np.ndarray] = None,
               stream=None) -> np.ndarray:
        """fields: per-field arrays/tensors with leading dim n (host numpy or device tensors)."""
        n = int(fields[0].shape[0])
        keys = np.empty(n, np.uint64)
        on_dev = isinstance(fields[0], torch.Tensor) and fields[0].is_cuda
        keep = []
        ptrs = (ctypes.c_void_p * len(fields))()
        for i, f in enumerate(fields):
            if on_dev:
                t = f.contiguous()
                keep.append(t)
                ptrs[i] = t.data_ptr()
            else:
                a = np.ascontiguousarray(f)
                keep.append(a)
                ptrs[i] = a.ctypes.data
            nbytes = keep[-1].nbytes if not on_dev else keep[-1].numel() * keep[-1].element_size()
            if nbytes != n * self.field_bytes[i]:
                raise ValueError(f"field {i}: expected {n * self.field_bytes[i]} bytes, got {nbytes}")
        pr = None
        if priorities is not None:
            pr = np.ascontiguousarray(priorities, np.float64)
            if pr.shape != (n,):
                raise ValueError("priorities must have shape [n]")
        check(lib().acme_replay_insert(self._h, ptrs, n, None if pr is None else pr.ctypes.data,
                                       1 if on_dev else 0, keys.ctypes.data, stream_ptr(stream)),
              "replay insert")
        return keys

    def stage_capacity(self) -> int:
        """Items per pinned staging chunk (acme_replay_stage_capacity)."""
        n = int(lib().acme_replay_stage_capacity(self._h))
        if n <= 0:
            check(_lib.ACME_ERR_HIP, "replay staging")
        return n

    def stage(self, n: int) -> List[np.ndarray]:
        """Pinned host rows for n items: one writable uint8 [n, field_bytes[f]] array per
        field (valid until the matching commit)."""
        ptrs = (ctypes.c_void_p * len(self.field_bytes))()
        check(lib().acme_replay_stage(self._h, int(n), ptrs), "replay stage")
        return [np.ctypeslib.as_array((ctypes.c_uint8 * (n * b)).from_address(ptrs[i]))
                .reshape(n, b) for i, b in enumerate(self.field_bytes)]

    def commit(self, n: int, priorities: Optional[np.ndarray] = None, stream=None) -> np.ndarray:
        """Issues the first n staged items (side-stream H2D, no host wait); returns keys."""
        keys = np.empty(n, np.uint64)
        pr = None
        if priorities is not None:
            pr = np.ascontiguousarray(priorities, np.float64)
            if pr.shape != (n,):
                raise ValueError("priorities must have shape [n]")
        check(lib().acme_replay_commit(self._h, int(n), None if pr is None else pr.ctypes.data,
                                       keys.ctypes.data, stream_ptr(stream)), "replay commit")
        return keys

    def sync_inserts(self) -> None:
        check(lib().acme_replay_sync_inserts(self._h), "replay sync_inserts")

    def fill_synthetic(self, n: int, layout: int, num_actions: int = 18, seed: int = 0,
                       stream=None) -> None:
        check(lib().acme_replay_fill_synthetic(self._h, int(n), int(layout), int(num_actions),
                                               int(seed), stream_ptr(stream)), "fill_synthetic")

    def sample(self, batch: int, step: int, out: Optional[Dict[str, torch.Tensor]] = None,
               stream=None) -> Dict[str, torch.Tensor]:
        if out is None:
            out = self.alloc_sample_info(batch)
        check(lib().acme_replay_sample(self._h, int(batch), int(step) & 0xFFFFFFFFFFFFFFFF,
                                       ptr(out["slots"]), ptr(out["keys"]),
                                       ptr(out["probabilities"]), ptr(out["table_size"]),
                                       ptr(out["priorities"]), stream_ptr(stream)),
              "replay sample")
        return out

    def alloc_sample_info(self, batch: int) -> Dict[str, torch.Tensor]:
        d = self.device
        return dict(slots=torch.empty(batch, dtype=torch.int64, device=d),
                    keys=torch.empty(batch, dtype=torch.uint64, device=d),
                    probabilities=torch.empty(batch, dtype=torch.float64, device=d),
                    table_size=torch.empty(batch, dtype=torch.int64, device=d),
                    priorities=torch.empty(batch, dtype=torch.float64, device=d))

    def gather(self, slots: torch.Tensor, outs: Sequence[torch.Tensor], stream=None) -> None:
        ptrs = (ctypes.c_void_p * len(outs))(*[o.data_ptr() for o in outs])
        check(lib().acme_replay_gather(self._h, ptr(slots), int(slots.numel()), ptrs,
                                       stream_ptr(stream)), "replay gather")

    def update_priorities(self, keys: torch.Tensor, priorities: torch.Tensor, stream=None,
                          skip_word: Optional[int] = None) -> None:
        """skip_word: a learner's device skip word (NativeDQN.skip_word): the update is
        dropped when the step that produced the priorities was skipped."""
        keys = keys.to(self.device, torch.uint64).contiguous()
        priorities = priorities.to(self.device, torch.float64).contiguous()
        if skip_word:
            check(lib().acme_replay_update_priorities_gated(
                self._h, ptr(keys), ptr(priorities), int(keys.numel()), ctypes.c_void_p(skip_word),
                stream_ptr(stream)), "update_priorities")
            return
        check(lib().acme_replay_update_priorities(self._h, ptr(keys), ptr(priorities),
                                                  int(keys.numel()), stream_ptr(stream)),
              "update_priorities")

    def export_state(self) -> Dict[str, np.ndarray]:
        """Host copy of the live table (checkpoints): field rows, keys and raw priorities of
        slots [0, size), the insert counter.  Leaves and tree levels are derived data."""
        L = lib()
        n = self.size()
        torch.cuda.synchronize(self.device)
        out = {"inserted": np.int64(L.acme_replay_inserted(self._h))}
        for f, b in enumerate(self.field_bytes):
            p = ctypes.c_void_p()
            check(L.acme_replay_storage(self._h, f, ctypes.byref(p)))
            out[f"field_{f}"] = _device_array(p.value, n * b, np.uint8, self.device).cpu() \
                .numpy().reshape(n, b).copy()
        lv, rp, ks = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        check(L.acme_replay_debug_leaves(self._h, ctypes.byref(lv), ctypes.byref(rp),
                                         ctypes.byref(ks)))
        out["raw_priorities"] = _device_array(rp.value, n, np.float64, self.device).cpu() \
            .numpy().view(np.float64).copy()
        out["keys"] = _device_array(ks.value, n, np.uint64, self.device).cpu().numpy() \
            .view(np.uint64).copy()
        return out

    def import_state(self, state: Dict[str, np.ndarray]) -> None:
        """Inverse of export_state (same capacity and field layout): writes rows, keys and
        raw priorities, then rebuilds leaves and levels on the device."""
        L = lib()
        keys = np.asarray(state["keys"], np.uint64)
        n = len(keys)
        if n > self.capacity:
            raise ValueError(f"state holds {n} items, table capacity is {self.capacity}")
        torch.cuda.synchronize(self.device)
        for f, b in enumerate(self.field_bytes):
            rows = np.ascontiguousarray(state[f"field_{f}"], np.uint8)
            if rows.shape != (n, b):
                raise ValueError(f"field {f}: state rows {rows.shape}, table expects {(n, b)}")
            p = ctypes.c_void_p()
            check(L.acme_replay_storage(self._h, f, ctypes.byref(p)))
            _memcpy_htod(p.value, rows)
        lv, rp, ks = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        check(L.acme_replay_debug_leaves(self._h, ctypes.byref(lv), ctypes.byref(rp),
                                         ctypes.byref(ks)))
        _memcpy_htod(rp.value, np.asarray(state["raw_priorities"], np.float64))
        _memcpy_htod(ks.value, keys)
        check(L.acme_replay_restore(self._h, int(state["inserted"]), None), "replay restore")
        torch.cuda.synchronize(self.device)

    def debug_state(self) -> Dict[str, np.ndarray]:
        """Host copies of leaf weights / raw priorities / keys (tests)."""
        lv, rp, ks = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().acme_replay_debug_leaves(self._h, ctypes.byref(lv), ctypes.byref(rp),
                                             ctypes.byref(ks)))
        torch.cuda.synchronize(self.device)
        n = self.capacity
        out = {}
        for name, p, dt, cnt in (("leaves", lv, np.float64, n), ("raw", rp, np.float64, n),
                                 ("keys", ks, np.uint64, n)):
            out[name] = _device_array(p.value, cnt, dt, self.device).cpu().numpy().view(dt).copy()
        return out


class NativeNStepWriter:
    """acme_nstep_writer: the native side of NStepTransitionAdder (rows formed and packed in
    C, straight into pinned chunks).  `add_raw(act_ptr, reward, discount, obs_ptr, last,
    priority)` is the per-step entry, with the pointers of host arrays the caller keeps alive
    for the call."""

    def __init__(self, table: NativeReplay, n_step: int, discount: float, obs_bytes: int,
                 action_bytes: int, rows_per_chunk: int = 64):
        h = ctypes.c_void_p()
        L = lib()
        check(L.acme_nstep_writer_create(table.handle, int(n_step), float(discount),
                                         int(obs_bytes), int(action_bytes), int(rows_per_chunk),
                                         ctypes.byref(h)), "n-step writer create")
        self._table = table  # the writer commits into it: keep it alive
        self._h = h
        self._add = L.acme_nstep_writer_add
        self._pending = L.acme_nstep_writer_pending

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().acme_nstep_writer_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self._h = None

    def start(self, obs_ptr: int) -> None:
        check(lib().acme_nstep_writer_start(self._h, obs_ptr), "n-step writer start")

    def add_raw(self, act_ptr: int, reward: float, discount: float, obs_ptr: int, last: bool,
                priority: float = 1.0) -> None:
        rc = self._add(self._h, act_ptr, reward, discount, obs_ptr, 1 if last else 0, priority)
        if rc:
            check(rc, "n-step writer add")

    def flush(self) -> None:
        check(lib().acme_nstep_writer_flush(self._h), "n-step writer flush")

    def reset(self) -> None:
        check(lib().acme_nstep_writer_reset(self._h), "n-step writer reset")

    def pending(self) -> int:
        return int(self._pending(self._h))


def _device_array(address: int, count: int, dtype, device) -> torch.Tensor:
    """Copies `count` elements at a raw device address into a new tensor (test helper)."""
    nbytes = count * np.dtype(dtype).itemsize
    dst = torch.empty(nbytes, dtype=torch.uint8, device=device)
    torch.cuda.synchronize(device)
    _memcpy_dtod(dst.data_ptr(), address, nbytes)
    return dst


_hip = None


def _hip_memcpy(dst: int, src: int, nbytes: int, kind: int) -> None:
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipMemcpy.restype = ctypes.c_int
    rc = _hip.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), ctypes.c_size_t(nbytes), kind)
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed ({rc})")


def _memcpy_dtod(dst: int, src: int, nbytes: int) -> None:
    _hip_memcpy(dst, src, nbytes, 3)


def _memcpy_htod(dst: int, host: np.ndarray) -> None:
    """Synchronous host -> device copy of a numpy array to a raw device address."""
    a = np.ascontiguousarray(host)
    if a.nbytes:
        _hip_memcpy(dst, a.ctypes.data, a.nbytes, 1)


NET_NATURE = 0
NET_MLP = 1
OBS_U8 = 0
OBS_F32 = 1


class NativeDQN:
    """acme_dqn learner + its flat buffers."""

    def __init__(self, *, network: str, num_actions: int, max_batch: int, obs_dtype: str,
                 obs_dim: int = 0, hidden: Sequence[int] = (), discount: float = 0.99,
                 importance_sampling_exponent: float = 0.2, learning_rate: float = 1e-3,
                 huber_loss_parameter: float = 1.0, target_update_period: int = 100,
                 max_abs_reward: float = 1.0, adam_beta1: float = 0.9, adam_beta2: float = 0.999,
                 adam_epsilon: float = 1e-8, semantics: str = "tf", device=None):
        """semantics: "tf" restates acme/agents/tf/dqn/learning.py, "jax" the JAX learner
        (acme/agents/jax/dqn/learning.py: f32 IS weights, steps+1 target cadence, optix.adam)."""
        _lib.require_gpu()
        if semantics not in ("tf", "jax"):
            raise ValueError(f"semantics must be 'tf' or 'jax', got {semantics!r}")
        if huber_loss_parameter < 0:
            raise ValueError("quadratic_linear_boundary must be >= 0.")
        cfg = _lib.DQNConfig()
        cfg.network = NET_NATURE if network == "nature" else NET_MLP
        cfg.obs_dtype = OBS_U8 if obs_dtype == "uint8" else OBS_F32
        cfg.num_actions = int(num_actions)
        cfg.max_batch = int(max_batch)
        cfg.obs_dim = int(obs_dim)
        if len(hidden) > _lib.MAX_MLP_LAYERS:
            raise ValueError(f"at most {_lib.MAX_MLP_LAYERS} hidden layers")
        cfg.num_hidden = len(hidden)
        for i, h in enumerate(hidden):
            cfg.hidden[i] = int(h)
        cfg.discount = discount
        cfg.importance_sampling_exponent = importance_sampling_exponent
        cfg.learning_rate = learning_rate
        cfg.huber_loss_parameter = huber_loss_parameter
        cfg.adam_beta1, cfg.adam_beta2, cfg.adam_epsilon = adam_beta1, adam_beta2, adam_epsilon
        cfg.target_update_period = int(target_update_period)
        cfg.max_abs_reward = max_abs_reward
        cfg.semantics = _lib.SEMANTICS_JAX if semantics == "jax" else _lib.SEMANTICS_TF
        self.cfg = cfg
        self.semantics = semantics
        self.network = network
        self.num_actions = int(num_actions)
        self.max_batch = int(max_batch)
        self.device = torch.device(device or "cuda")
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().acme_dqn_create(ctypes.byref(cfg), ctypes.byref(h)), "dqn create")
        self._h = h
        L = lib()
        self.flat_size = int(L.acme_dqn_flat_size(h))
        self.num_params = int(L.acme_dqn_num_params(h))
        self.tensors: List[Tuple[str, int, Tuple[int, ...]]] = []
        for i in range(L.acme_dqn_num_tensors(h)):
            off, numel, nd = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
            shape = (ctypes.c_int64 * 4)()
            name = ctypes.c_char_p()
            check(L.acme_dqn_tensor_info(h, i, ctypes.byref(off), ctypes.byref(numel),
                                         ctypes.byref(nd), shape, ctypes.byref(name)))
            self.tensors.append((name.value.decode(), int(off.value),
                                 tuple(int(shape[k]) for k in range(nd.value))))
        d = self.device
        z = lambda: torch.zeros(self.flat_size, dtype=torch.float32, device=d)  # noqa: E731
        self.params, self.target, self.grads, self.m, self.v = z(), z(), z(), z(), z()
        check(L.acme_dqn_bind(h, ptr(self.params), ptr(self.target), ptr(self.grads),
                              ptr(self.m), ptr(self.v)), "dqn bind")
        self.loss = torch.zeros(1, dtype=torch.float32, device=d)
        self.td_error = torch.zeros(max_batch, dtype=torch.float32, device=d)
        self.priorities = torch.zeros(max_batch, dtype=torch.float64, device=d)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().acme_dqn_destroy(h)
            except Exception:
                pass
            self._h = None

    # --------------------------------------------------------------- parameters
    def views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        out = {}
        for name, off, shape in self.tensors:
            n = int(np.prod(shape))
            out[name] = flat[off:off + n].view(shape)
        return out

    def set_params(self, params: Dict[str, np.ndarray], target: Optional[Dict] = None) -> None:
        for flat, src in ((self.params, params), (self.target, target if target is not None else params)):
            v = self.views(flat)
            for name, t in v.items():
                t.copy_(torch.as_tensor(np.asarray(src[name], np.float32)).view(t.shape))
        self.params_changed()

    def params_changed(self) -> None:
        """Tells the learner its params / target buffers were written from outside (its
        derived f16 parameter planes are rebuilt before the next use)."""
        check(lib().acme_dqn_params_changed(self._h), "dqn params_changed")

    def scale_state(self) -> np.ndarray:
        """The plane scales (learner state for checkpoints; empty without the plane path)."""
        n = ctypes.c_int32(0)
        check(lib().acme_dqn_scale_state(self._h, None, 0, ctypes.byref(n)), "dqn scale_state")
        out = np.zeros(n.value, np.float32)
        if n.value:
            check(lib().acme_dqn_scale_state(self._h, out.ctypes.data, n.value, ctypes.byref(n)),
                  "dqn scale_state")
        return out

    def set_scale_state(self, state) -> None:
        """Restores scale_state() (after params_changed): resumed steps are bit-identical."""
        a = np.ascontiguousarray(np.asarray(state, np.float32))
        if a.size:
            check(lib().acme_dqn_set_scale_state(self._h, a.ctypes.data, a.size),
                  "dqn set_scale_state")

    def plane_overflow(self, reset: bool = False) -> bool:
        """True if a plane tensor of the uint8 Nature path exceeded f16's range at its scale
        since the last reset (synchronises the device; acme_dqn_plane_overflow)."""
        v = ctypes.c_int32(0)
        check(lib().acme_dqn_plane_overflow(self._h, ctypes.byref(v), int(reset)), "dqn plane_overflow")
        return bool(v.value)

    # ---- step guard (acme_dqn_guard_state: the skip-on-overflow rule of the plane path)
    @property
    def skipped_steps(self) -> int:
        """Steps skipped so far among those the device has finished (no synchronisation)."""
        return int(lib().acme_dqn_skipped_steps(self._h))

    def guard_state(self) -> Dict[str, int]:
        """{applied, skipped, last_skipped, q_values_overflowed, verdict_timeouts} (synchronises
        the device)."""
        a = (ctypes.c_int64 * 4)()
        check(lib().acme_dqn_guard_state(self._h, a), "dqn guard_state")
        t = ctypes.c_int64()
        check(lib().acme_dqn_verdict_timeouts(self._h, ctypes.byref(t)), "dqn verdict_timeouts")
        return dict(applied=int(a[0]), skipped=int(a[1]), last_skipped=int(a[2]),
                    q_values_overflowed=int(a[3]), verdict_timeouts=int(t.value))

    @property
    def applied_steps(self) -> int:
        """Updates applied (Adam's t after the last step); synchronises."""
        return self.guard_state()["applied"]

    @applied_steps.setter
    def applied_steps(self, n: int) -> None:
        check(lib().acme_dqn_set_applied_steps(self._h, int(n)), "dqn set_applied_steps")

    @property
    def skip_word(self) -> Optional[int]:
        """Device address of the word an after-step priority update is gated on."""
        p = ctypes.c_void_p()
        check(lib().acme_dqn_skip_word(self._h, ctypes.byref(p)), "dqn skip_word")
        return p.value

    # ---- re-issue of skipped steps (acme_dqn_set_reissue / _verdicts_issued / _step_verdict)
    def set_reissue(self, enable: bool) -> None:
        """A skipped step holds every later step skipped until the next calibration, so the
        caller can re-issue the held batches in order (DQNLearner)."""
        check(lib().acme_dqn_set_reissue(self._h, 1 if enable else 0), "dqn set_reissue")

    @property
    def verdicts_issued(self) -> int:
        """Step verdicts issued so far (the next step's verdict has this sequence number)."""
        return int(lib().acme_dqn_verdicts_issued(self._h))

    def step_verdict(self, seq: int) -> Optional[bool]:
        """None while verdict `seq` is undecided, else whether that step was skipped (no
        synchronisation: a pinned ring the device writes)."""
        v = ctypes.c_int32(-1)
        check(lib().acme_dqn_step_verdict(self._h, int(seq), ctypes.byref(v)), "dqn step_verdict")
        return None if v.value < 0 else bool(v.value)

    def set_data_parallel_gate(self, enable: bool) -> None:
        check(lib().acme_dqn_set_data_parallel_gate(self._h, 1 if enable else 0), "dqn dp gate")

    def get_params(self, which: str = "params") -> Dict[str, np.ndarray]:
        flat = getattr(self, which)
        return {k: v.detach().cpu().numpy().copy() for k, v in self.views(flat).items()}

    @property
    def num_steps(self) -> int:
        return int(lib().acme_dqn_num_steps(self._h))

    @num_steps.setter
    def num_steps(self, n: int) -> None:
        check(lib().acme_dqn_set_num_steps(self._h, int(n)))

    def debug_buffer(self, name: str) -> np.ndarray:
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        check(lib().acme_dqn_debug_buffer(self._h, name.encode(), ctypes.byref(p),
                                          ctypes.byref(n)))
        return _device_array(p.value, n.value, np.float32, self.device).cpu().numpy().view(
            np.float32).copy()

    # --------------------------------------------------------------- step
    def _batch(self, o_tm1, a_tm1, r_t, d_t, o_t, probabilities, global_min_probability=None,
               mean_over=None, obs_f16=None):
        B = int(a_tm1.shape[0])
        if B < 1 or B > self.max_batch:
            raise ValueError(f"batch of {B} rows: the learner takes 1..{self.max_batch}")
        for name, t in (("o_tm1", o_tm1), ("a_tm1", a_tm1), ("r_t", r_t), ("d_t", d_t),
                        ("o_t", o_t), ("probabilities", probabilities)):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.is_contiguous()):
                raise ValueError(f"{name} must be a contiguous device tensor")
            if t.shape[0] != B:
                raise ValueError(f"{name} has leading dim {t.shape[0]}, expected {B}")
        if a_tm1.dtype != torch.int32 or r_t.dtype != torch.float32 or d_t.dtype != torch.float32:
            raise ValueError("a_tm1 must be int32, r_t and d_t float32")
        if probabilities.dtype != torch.float64:
            raise ValueError("probabilities must be float64")
        want = torch.uint8 if self.cfg.obs_dtype == OBS_U8 else torch.float32
        if o_tm1.dtype != want or o_t.dtype != want:
            raise ValueError(f"observations must be {want}")
        tb = _lib.TransitionBatch()
        tb.o_tm1, tb.a_tm1, tb.r_t, tb.d_t, tb.o_t = (ptr(o_tm1), ptr(a_tm1), ptr(r_t), ptr(d_t),
                                                      ptr(o_t))
        tb.probabilities = ptr(probabilities)
        tb.batch = B
        tb.global_min_probability = ptr(global_min_probability)
        tb.mean_over = int(mean_over or 0)
        if obs_f16 is not None:  # [2B, obs] f16 bits of [o_tm1; o_t] (the dataset's copy)
            if not (isinstance(obs_f16, torch.Tensor) and obs_f16.is_cuda and
                    obs_f16.dtype in (torch.int16, torch.uint16, torch.float16) and
                    obs_f16.is_contiguous() and obs_f16.shape[0] >= 2 * B and
                    obs_f16[0].numel() == o_tm1[0].numel()):
                raise ValueError("obs_f16 must be a contiguous [2B, obs] 16-bit device tensor")
            tb.obs_f16 = ptr(obs_f16)
        return tb

    @staticmethod
    def _event_handle(ev) -> Optional[int]:
        if ev is None:
            return None
        return ev.handle if hasattr(ev, "handle") else int(ev.cuda_event)

    def _outputs(self, q_tm1=None):
        o = _lib.DQNOutputs()
        o.loss, o.td_error, o.priorities = ptr(self.loss), ptr(self.td_error), ptr(self.priorities)
        o.q_tm1 = ptr(q_tm1)
        return o

    def forward_backward(self, *batch, global_min_probability=None, q_tm1=None, stream=None):
        tb = self._batch(*batch, global_min_probability=global_min_probability)
        out = self._outputs(q_tm1)
        check(lib().acme_dqn_forward_backward(self._h, ctypes.byref(tb), ctypes.byref(out),
                                              stream_ptr(stream)), "dqn forward_backward")

    def forward_backward_stage(self, stage: int, *batch, global_min_probability=None,
                               q_tm1=None, stream=None, mean_over=None, obs_f16=None,
                               inputs_event=None):
        """Stage 0: forwards, loss, head/dense backward (grads[grad_split:]); stage 1: torso
        backward (grads[:grad_split]).  Stage 0 may be issued as stage 2 (forwards) then
        stage 3 (loss and dense backward; global_min_probability is read from here on) or
        stage 4 (stage 3 without ordering the stream after the dense gradients: see
        dense_grads_ready).  mean_over: the batch mean's denominator (default the batch; a
        data-parallel share passes the nominal per-rank batch).  inputs_event: as for
        step()."""
        tb = self._batch(*batch, global_min_probability=global_min_probability,
                         mean_over=mean_over, obs_f16=obs_f16)
        tb.inputs_event = self._event_handle(inputs_event)
        out = self._outputs(q_tm1)
        check(lib().acme_dqn_forward_backward_stage(self._h, ctypes.byref(tb), ctypes.byref(out),
                                                    int(stage), stream_ptr(stream)),
              f"dqn forward_backward stage {stage}")

    def dense_grads_ready(self, stream=None) -> None:
        """Orders `stream` (default: the current one) after the dense gradients
        grads[grad_split:] of the last stage 3 / 4."""
        check(lib().acme_dqn_dense_grads_ready(self._h, stream_ptr(stream)), "dense grads ready")

    def dp_init(self, comm, world_size: int) -> None:
        """Binds a caller-owned RCCL communicator (ncclComm_t) for dp_step."""
        check(lib().acme_dqn_dp_init(self._h, ctypes.c_void_p(comm), int(world_size)), "dp init")

    def dp_step(self, *batch, mean_over=None, q_tm1=None, stream=None, obs_f16=None):
        """One data-parallel step over the bound communicator (acme_dqn_dp_step)."""
        tb = self._batch(*batch, mean_over=mean_over, obs_f16=obs_f16)
        out = self._outputs(q_tm1)
        check(lib().acme_dqn_dp_step(self._h, ctypes.byref(tb), ctypes.byref(out),
                                     stream_ptr(stream)), "dqn dp step")

    @property
    def grad_split(self) -> int:
        s = ctypes.c_int64()
        check(lib().acme_dqn_grad_split(self._h, ctypes.byref(s)))
        return int(s.value)

    def batch_min_probability(self, probabilities: torch.Tensor, out: torch.Tensor, stream=None):
        """out[0] = min(probabilities) on the device (data-parallel IS normaliser)."""
        check(lib().acme_min_f64(ptr(probabilities), int(probabilities.numel()), ptr(out),
                                 stream_ptr(stream)), "min_f64")

    def apply(self, stream=None):
        check(lib().acme_dqn_apply(self._h, stream_ptr(stream)), "dqn apply")

    def step(self, *batch, q_tm1=None, stream=None, obs_f16=None, priority_update=None,
             inputs_event=None):
        """One SGD step.  priority_update = (native replay handle, uint64 keys tensor[, raw
        hipEvent_t of the table's last device read or None]): the batch's priorities are
        written back to that table as part of the step (acme_dqn_step_update: beside the
        backward on the plane path, after that read).  inputs_event: an event at which the
        batch's inputs are complete (acme_transition_batch.inputs_event)."""
        tb = self._batch(*batch, obs_f16=obs_f16)
        tb.inputs_event = self._event_handle(inputs_event)
        out = self._outputs(q_tm1)
        if priority_update is None:
            check(lib().acme_dqn_step(self._h, ctypes.byref(tb), ctypes.byref(out),
                                      stream_ptr(stream)), "dqn step")
            return
        handle, keys, after = (tuple(priority_update) + (None,))[:3]
        if keys.dtype not in (torch.uint64, torch.int64) or not keys.is_contiguous():
            raise ValueError("priority_update keys must be a contiguous 64-bit tensor")
        if keys.numel() != int(tb.batch) or not keys.is_cuda:
            raise ValueError("priority_update keys must hold one key per batch row, on the "
                             "learner's device")
        check(lib().acme_dqn_step_update(self._h, ctypes.byref(tb), ctypes.byref(out), handle,
                                         ptr(keys), after, stream_ptr(stream)), "dqn step")

    def q_values(self, obs: torch.Tensor, use_target: bool = False, stream=None) -> torch.Tensor:
        B = int(obs.shape[0])
        q = torch.empty(B, self.num_actions, dtype=torch.float32, device=self.device)
        check(lib().acme_dqn_q_values(self._h, ptr(obs.contiguous()), B, 1 if use_target else 0,
                                      ptr(q), stream_ptr(stream)), "dqn q_values")
        return q


def nccl_unique_id() -> bytes:
    """A fresh RCCL unique id (128 bytes) for nccl_comm_init on every rank."""
    buf = (ctypes.c_uint8 * 128)()
    check(lib().acme_nccl_get_unique_id(buf), "nccl unique id")
    return bytes(buf)


def nccl_comm_init(uid: bytes, world_size: int, rank: int) -> int:
    """An RCCL communicator handle (ncclComm_t as an int) for rank of world_size."""
    buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
    comm = ctypes.c_void_p()
    check(lib().acme_nccl_comm_init(buf, int(world_size), int(rank), ctypes.byref(comm)),
          "nccl comm init")
    return int(comm.value)


def nccl_comm_destroy(comm: int) -> None:
    check(lib().acme_nccl_comm_destroy(ctypes.c_void_p(comm)), "nccl comm destroy")


class NativeD4PG:
    """acme_d4pg learner + its flat buffers (policy tensors first, then critic tensors)."""

    def __init__(self, *, obs_dim: int, act_dim: int, max_batch: int,
                 policy_sizes: Sequence[int] = (256, 256, 256),
                 critic_sizes: Sequence[int] = (512, 512, 256), num_atoms: int = 51,
                 vmin: float = -150.0, vmax: float = 150.0, action_min=None, action_max=None,
                 discount: float = 0.99, target_update_period: int = 100,
                 policy_learning_rate: float = 1e-4, critic_learning_rate: float = 1e-4,
                 clipping: bool = True, adam_beta1: float = 0.9, adam_beta2: float = 0.999,
                 adam_epsilon: float = 1e-8, layer_norm_epsilon: float = 1e-5, device=None):
        _lib.require_gpu()
        cfg = _lib.D4PGConfig()
        cfg.obs_dim, cfg.act_dim, cfg.max_batch = int(obs_dim), int(act_dim), int(max_batch)
        for n, sizes in (("policy", policy_sizes), ("critic", critic_sizes)):
            if not 1 <= len(sizes) <= _lib.D4PG_MAX_LAYERS:
                raise ValueError(f"{n} needs 1..{_lib.D4PG_MAX_LAYERS} layer sizes")
        cfg.num_policy_layers = len(policy_sizes)
        cfg.num_critic_layers = len(critic_sizes)
        for i, s in enumerate(policy_sizes):
            cfg.policy_sizes[i] = int(s)
        for i, s in enumerate(critic_sizes):
            cfg.critic_sizes[i] = int(s)
        if act_dim > _lib.D4PG_MAX_ACT:
            raise ValueError(f"act_dim must be <= {_lib.D4PG_MAX_ACT}")
        lo = np.broadcast_to(np.asarray(-1.0 if action_min is None else action_min, np.float32),
                             (act_dim,))
        hi = np.broadcast_to(np.asarray(1.0 if action_max is None else action_max, np.float32),
                             (act_dim,))
        for j in range(act_dim):
            cfg.action_min[j], cfg.action_max[j] = float(lo[j]), float(hi[j])
        cfg.num_atoms, cfg.vmin, cfg.vmax = int(num_atoms), vmin, vmax
        cfg.discount, cfg.target_update_period = discount, int(target_update_period)
        cfg.policy_learning_rate, cfg.critic_learning_rate = policy_learning_rate, critic_learning_rate
        cfg.adam_beta1, cfg.adam_beta2, cfg.adam_epsilon = adam_beta1, adam_beta2, adam_epsilon
        cfg.clipping = 1 if clipping else 0
        cfg.layer_norm_epsilon = layer_norm_epsilon
        self.cfg = cfg
        self.obs_dim, self.act_dim, self.max_batch = int(obs_dim), int(act_dim), int(max_batch)
        self.device = torch.device(device or "cuda")
        h = ctypes.c_void_p()
        L = lib()
        with torch.cuda.device(self.device):
            check(L.acme_d4pg_create(ctypes.byref(cfg), ctypes.byref(h)), "d4pg create")
        self._h = h
        self.flat_size = int(L.acme_d4pg_flat_size(h))
        self.policy_size = int(L.acme_d4pg_policy_size(h))
        self.tensors: List[Tuple[str, int, Tuple[int, ...]]] = []
        for i in range(L.acme_d4pg_num_tensors(h)):
            off, numel, nd = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
            shape = (ctypes.c_int64 * 4)()
            name = ctypes.c_char_p()
            check(L.acme_d4pg_tensor_info(h, i, ctypes.byref(off), ctypes.byref(numel),
                                          ctypes.byref(nd), shape, ctypes.byref(name)))
            self.tensors.append((name.value.decode(), int(off.value),
                                 tuple(int(shape[k]) for k in range(nd.value))))
        d = self.device
        z = lambda: torch.zeros(self.flat_size, dtype=torch.float32, device=d)  # noqa: E731
        self.params, self.target, self.grads, self.m, self.v = z(), z(), z(), z(), z()
        check(L.acme_d4pg_bind(h, ptr(self.params), ptr(self.target), ptr(self.grads),
                               ptr(self.m), ptr(self.v)), "d4pg bind")
        self.critic_loss = torch.zeros(1, dtype=torch.float32, device=d)
        self.policy_loss = torch.zeros(1, dtype=torch.float32, device=d)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().acme_d4pg_destroy(h)
            except Exception:
                pass
            self._h = None

    views = NativeDQN.views
    set_params = NativeDQN.set_params
    get_params = NativeDQN.get_params

    def params_changed(self) -> None:  # the D4PG step reads the f32 buffers directly
        pass

    @property
    def num_steps(self) -> int:
        return int(lib().acme_d4pg_num_steps(self._h))

    @num_steps.setter
    def num_steps(self, n: int) -> None:
        check(lib().acme_d4pg_set_num_steps(self._h, int(n)))

    def debug_buffer(self, name: str) -> np.ndarray:
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        check(lib().acme_d4pg_debug_buffer(self._h, name.encode(), ctypes.byref(p),
                                           ctypes.byref(n)))
        return _device_array(p.value, n.value, np.float32, self.device).cpu().numpy().view(
            np.float32).copy()

    def step(self, o_tm1, a_tm1, r_t, d_t, o_t, stream=None):
        B = int(r_t.shape[0])
        for name, t, cols in (("o_tm1", o_tm1, self.obs_dim), ("a_tm1", a_tm1, self.act_dim),
                              ("r_t", r_t, None), ("d_t", d_t, None), ("o_t", o_t, self.obs_dim)):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.is_contiguous()
                    and t.dtype == torch.float32):
                raise ValueError(f"{name} must be a contiguous float32 device tensor")
            if t.shape[0] != B or (cols is not None and t.numel() != B * cols):
                raise ValueError(f"{name} has shape {tuple(t.shape)}, expected [{B}, {cols}]")
        b = _lib.D4PGBatch()
        b.o_tm1, b.a_tm1, b.r_t, b.d_t, b.o_t = (ptr(o_tm1), ptr(a_tm1), ptr(r_t), ptr(d_t),
                                                 ptr(o_t))
        b.batch = B
        out = _lib.D4PGOutputs()
        out.critic_loss, out.policy_loss = ptr(self.critic_loss), ptr(self.policy_loss)
        check(lib().acme_d4pg_step(self._h, ctypes.byref(b), ctypes.byref(out),
                                   stream_ptr(stream)), "d4pg step")

    def policy(self, obs: torch.Tensor, use_target: bool = False, stream=None) -> torch.Tensor:
        rows = int(obs.shape[0])
        obs = obs.reshape(rows, -1).to(self.device, torch.float32).contiguous()
        if obs.shape[1] != self.obs_dim:
            raise ValueError(f"observations must have {self.obs_dim} features")
        a = torch.empty(rows, self.act_dim, dtype=torch.float32, device=self.device)
        check(lib().acme_d4pg_policy(self._h, ptr(obs), rows, 1 if use_target else 0, ptr(a),
                                     stream_ptr(stream)), "d4pg policy")
        return a


class NativeIMPALA:
    """acme_impala learner + its flat buffers (no target network)."""

    def __init__(self, *, num_actions: int, max_batch: int, max_sequence_length: int,
                 torso: str = "atari", obs_dim: int = 0, lstm_size: int = 256,
                 head_size: int = 256, discount: float = 0.99, entropy_cost: float = 0.0,
                 baseline_cost: float = 1.0, max_abs_reward: Optional[float] = None,
                 max_gradient_norm: Optional[float] = None, learning_rate: float = 1e-3,
                 adam_beta1: float = 0.9, adam_beta2: float = 0.999, adam_epsilon: float = 1e-8,
                 semantics: str = "tf", device=None, shared_params: Optional[torch.Tensor] = None):
        """semantics: "tf" (acme/agents/tf/impala) or "jax" (acme/agents/jax/impala: the
        optix.chain(clip_by_global_norm, adam) update; max_gradient_norm None = inf).
        shared_params: bind another instance's parameter buffer (an actor-side network with
        its own workspace, reading the learner's current parameters)."""
        _lib.require_gpu()
        if semantics not in ("tf", "jax"):
            raise ValueError(f"semantics must be 'tf' or 'jax', got {semantics!r}")
        cfg = _lib.IMPALAConfig()
        cfg.torso = _lib.IMPALA_TORSO_ATARI if torso == "atari" else _lib.IMPALA_TORSO_FLAT
        cfg.obs_dim, cfg.num_actions = int(obs_dim), int(num_actions)
        cfg.max_batch, cfg.max_sequence_length = int(max_batch), int(max_sequence_length)
        cfg.lstm_size, cfg.head_size = int(lstm_size), int(head_size)
        cfg.discount, cfg.entropy_cost, cfg.baseline_cost = discount, entropy_cost, baseline_cost
        # learning.py:67-71: None -> no reward clipping, gradient norm 1e10.
        cfg.max_abs_reward = float("inf") if max_abs_reward is None else max_abs_reward
        cfg.max_gradient_norm = ((float("inf") if semantics == "jax" else 1e10)
                                 if max_gradient_norm is None else max_gradient_norm)
        cfg.semantics = _lib.SEMANTICS_JAX if semantics == "jax" else _lib.SEMANTICS_TF
        cfg.learning_rate = learning_rate
        cfg.adam_beta1, cfg.adam_beta2, cfg.adam_epsilon = adam_beta1, adam_beta2, adam_epsilon
        self.cfg = cfg
        self.torso, self.obs_dim = torso, int(obs_dim)
        self.num_actions, self.lstm_size = int(num_actions), int(lstm_size)
        self.max_batch, self.max_sequence_length = int(max_batch), int(max_sequence_length)
        self.device = torch.device(device or "cuda")
        h = ctypes.c_void_p()
        L = lib()
        with torch.cuda.device(self.device):
            check(L.acme_impala_create(ctypes.byref(cfg), ctypes.byref(h)), "impala create")
        self._h = h
        self.flat_size = int(L.acme_impala_flat_size(h))
        self.tensors: List[Tuple[str, int, Tuple[int, ...]]] = []
        for i in range(L.acme_impala_num_tensors(h)):
            off, numel, nd = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
            shape = (ctypes.c_int64 * 4)()
            name = ctypes.c_char_p()
            check(L.acme_impala_tensor_info(h, i, ctypes.byref(off), ctypes.byref(numel),
                                            ctypes.byref(nd), shape, ctypes.byref(name)))
            self.tensors.append((name.value.decode(), int(off.value),
                                 tuple(int(shape[k]) for k in range(nd.value))))
        z = lambda: torch.zeros(self.flat_size, dtype=torch.float32, device=self.device)  # noqa
        if shared_params is not None:
            if shared_params.numel() != self.flat_size or not shared_params.is_cuda:
                raise ValueError("shared_params must be a device buffer of the same layout")
            self.params = shared_params
        else:
            self.params = z()
        self.grads, self.m, self.v = z(), z(), z()
        check(L.acme_impala_bind(h, ptr(self.params), ptr(self.grads), ptr(self.m),
                                 ptr(self.v)), "impala bind")
        self.metrics = torch.zeros(4, dtype=torch.float32, device=self.device)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().acme_impala_destroy(h)
            except Exception:
                pass
            self._h = None

    views = NativeDQN.views
    get_params = NativeDQN.get_params

    def set_params(self, params: Dict[str, np.ndarray]) -> None:
        for name, t in self.views(self.params).items():
            t.copy_(torch.as_tensor(np.asarray(params[name], np.float32)).view(t.shape))
        self.params_changed()

    def params_changed(self) -> None:
        """The bound parameters were written directly: plane scales recalibrate."""
        check(lib().acme_impala_params_changed(self._h), "impala params_changed")

    @property
    def num_steps(self) -> int:
        return int(lib().acme_impala_num_steps(self._h))

    @num_steps.setter
    def num_steps(self, n: int) -> None:
        check(lib().acme_impala_set_num_steps(self._h, int(n)))

    def debug_buffer(self, name: str) -> np.ndarray:
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        check(lib().acme_impala_debug_buffer(self._h, name.encode(), ctypes.byref(p),
                                             ctypes.byref(n)))
        return _device_array(p.value, n.value, np.float32, self.device).cpu().numpy().view(
            np.float32).copy()

    def plane_overflow(self, reset: bool = False) -> bool:
        """As NativeDQN.plane_overflow, for the Atari torso's plane path."""
        v = ctypes.c_int32(0)
        check(lib().acme_impala_plane_overflow(self._h, ctypes.byref(v), int(reset)),
              "impala plane_overflow")
        return bool(v.value)

    @property
    def skipped_steps(self) -> int:
        """Steps skipped (plane overflow or LSTM timeout) among those the device finished."""
        return int(lib().acme_impala_skipped_steps(self._h))

    def guard_state(self) -> Dict[str, int]:
        """{applied, skipped, last_skipped, lstm_timeouts} (synchronises the device)."""
        a = (ctypes.c_int64 * 4)()
        check(lib().acme_impala_guard_state(self._h, a), "impala guard_state")
        return dict(applied=int(a[0]), skipped=int(a[1]), last_skipped=int(a[2]),
                    lstm_timeouts=int(a[3]))

    @property
    def applied_steps(self) -> int:
        return self.guard_state()["applied"]

    @applied_steps.setter
    def applied_steps(self, n: int) -> None:
        check(lib().acme_impala_set_applied_steps(self._h, int(n)), "impala set_applied_steps")

    def scale_state(self) -> np.ndarray:
        """The plane scales (learner state for checkpoints; empty without the plane path)."""
        n = ctypes.c_int32(0)
        check(lib().acme_impala_scale_state(self._h, None, 0, ctypes.byref(n)), "impala scales")
        out = np.zeros(n.value, np.float32)
        if n.value:
            check(lib().acme_impala_scale_state(self._h, out.ctypes.data, n.value,
                                                ctypes.byref(n)), "impala scales")
        return out

    def set_scale_state(self, state) -> None:
        a = np.ascontiguousarray(np.asarray(state, np.float32))
        if a.size:
            check(lib().acme_impala_set_scale_state(self._h, a.ctypes.data, a.size),
                  "impala set_scale_state")

    def set_policy_planes(self, on: bool = True) -> None:
        """Policy steps (>= 64 rows, Atari torso) on the plane engine: for actor-side networks
        that only run policy steps (acme_impala_set_policy_planes)."""
        check(lib().acme_impala_set_policy_planes(self._h, 1 if on else 0), "policy planes")

    def set_lstm_unroll(self, per_step: bool) -> None:
        """Per-step LSTM launches instead of the one-launch unroll (tests compare the two)."""
        check(lib().acme_impala_set_lstm_unroll(self._h, 1 if per_step else 0), "lstm unroll")

    def step(self, observation, prev_action, prev_reward, action, reward, discount,
             behaviour_logits, h0, c0, stream=None):
        """Batch-major [B, T, ...] device tensors; h0 / c0 are [B, H] views (any row stride
        that is a multiple of 4 floats, e.g. core_state[:, 0] of a [B, T, H] tensor)."""
        B, T = int(action.shape[0]), int(action.shape[1])
        want = torch.uint8 if self.torso == "atari" else torch.float32
        checks = (("observation", observation, want), ("prev_action", prev_action, torch.int32),
                  ("prev_reward", prev_reward, torch.float32), ("action", action, torch.int32),
                  ("reward", reward, torch.float32), ("discount", discount, torch.float32),
                  ("behaviour_logits", behaviour_logits, torch.float32))
        for name, t, dt in checks:
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.is_contiguous()
                    and t.dtype == dt):
                raise ValueError(f"{name} must be a contiguous {dt} device tensor")
            if tuple(t.shape[:2]) != (B, T):
                raise ValueError(f"{name} has shape {tuple(t.shape)}, expected [{B}, {T}, ...]")
        for name, t in (("h0", h0), ("c0", c0)):
            if t.dtype != torch.float32 or t.shape != (B, self.lstm_size) or t.stride(1) != 1:
                raise ValueError(f"{name} must be float32 [{B}, {self.lstm_size}] with unit "
                                 "inner stride")
        if h0.stride(0) != c0.stride(0):
            raise ValueError("h0 and c0 must share a row stride")
        b = _lib.SequenceBatch()
        b.observation, b.prev_action, b.prev_reward = ptr(observation), ptr(prev_action), ptr(prev_reward)
        b.action, b.reward, b.discount = ptr(action), ptr(reward), ptr(discount)
        b.behaviour_logits, b.h0, b.c0 = ptr(behaviour_logits), ptr(h0), ptr(c0)
        b.state_stride, b.batch, b.sequence_length = int(h0.stride(0)), B, T
        check(lib().acme_impala_step(self._h, ctypes.byref(b), ptr(self.metrics),
                                     stream_ptr(stream)), "impala step")

    def policy_step(self, obs, prev_action, prev_reward, h, c, stream=None, out=None):
        """One network step for `rows` actors; returns (logits, values, h, c) (into `out`,
        four contiguous device tensors of those shapes, when given)."""
        rows = int(prev_action.shape[0])
        A, H = self.num_actions, self.lstm_size
        if out is None:
            out = [torch.empty(rows, A, dtype=torch.float32, device=self.device),
                   torch.empty(rows, dtype=torch.float32, device=self.device),
                   torch.empty(rows, H, dtype=torch.float32, device=self.device),
                   torch.empty(rows, H, dtype=torch.float32, device=self.device)]
        check(lib().acme_impala_policy_step(
            self._h, ptr(obs.contiguous()), ptr(prev_action.contiguous()),
            ptr(prev_reward.contiguous()), ptr(h.contiguous()), ptr(c.contiguous()), rows,
            *[ptr(o) for o in out], stream_ptr(stream)), "impala policy_step")
        return tuple(out)


class NativeR2D2:
    """acme_r2d2 learner + its flat buffers (params, target, grads, Adam m / v):
    R2D2Learner._step (acme/agents/tf/r2d2/learning.py:112-200) on R2D2AtariNetwork."""

    def __init__(self, *, num_actions: int, max_batch: int, max_sequence_length: int,
                 burn_in_length: int, torso: str = "atari", obs_dim: int = 0,
                 lstm_size: int = 512, head_size: int = 512, n_step: int = 5,
                 discount: float = 0.99, importance_sampling_exponent: float = 0.2,
                 max_replay_size: int = 1_000_000, max_priority_weight: float = 0.9,
                 target_update_period: int = 100, learning_rate: float = 1e-3,
                 adam_beta1: float = 0.9, adam_beta2: float = 0.999, adam_epsilon: float = 1e-3,
                 store_lstm_state: bool = True, device=None):
        """Defaults are R2D2Learner's (learning.py:47-66; snt.Adam epsilon 1e-3, :78)."""
        _lib.require_gpu()
        cfg = _lib.R2D2Config()
        cfg.torso = _lib.IMPALA_TORSO_ATARI if torso == "atari" else _lib.IMPALA_TORSO_FLAT
        cfg.obs_dim, cfg.num_actions = int(obs_dim), int(num_actions)
        cfg.max_batch, cfg.max_sequence_length = int(max_batch), int(max_sequence_length)
        cfg.burn_in_length = int(burn_in_length)
        cfg.lstm_size, cfg.head_size, cfg.n_step = int(lstm_size), int(head_size), int(n_step)
        cfg.store_lstm_state = 1 if store_lstm_state else 0
        cfg.target_update_period = int(target_update_period)
        cfg.max_replay_size = int(max_replay_size)
        cfg.discount = discount
        cfg.importance_sampling_exponent = importance_sampling_exponent
        cfg.max_priority_weight = max_priority_weight
        cfg.learning_rate = learning_rate
        cfg.adam_beta1, cfg.adam_beta2, cfg.adam_epsilon = adam_beta1, adam_beta2, adam_epsilon
        self.cfg = cfg
        self.torso, self.obs_dim = torso, int(obs_dim)
        self.num_actions, self.lstm_size = int(num_actions), int(lstm_size)
        self.max_batch, self.max_sequence_length = int(max_batch), int(max_sequence_length)
        self.burn_in_length = int(burn_in_length)
        self.store_lstm_state = bool(store_lstm_state)
        self.device = torch.device(device or "cuda")
        h = ctypes.c_void_p()
        L = lib()
        with torch.cuda.device(self.device):
            check(L.acme_r2d2_create(ctypes.byref(cfg), ctypes.byref(h)), "r2d2 create")
        self._h = h
        self.flat_size = int(L.acme_r2d2_flat_size(h))
        self.tensors: List[Tuple[str, int, Tuple[int, ...]]] = []
        for i in range(L.acme_r2d2_num_tensors(h)):
            off, numel, nd = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
            shape = (ctypes.c_int64 * 4)()
            name = ctypes.c_char_p()
            check(L.acme_r2d2_tensor_info(h, i, ctypes.byref(off), ctypes.byref(numel),
                                          ctypes.byref(nd), shape, ctypes.byref(name)))
            self.tensors.append((name.value.decode(), int(off.value),
                                 tuple(int(shape[k]) for k in range(nd.value))))
        z = lambda: torch.zeros(self.flat_size, dtype=torch.float32, device=self.device)  # noqa
        self.params, self.target, self.grads, self.m, self.v = z(), z(), z(), z(), z()
        check(L.acme_r2d2_bind(h, ptr(self.params), ptr(self.target), ptr(self.grads),
                               ptr(self.m), ptr(self.v)), "r2d2 bind")
        T, B = self.max_sequence_length, self.max_batch
        self.loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        self._errors = torch.zeros(max(T - self.burn_in_length - 1, 1) * B, dtype=torch.float32,
                                   device=self.device)
        self._last = (1, B)
        self.priorities = torch.zeros(B, dtype=torch.float64, device=self.device)

    @property
    def errors(self) -> torch.Tensor:
        """The last step's errors [T - burn_in - 1, B] (time-major, extra.errors)."""
        tm, b = self._last
        return self._errors[:tm * b].view(tm, b)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().acme_r2d2_destroy(h)
            except Exception:
                pass
            self._h = None

    views = NativeDQN.views
    get_params = NativeDQN.get_params

    def set_params(self, params: Dict[str, np.ndarray], target: Dict[str, np.ndarray]) -> None:
        for buf, src in ((self.params, params), (self.target, target)):
            for name, t in self.views(buf).items():
                t.copy_(torch.as_tensor(np.asarray(src[name], np.float32)).view(t.shape))
        self.params_changed()

    def params_changed(self) -> None:
        """The bound buffers were written directly: the plane scales recalibrate."""
        check(lib().acme_r2d2_params_changed(self._h), "r2d2 params_changed")

    @property
    def skipped_steps(self) -> int:
        """Steps skipped on plane overflow among those the device finished."""
        return int(lib().acme_r2d2_skipped_steps(self._h))

    def scale_state(self) -> np.ndarray:
        """The plane scales (learner state for checkpoints; empty without the plane path)."""
        n = ctypes.c_int32(0)
        check(lib().acme_r2d2_scale_state(self._h, None, 0, ctypes.byref(n)), "r2d2 scales")
        out = np.zeros(n.value, np.float32)
        if n.value:
            check(lib().acme_r2d2_scale_state(self._h, out.ctypes.data, n.value,
                                              ctypes.byref(n)), "r2d2 scales")
        return out

    def set_scale_state(self, state) -> None:
        """Restores scale_state() (after params_changed): resumed steps are bit-identical."""
        a = np.ascontiguousarray(np.asarray(state, np.float32))
        if a.size:
            check(lib().acme_r2d2_set_scale_state(self._h, a.ctypes.data, a.size),
                  "r2d2 set_scale_state")

    def guard_state(self) -> Dict[str, int]:
        """{applied, skipped, last_skipped} (synchronises the device)."""
        a = (ctypes.c_int64 * 3)()
        check(lib().acme_r2d2_guard_state(self._h, a), "r2d2 guard_state")
        return dict(applied=int(a[0]), skipped=int(a[1]), last_skipped=int(a[2]))

    def set_applied_steps(self, n: int) -> None:
        check(lib().acme_r2d2_set_applied_steps(self._h, int(n)), "r2d2 set_applied_steps")

    @property
    def skip_word(self) -> Optional[int]:
        """Device address of the step's skip word (gates the priority write-back), or None."""
        return lib().acme_r2d2_skip_word(self._h) or None

    @property
    def num_steps(self) -> int:
        return int(lib().acme_r2d2_num_steps(self._h))

    @num_steps.setter
    def num_steps(self, n: int) -> None:
        check(lib().acme_r2d2_set_num_steps(self._h, int(n)))

    def set_lstm_unroll(self, per_step: bool) -> None:
        """per_step=True: one LSTM launch per time step instead of the one-launch unroll."""
        check(lib().acme_r2d2_set_lstm_unroll(self._h, 1 if per_step else 0), "r2d2 lstm unroll")

    def debug_buffer(self, name: str) -> np.ndarray:
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        check(lib().acme_r2d2_debug_buffer(self._h, name.encode(), ctypes.byref(p),
                                           ctypes.byref(n)))
        return _device_array(p.value, n.value, np.float32, self.device).cpu().numpy().view(
            np.float32).copy()

    def step(self, observation, prev_action, prev_reward, action, reward, discount,
             probabilities, h0=None, c0=None, stream=None):
        """Batch-major [B, T, ...] device tensors (the sequence dataset's layout: the OAR
        observation's frames, previous action and reward; action, reward, discount), the
        sample's probabilities [B] (f64) and the core state at t = 0 (h0 / c0 [B, H] views
        with unit inner stride; ignored with store_lstm_state=False).  Loss, errors
        [T - burn_in - 1, B] and priorities [B] land in .loss / .errors / .priorities."""
        B, T = int(action.shape[0]), int(action.shape[1])
        want = torch.uint8 if self.torso == "atari" else torch.float32
        checks = (("observation", observation, want), ("prev_action", prev_action, torch.int32),
                  ("prev_reward", prev_reward, torch.float32), ("action", action, torch.int32),
                  ("reward", reward, torch.float32), ("discount", discount, torch.float32))
        for name, t, dt in checks:
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.is_contiguous()
                    and t.dtype == dt):
                raise ValueError(f"{name} must be a contiguous {dt} device tensor")
            if tuple(t.shape[:2]) != (B, T):
                raise ValueError(f"{name} has shape {tuple(t.shape)}, expected [{B}, {T}, ...]")
        if not (probabilities.is_cuda and probabilities.dtype == torch.float64
                and probabilities.is_contiguous() and probabilities.numel() == B):
            raise ValueError(f"probabilities must be a contiguous float64 [{B}] device tensor")
        b = _lib.SequenceBatch()
        b.observation, b.prev_action, b.prev_reward = ptr(observation), ptr(prev_action), ptr(prev_reward)
        b.action, b.reward, b.discount = ptr(action), ptr(reward), ptr(discount)
        b.behaviour_logits = None
        if self.store_lstm_state:
            for name, t in (("h0", h0), ("c0", c0)):
                if (t is None or t.dtype != torch.float32 or t.shape != (B, self.lstm_size)
                        or t.stride(1) != 1):
                    raise ValueError(f"{name} must be float32 [{B}, {self.lstm_size}] with unit "
                                     "inner stride")
            if h0.stride(0) != c0.stride(0):
                raise ValueError("h0 and c0 must share a row stride")
            b.h0, b.c0, b.state_stride = ptr(h0), ptr(c0), int(h0.stride(0))
        else:
            b.h0 = b.c0 = None
            b.state_stride = self.lstm_size
        b.batch, b.sequence_length = B, T
        o = _lib.R2D2Outputs()
        o.loss, o.errors, o.priorities = ptr(self.loss), ptr(self._errors), ptr(self.priorities)
        self._last = (T - self.burn_in_length - 1, B)
        check(lib().acme_r2d2_step(self._h, ctypes.byref(b), ptr(probabilities), ctypes.byref(o),
                                   stream_ptr(stream)), "r2d2 step")
