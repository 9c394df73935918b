"""In-process, GPU-resident replacement for the Reverb surface the agents use.

Reference call sites (all in-process `localhost:<port>` gRPC in the reference):
  reverb.Table(name, sampler=Prioritized(a) | Uniform(), remover=Fifo(), max_size,
               rate_limiter=MinSize(n), signature)        acme/agents/tf/dqn/agent.py:95-101
  reverb.Table.queue(name, max_size)                       acme/agents/tf/impala/agent.py:68-74
                                                           (device FIFO, QueueTable)
  reverb.Server([tables], port=None).port                  acme/agents/tf/dqn/agent.py:102
  reverb.Client(address).writer(...) -> append/create_item acme/adders/reverb/base.py:112-118
  reverb.TFClient(address).update_priorities(table, keys, priorities)
                                                           acme/agents/tf/dqn/learning.py:151-154
  Client.mutate_priorities(table, updates)                 acme/agents/jax/dqn/learning.py:131-134
  ReplaySample(info=SampleInfo(key, probability, table_size, priority), data)

Items live in HBM (acme_amd.native.NativeReplay: one row per item per flattened field,
64-ary sum tree for Prioritized).  Writers stage items on the host and flush them in
batches straight into the table's pinned staging ring (side-stream hipMemcpyAsync, no
host wait); a table flushes pending items before every sample, so a sample always sees
every item created before it.
"""

from __future__ import annotations

import collections
import itertools
import threading
import time
import weakref
from typing import Any, Dict, List, NamedTuple, Optional, Sequence

import numpy as np

from acme_amd.utils import tree


class SampleInfo(NamedTuple):
    key: Any
    probability: Any
    table_size: Any
    priority: Any


class ReplaySample(NamedTuple):
    info: SampleInfo
    data: Any


# ---------------------------------------------------------------- selectors / limiters
class selectors:  # noqa: N801  (module-like namespace, as reverb.selectors)
    class Prioritized(NamedTuple):
        priority_exponent: float

    class Uniform(NamedTuple):
        pass

    class Fifo(NamedTuple):
        pass

    class Lifo(NamedTuple):
        pass


class rate_limiters:  # noqa: N801
    class MinSize(NamedTuple):
        min_size_to_sample: int

    class Queue(NamedTuple):
        size: int


# ---------------------------------------------------------------- field layout
class _Field(NamedTuple):
    shape: tuple
    dtype: np.dtype
    nbytes: int       # logical bytes per item
    row_bytes: int    # stored bytes per item (multiple of 4)


def _row_bytes(nbytes: int, itemsize: int) -> int:
    align = max(4, itemsize)
    return max(align, (nbytes + align - 1) // align * align)


def _layout_from_item(item) -> List[_Field]:
    out = []
    for leaf in tree.flatten(item):
        a = np.asarray(leaf)
        nb = int(a.nbytes)
        out.append(_Field(tuple(a.shape), a.dtype, nb, _row_bytes(nb, a.dtype.itemsize)))
    return out


def _layout_from_signature(signature) -> List[_Field]:
    out = []
    for s in tree.flatten(signature):
        dt = np.dtype(s.dtype)
        nb = int(np.prod(s.shape, dtype=np.int64)) * dt.itemsize
        out.append(_Field(tuple(s.shape), dt, nb, _row_bytes(nb, dt.itemsize)))
    return out


# ---------------------------------------------------------------- table
class Table:
    """A named GPU replay table (Reverb Table semantics for the transition path)."""

    def __init__(self, name: str, sampler, remover, max_size: int, rate_limiter=None,
                 signature=None, seed: int = 1234, device=None, flush_every: int = 256):
        if not isinstance(remover, (selectors.Fifo,)):
            raise ValueError("only the Fifo remover is supported (as used by the agents)")
        if isinstance(sampler, selectors.Prioritized):
            self._prioritized, self._alpha = True, float(sampler.priority_exponent)
        elif isinstance(sampler, selectors.Uniform):
            self._prioritized, self._alpha = False, 0.0
        else:
            raise ValueError(f"unsupported sampler {sampler!r}")
        self.name = name
        self.max_size = int(max_size)
        self._min_size = rate_limiter.min_size_to_sample if rate_limiter is not None else 1
        self._signature = signature
        self._structure = None
        self._fields: Optional[List[_Field]] = None
        self._native = None
        self._seed = int(seed)
        self._device = device
        self._flush_every = max(1, int(flush_every))
        # Items accepted but not yet committed: row i of every field's host buffer (packed
        # at insert, one copy per field), copied to the native table's pinned staging chunk
        # in one block per field at flush.
        self._pend: Optional[List[np.ndarray]] = None
        self._pend_prio = np.zeros(self._flush_every, np.float64)
        self._fill = 0
        # Native n-step writers feeding this table (NStepTransitionAdder's fast path): their
        # pending rows count towards size() and a flush() commits them.
        self._writers = weakref.WeakSet()
        self._mu = threading.RLock()
        self._cv = threading.Condition(self._mu)
        self._draws = 0
        self._seq_len: Optional[int] = None
        # The last sample/gather a prefetching dataset issued on its own stream: writers
        # (priority updates, inserts) order the caller's stream after it, so a queued draw
        # never reads a half-updated tree or a slot being overwritten.
        self._reader_event = None
        if signature is not None:
            self._init_layout(signature, _layout_from_signature(signature))

    @classmethod
    def queue(cls, name: str, max_size: int, signature=None, device=None):
        return QueueTable(name, max_size, signature, device=device)

    # -- layout / storage
    def _init_layout(self, structure, fields):
        from acme_amd.native import NativeReplay
        self._structure = structure
        self._fields = fields
        self._flat_tuple = (isinstance(structure, tuple) and not hasattr(structure, "_fields")
                            and len(structure) == len(fields))
        self._pend = [np.zeros((self._flush_every, f.row_bytes), np.uint8) for f in fields]
        self._fill = 0
        self._native = NativeReplay(self.max_size, [f.row_bytes for f in fields],
                                    prioritized=self._prioritized, priority_exponent=self._alpha,
                                    seed=self._seed, device=self._device)

    @property
    def native(self):
        return self._native

    @property
    def fields(self):
        return self._fields

    def size(self) -> int:
        with self._mu:
            n = self._native.size() if self._native is not None else 0
            return min(self.max_size, n + self._fill + sum(w.pending() for w in self._writers))

    def committed_size(self) -> int:
        """Items on the device (what a draw can return now)."""
        return self._native.size() if self._native is not None else 0

    def register_writer(self, writer) -> None:
        with self._mu:
            self._writers.add(writer)

    def can_sample(self, num_samples: int = 1) -> bool:
        return self.size() >= max(self._min_size, 1)

    # -- inserts
    def insert(self, item, priority: float) -> None:
        with self._mu:
            if self._fields is None:
                self._init_layout(item, _layout_from_item(item))
            # A flat tuple item (the transition adder's) is its own leaf list.
            leaves = (item if self._flat_tuple and type(item) is tuple
                      and len(item) == len(self._fields) else tree.flatten(item))
            if len(leaves) != len(self._fields):
                raise ValueError(f"item has {len(leaves)} leaves, table expects "
                                 f"{len(self._fields)}")
            self._maybe_sequence_layout(leaves)
            r = self._fill
            for leaf, f, buf in zip(leaves, self._fields, self._pend):
                a = leaf if type(leaf) is np.ndarray and leaf.dtype == f.dtype else \
                    np.asarray(leaf, dtype=f.dtype)
                if a.shape != f.shape:
                    raise ValueError(f"leaf shape {a.shape} does not match table signature "
                                     f"{f.shape}")
                # One copy into the row (the bytes, in C order); the row padding stays 0.
                buf[r, :f.nbytes].view(f.dtype).reshape(f.shape)[...] = a
            self._pend_prio[r] = priority
            self._fill = r + 1
            if self._fill >= self._flush_every:
                self.flush()
            self._cv.notify_all()

    def _maybe_sequence_layout(self, leaves) -> None:
        """Sequence items (SequenceAdder, R2D2): Reverb signatures are per timestep
        (adders/reverb/base.py:179-206) and the table stores T-step items.  The first item
        whose every leaf is [T] + the signature's shape fixes the stored layout to T steps."""
        if self._seq_len is not None or self._fill or self._native.size() > 0:
            return
        shapes = [np.shape(x) for x in leaves]
        if all(s == f.shape for s, f in zip(shapes, self._fields)):
            self._seq_len = 0
            return
        T = shapes[0][0] if shapes[0] else None
        if T is None or not all(len(s) == len(f.shape) + 1 and s[0] == T and s[1:] == f.shape
                                for s, f in zip(shapes, self._fields)):
            return  # a genuine mismatch: reported by the caller's shape check
        self._seq_len = int(T)
        seq = [_Field((T,) + f.shape, f.dtype, T * f.nbytes, _row_bytes(T * f.nbytes,
                                                                      f.dtype.itemsize))
               for f in self._fields]
        self._native = None
        self._init_layout(self._structure, seq)

    def set_sequence_length(self, T: int) -> None:
        """Fixes the stored layout to T-step items before the first insert (what the first
        SequenceAdder item would do), e.g. for writers that pack rows themselves."""
        with self._mu:
            if self._seq_len == T:
                return
            if self._seq_len is not None or self._fill or self._native.size() > 0:
                raise ValueError("the table's layout is already fixed")
            self._maybe_sequence_layout([np.zeros((T,) + f.shape, f.dtype) for f in self._fields])

    @property
    def sequence_length(self) -> Optional[int]:
        """Steps per item for sequence tables (None until the first item, 0 if not)."""
        return self._seq_len

    def set_reader_event(self, event) -> None:
        """Called by a prefetching dataset after it issues device reads of this table."""
        self._reader_event = event

    def _after_readers(self) -> None:
        """Orders the current stream after the last issued prefetch read (a no-op when it
        has already completed, which is the steady state: a batch is issued P steps ahead)."""
        ev = self._reader_event
        if ev is not None and not ev.query():
            import torch
            torch.cuda.current_stream(self._native.device).wait_event(ev)

    def flush(self) -> None:
        """Commits the pending rows: one native call packs each field's block into the
        table's pinned staging chunk (a C memcpy outside the GIL) and issues hipMemcpyAsync
        on the table's side stream, no host wait.  The native table orders the copies after
        every stream that has read it (a queued prefetch gather never sees a slot
        overwritten under it) and every later sample after them."""
        with self._mu:
            for w in list(self._writers):
                w.flush()
            n = self._fill
            if not n:
                return
            self._native.insert([p[:n] for p in self._pend], self._pend_prio[:n])
            self._fill = 0

    # Pending rows older than this are committed by the next draw (bounded staleness).
    max_pending_seconds = 0.1

    def flush_for_sampling(self, batch_size: int) -> None:
        """A reader's flush: commits pending rows when the device table could not serve the
        draw without them (it holds fewer than the batch or MinSize), or when rows have been
        pending for longer than max_pending_seconds (a slow writer's rows become sampleable
        within that bound).  Otherwise rows become visible when their writer's buffer fills
        or the writer closes, as Reverb chunks do, so the learner's thread does not pack or
        issue the actors' inserts in the steady state."""
        with self._mu:
            if self.committed_size() < max(batch_size, self._min_size, 1):
                self.flush()
                self._pending_since = None
                return
            if not (self._fill or any(w.pending() for w in self._writers)):
                self._pending_since = None
                return
            now = time.monotonic()
            since = getattr(self, "_pending_since", None)
            if since is None:
                self._pending_since = now
            elif now - since > self.max_pending_seconds:
                self.flush()
                self._pending_since = None

    # -- checkpointing (optional replay state; core.Saveable interface)
    def save(self) -> Dict[str, Any]:
        """The live items, their keys and raw priorities, the insert and draw counters (a
        1M-slot Atari table is ~56 GB: include a table in a Checkpointer only on purpose)."""
        with self._mu:
            self.flush()
            if self._native is None:
                return {"draws": np.int64(self._draws)}
            state = self._native.export_state()
            state["draws"] = np.int64(self._draws)
            return state

    def restore(self, state: Dict[str, Any]) -> None:
        with self._mu:
            self._fill = 0
            if "keys" in state:
                if self._native is None:
                    raise ValueError("restore needs the table layout (construct the table "
                                     "with its signature)")
                self._after_readers()
                self._native.import_state(state)
            self._draws = int(state["draws"])

    # -- sampling
    def wait_for(self, batch_size: int, timeout: float) -> None:
        """Rate limiter MinSize: block until enough items exist (or time out)."""
        deadline = time.time() + timeout
        with self._cv:
            while self.size() < max(self._min_size, 1):
                left = deadline - time.time()
                if left <= 0:
                    raise RuntimeError(f"table '{self.name}' has {self.size()} items; "
                                       f"MinSize({self._min_size}) not reached within {timeout}s")
                # Native writers add without notifying: poll.
                self._cv.wait(min(left, 0.01))

    def next_draw(self) -> int:
        with self._mu:
            d = self._draws
            self._draws += 1
            return d

    def prepare_priority_update(self, keys):
        """For a learner that writes the batch's priorities back inside its step
        (acme_dqn_step_update): (native handle, device uint64 keys, raw event of the last
        prefetch read still in flight or None), the read the update must follow (as
        update_priorities orders the current stream after it); None when the table holds
        nothing to update."""
        import torch
        with self._mu:
            if self._native is None:
                return None
            k = keys if isinstance(keys, torch.Tensor) else torch.as_tensor(
                np.asarray(keys, np.uint64).view(np.int64)).view(torch.uint64)
            k = k.to(self._native.device).contiguous()
            if k.dtype == torch.int64:
                k = k.view(torch.uint64)
            ev = self._reader_event
            after = None
            if ev is not None and not ev.query():
                after = ev.handle if hasattr(ev, "handle") else int(ev.cuda_event)
            return self._native.handle, k, after

    def update_priorities(self, keys, priorities, skip_word=None) -> None:
        """skip_word (extension): a learner's device skip word; the update is dropped when
        the step that produced the priorities was skipped (NativeDQN.skip_word)."""
        import torch
        with self._mu:
            # Pending rows hold no keys yet: nothing to flush for an update.
            if self._native is None:
                return
            k = keys if isinstance(keys, torch.Tensor) else torch.as_tensor(
                np.asarray(keys, np.uint64).view(np.int64)).view(torch.uint64)
            p = priorities if isinstance(priorities, torch.Tensor) else torch.as_tensor(
                np.asarray(priorities, np.float64))
            self._after_readers()
            self._native.update_priorities(k, p, skip_word=skip_word)


from acme_amd.replay.frame_table import _make_frame_table  # noqa: E402

FrameTable = _make_frame_table(Table, _Field, _layout_from_signature)


class QueueTable(Table):
    """Table.queue (acme/agents/tf/impala/agent.py:68-74): a FIFO whose items are consumed
    once, device-resident.  Items (SequenceAdder sequences) go through the same pinned
    staging ring and side-stream copies as Table inserts, into an HBM ring of max_size
    slots; `pop_slots(B)` hands the next B items to the dataset, which gathers them on the
    GPU (rows of consecutive ring slots).  Reverb's Queue rate limiter blocks a writer while
    the queue is full and a reader while it holds fewer than the batch; so do insert() and
    pop_slots() (with a timeout).  An item's slot is reused only after its gather: the
    native table orders every insert after the streams that read it."""

    def __init__(self, name: str, max_size: int, signature=None, device=None,
                 flush_every: int = 16, timeout: float = 60.0):
        super().__init__(name, selectors.Uniform(), selectors.Fifo(), max_size, None,
                         signature=signature, device=device, flush_every=flush_every)
        self._accepted = 0   # items insert() took (pending or flushed)
        self._consumed = 0   # items handed to readers
        self._timeout = float(timeout)

    def size(self) -> int:
        with self._mu:
            return self._accepted - self._consumed

    def can_sample(self, num_samples: int = 1) -> bool:
        return self.size() >= num_samples

    def insert(self, item, priority: float) -> None:
        deadline = time.time() + self._timeout
        with self._cv:
            while self._accepted - self._consumed >= self.max_size:
                self.flush()
                left = deadline - time.time()
                if left <= 0:
                    raise RuntimeError(f"queue '{self.name}' stayed full ({self.max_size} items) "
                                       f"for {self._timeout}s")
                self._cv.wait(left)
            super().insert(item, priority)
            self._accepted += 1

    def insert_rows(self, rows: Sequence[np.ndarray], n: int) -> None:
        """n items already packed as the table's rows (rows[f]: uint8 [n, row_bytes[f]],
        e.g. a shared-memory ring of actor processes): one native insert, FIFO after every
        earlier item; blocks while the queue is full, as insert() does."""
        if n <= 0:
            return
        deadline = time.time() + self._timeout
        with self._cv:
            while self._accepted - self._consumed + n > self.max_size:
                self.flush()
                left = deadline - time.time()
                if left <= 0:
                    raise RuntimeError(f"queue '{self.name}' stayed full ({self.max_size} items) "
                                       f"for {self._timeout}s")
                self._cv.wait(min(left, 0.01))
            self.flush()  # earlier single inserts first (FIFO)
            for r, f in zip(rows, self._fields):
                if r.shape != (n, f.row_bytes):
                    raise ValueError(f"rows {r.shape} do not match the table's {(n, f.row_bytes)}")
            self._native.insert(list(rows), None)
            self._accepted += n
            self._cv.notify_all()

    def pop_slots(self, batch_size: int, timeout: Optional[float] = None,
                  read=None) -> int:
        """Blocks until `batch_size` items are queued, flushes them to the device and
        consumes them; returns the insertion index of the first one (its ring slot is that
        index modulo max_size, the next ones follow).  `read(first)` issues the device reads
        of those slots: it runs under the table lock BEFORE the slots are released to
        writers, so the native table orders any later insert into them after the reads (a
        writer blocked on a full queue cannot overwrite a slot whose gather is not yet on a
        stream)."""
        if batch_size > self.max_size:
            raise ValueError(f"batch {batch_size} exceeds the queue capacity {self.max_size}")
        deadline = time.time() + (self._timeout if timeout is None else timeout)
        with self._cv:
            while self._accepted - self._consumed < batch_size:
                left = deadline - time.time()
                if left <= 0:
                    raise RuntimeError(f"queue '{self.name}' has {self.size()} items, "
                                       f"{batch_size} requested")
                self._cv.wait(left)
            self.flush()
            first = self._consumed
            if read is not None:
                read(first)
            self._consumed += batch_size
            self._cv.notify_all()
            return first

    def pop_batch(self, batch_size: int, timeout: float = 60.0):
        raise NotImplementedError("the device queue is read through make_reverb_dataset")

    # A queue's items are consumed once and its counters live beside the ring: the plain
    # Table export would restore a ring the counters do not describe.  The reference's
    # IMPALA agent checkpoints the learner only (agents/tf/impala/agent.py), never its queue.
    def save(self) -> Dict[str, Any]:
        raise NotImplementedError(f"queue table '{self.name}' is not checkpointable "
                                  f"(its items are consumed once; checkpoint the learner)")

    def restore(self, state: Dict[str, Any]) -> None:
        raise NotImplementedError(f"queue table '{self.name}' is not checkpointable "
                                  f"(its items are consumed once; checkpoint the learner)")

    def update_priorities(self, keys, priorities, skip_word=None) -> None:
        pass  # queue items carry no priorities (Reverb ignores updates of consumed items)

    def prepare_priority_update(self, keys):
        return None


# ---------------------------------------------------------------- server / client
_SERVERS: Dict[int, "Server"] = {}
_PORTS = itertools.count(30000)


class Server:
    def __init__(self, tables: Sequence[Any], port: Optional[int] = None):
        self.tables = {t.name: t for t in tables}
        self.port = int(port) if port is not None else next(_PORTS)
        _SERVERS[self.port] = self

    def stop(self):
        _SERVERS.pop(self.port, None)

    def in_process_client(self) -> "Client":
        return Client(self)


def _resolve(address) -> Server:
    if isinstance(address, Server):
        return address
    if isinstance(address, (Table, QueueTable)):
        return _wrap_table(address)
    port = int(str(address).rsplit(":", 1)[-1])
    if port not in _SERVERS:
        raise ValueError(f"no replay server at {address!r}")
    return _SERVERS[port]


def _wrap_table(table) -> Server:
    s = Server.__new__(Server)
    s.tables = {table.name: table}
    s.port = -1
    return s


class Writer:
    """Reverb Writer surface: append(data), create_item(table, num_timesteps, priority)."""

    def __init__(self, server: Server, max_sequence_length: int):
        self._server = server
        self._history: collections.deque = collections.deque(maxlen=max_sequence_length)
        self.max_sequence_length = max_sequence_length
        self.closed = False

    def append(self, data):
        if self.closed:
            raise RuntimeError("append on a closed writer")
        self._history.append(data)

    def create_item(self, table: str, num_timesteps: int, priority: float):
        if self.closed:
            raise RuntimeError("create_item on a closed writer")
        if num_timesteps < 1 or num_timesteps > len(self._history):
            raise ValueError(f"num_timesteps={num_timesteps} but only {len(self._history)} "
                             "steps are available")
        steps = list(self._history)[-num_timesteps:]
        item = steps[0] if num_timesteps == 1 else tree.map_structure(
            lambda *xs: np.stack([np.asarray(x) for x in xs]), *steps)
        self._server.tables[table].insert(item, priority)

    def flush(self):
        for t in self._server.tables.values():
            t.flush()

    def close(self):
        if not self.closed:
            self.flush()
            self.closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Client:
    """reverb.Client / reverb.TFClient surface over the in-process server."""

    def __init__(self, server_address):
        self._server = _resolve(server_address)

    @property
    def server(self) -> Server:
        return self._server

    def writer(self, max_sequence_length: int, delta_encoded: bool = False,
               chunk_length: Optional[int] = None) -> Writer:
        del delta_encoded, chunk_length  # compression knobs of the gRPC path: not needed
        return Writer(self._server, max_sequence_length)

    def insert(self, data, priorities: Dict[str, float]):
        for table, p in priorities.items():
            self._server.tables[table].insert(data, p)

    def prepare_priority_update(self, table: str, keys):
        """(native handle, device keys) for a learner step that writes the priorities back
        itself (Table.prepare_priority_update), or None."""
        t = self._server.tables[table]
        prep = getattr(t, "prepare_priority_update", None)
        return prep(keys) if prep is not None else None

    def update_priorities(self, table: str, keys, priorities, skip_word=None):
        """TFClient.update_priorities: device or host keys (u64) / priorities (f64).
        skip_word (extension): see Table.update_priorities."""
        if skip_word is None:
            self._server.tables[table].update_priorities(keys, priorities)
        else:
            self._server.tables[table].update_priorities(keys, priorities, skip_word=skip_word)

    def mutate_priorities(self, table: str, updates: Optional[Dict[int, float]] = None,
                          deletes: Optional[Sequence[int]] = None):
        if deletes:
            raise NotImplementedError("item deletion is not supported by the GPU table")
        if updates:
            keys = np.fromiter(updates.keys(), np.uint64, len(updates))
            pr = np.fromiter(updates.values(), np.float64, len(updates))
            self._server.tables[table].update_priorities(keys, pr)

    def server_info(self):
        return {name: dict(current_size=t.size(), max_size=t.max_size)
                for name, t in self._server.tables.items()}


TFClient = Client
