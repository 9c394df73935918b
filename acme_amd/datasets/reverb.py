"""make_reverb_dataset — drop-in for acme/datasets/reverb.py:36-139.

The reference streams every sample through gRPC, decompresses it on a tf.data thread,
batches on the host and copies the batch to the device.  Here a batch is drawn and
gathered on the GPU: one sampling kernel (prioritized 64-ary sum tree or uniform) and
one row-gather per field into device buffers, so `next(iterator)` returns a
ReplaySample whose data are device tensors.  A sample stays valid until the iterator is
advanced twice.

`prefetch_size` keeps the reference's tf.data prefetch (datasets/reverb.py:136-137; the
DQN agent asks for 4, agents/tf/dqn/agent.py:50): with P > 0 the sample and gather of batch
k + P are issued on the dataset's own stream when batch k is handed out, ordered after
every kernel already queued on the caller's stream (so they see the priority updates of
steps < k, like Reverb's prefetched samples), and the caller's stream waits only for the
batch it receives.  Priority updates in turn order the caller's stream after the last
issued prefetch (Table._after_readers), and host inserts are ordered after every stream
that has read the table (inside the native table, csrc/replay.hip), so a queued draw never
overlaps a tree update or a slot overwrite; a draw and its row gather are one unit with
respect to inserts (acme_replay_sample_gather).  The draw order, and so every sampled
index, is deterministic for a given interleaving of inserts.  With P >= 2 on the transition
layout the draws are pipelined (acme_replay_sample_gather_pipe): batch k + P's rows are
copied by batch k + P + 1's launch, beside that draw's tree descent; an insert issues the
pending copy before it lands, so the rows are still those of the drawn keys.

`server_address` may be the in-process address ('localhost:<port>'), a Server, a Table
or a Client.  Sampling is deterministic given the table seed: draw i uses Philox
counter block i.
"""

from __future__ import annotations

import os
from typing import Any, Optional, Tuple

import numpy as np
import torch

from acme_amd import replay
from acme_amd.adders import reverb as adders
from acme_amd.replay.sharding import LAG as _LAG
from acme_amd.replay.sharding import allocate_shares
from acme_amd.utils import tree

_TORCH = {np.dtype(k): v for k, v in [
    ("uint8", torch.uint8), ("int8", torch.int8), ("int16", torch.int16),
    ("int32", torch.int32), ("int64", torch.int64), ("float16", torch.float16),
    ("float32", torch.float32), ("float64", torch.float64), ("bool", torch.bool),
    ("uint64", torch.uint64), ("uint32", torch.uint32)]}


class TensorSpec:
    """Shape (None for a dimension known only at run time) and dtype of a yielded tensor:
    the role tf.TensorSpec plays in the reference's dataset.element_spec (a leaf, not a
    tuple, for acme_amd.utils.tree)."""
    __slots__ = ("shape", "dtype")

    def __init__(self, shape: Tuple[Optional[int], ...], dtype: Any):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)

    def __eq__(self, other) -> bool:
        return (isinstance(other, TensorSpec) and self.shape == other.shape
                and self.dtype == other.dtype)

    def __repr__(self) -> str:
        return f"TensorSpec(shape={self.shape}, dtype={self.dtype})"


def _adder_spec(transition_adder: bool, environment_spec, extra_spec):
    """The structure of the items the adders write (acme/datasets/reverb.py:141-187):
    transitions (o, a, r, d, o', [extras]) or Step(observation, action, reward, discount,
    start_of_episode, extras)."""
    if transition_adder:
        spec = tuple(environment_spec) + (environment_spec.observations,)
        if extra_spec:
            spec += (extra_spec,)
        return spec
    from acme_amd import specs
    return adders.Step(observation=environment_spec.observations,
                       action=environment_spec.actions, reward=environment_spec.rewards,
                       discount=environment_spec.discounts,
                       start_of_episode=specs.Array(shape=(), dtype=bool),
                       extras=() if not extra_spec else extra_spec)


def _element_shapes(adder_spec, sequence_length, convert_zero_size_to_none, batch_size):
    """Per-leaf TensorSpecs as the reference derives them (datasets/reverb.py:189-198; as
    there, convert_zero_size_to_none replaces the sequence dimension rule) with the batch
    dimension of the drop-remainder batching in front."""
    def shape(x):
        if convert_zero_size_to_none:
            s = tuple(d if d else None for d in x.shape)
        elif sequence_length:
            s = (int(sequence_length),) + tuple(x.shape)
        else:
            s = tuple(x.shape)
        return TensorSpec(((int(batch_size),) if batch_size else ()) + s, np.dtype(x.dtype))
    leaves = tree.flatten(adder_spec)
    return tree.unflatten_as(adder_spec, [shape(x) for x in leaves])


def _server_of(address) -> replay.Server:
    if isinstance(address, replay.Client):
        return address.server
    return replay._resolve(address)  # noqa: SLF001


def _data_parallel():
    """(world, rank) of an initialised torch.distributed group with more than one rank."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.get_world_size(), dist.get_rank()
    return None


class ReplayDataset:
    """Iterable over batched ReplaySamples of one table.

    global_sampling (default: on when torch.distributed runs more than one rank): the table
    is this rank's shard of a global replay; each batch is this rank's share of a global draw
    of world * batch_size items (acme_amd.replay.sharding), so it holds a varying number of
    items (at most 2 * batch_size) whose probabilities are their global marginals."""

    def __init__(self, table, batch_size: Optional[int], timeout: float = 60.0, prefetch: int = 0,
                 global_sampling: Optional[bool] = None, data_spec=None):
        if batch_size is not None and batch_size < 1:
            raise ValueError("batch_size must be >= 1 (or None for single items)")
        if prefetch < 0:
            raise ValueError("prefetch_size must be >= 0")
        self.table = table
        # batch_size None: single items without a batch dimension (the reference's
        # unbatched dataset), drawn as batches of one.
        self.batched = batch_size is not None
        self.batch_size = int(batch_size) if batch_size is not None else 1
        self.timeout = timeout
        self.prefetch = int(prefetch)
        self.global_sampling = global_sampling
        self._data_spec = data_spec

    @property
    def element_spec(self) -> replay.ReplaySample:
        """TensorSpecs of what next() yields (tf.data's element_spec): the data from the
        environment spec given to make_reverb_dataset (as the reference), else from the
        table's item layout; the info fields per item."""
        B = (self.batch_size,) if self.batched else ()
        data = self._data_spec
        if data is None:
            t = self.table
            if t.fields is None:
                raise ValueError("element_spec needs an environment_spec or a table signature")
            data = tree.unflatten_as(t._structure, [  # noqa: SLF001
                TensorSpec(B + tuple(f.shape), np.dtype(f.dtype)) for f in t.fields])
        info = replay.SampleInfo(key=TensorSpec(B, np.dtype(np.uint64)),
                                 probability=TensorSpec(B, np.dtype(np.float64)),
                                 table_size=TensorSpec(B, np.dtype(np.int64)),
                                 priority=TensorSpec(B, np.dtype(np.float64)))
        return replay.ReplaySample(info=info, data=data)

    def __iter__(self):
        if isinstance(self.table, replay.QueueTable):
            it = _QueueIterator(self.table, self.batch_size, self.timeout)
        else:
            dp = _data_parallel()
            shard = dp if (self.global_sampling if self.global_sampling is not None
                           else dp is not None) else None
            if shard is None and self.global_sampling:
                raise ValueError("global_sampling needs an initialised torch.distributed group")
            it = _TableIterator(self.table, self.batch_size, self.timeout, self.prefetch, shard)
        return it if self.batched else _Unbatched(it)


class _Unbatched:
    """Single items (batch_size None): the batch-of-one samples with the batch dimension
    dropped (views of the iterator's buffers, valid until it advances twice)."""

    def __init__(self, it):
        self._it = it

    def __iter__(self):
        return self

    def __next__(self) -> replay.ReplaySample:
        s = next(self._it)
        first = lambda x: x[0]  # noqa: E731
        return replay.ReplaySample(
            info=replay.SampleInfo(*[None if x is None else x[0] for x in s.info]),
            data=tree.unflatten_as(s.data, [first(x) for x in tree.flatten(s.data)]))


class _TableIterator:
    # The batches handed out by the last two next() calls stay intact until the following
    # next() (the buffer ring holds 2, or P + 2 with prefetch): DQNLearner re-issues a skipped
    # step from them without copying (acme_amd/agents/dqn/learning.py).
    holds_last_batches = 2

    def __init__(self, table: replay.Table, batch: int, timeout: float, prefetch: int = 0,
                 shard=None):
        self._t = table
        self._B = batch
        self._timeout = timeout
        self._P = prefetch
        self._slots = None
        self._queue = []  # (slot index, ready event) of batches issued ahead
        # Global-probability sampling over shards: (world, rank), buffers for shares of up to
        # 2 B items, the mass snapshots by draw index, the share of each buffer slot.
        self._shard = shard
        self._rows = 2 * batch if shard is not None else batch
        self._snaps = {}
        self._share = {}
        # The exact f16 copy of [o_tm1; o_t] written by the fused sample + gather (uint8
        # transition tables): per buffer slot, or None; `last_frames_f16` is the copy of
        # the batch handed out last (the DQN learner then skips its own conversion).
        self._fb = []
        self.last_frames_f16 = None
        self.last_inputs_event = None  # see __next__
        if shard is not None and isinstance(table, replay.FrameTable):
            raise ValueError("global sampling over FrameTable shards is not supported")

    def _alloc(self):
        import ctypes
        native = self._t.native
        dev = native.device
        self._slots = []
        if self._P > 0:
            self._stream = torch.cuda.Stream(device=dev)
            # Device-scope events (no system-scope cache writeback and invalidation).
            from acme_amd._lib import OrderEvent
            self._issued = OrderEvent()
            self._ready = [OrderEvent() for _ in range(self._P + 2)]
            self._next_slot = 0
            self._open_pipe()
        if self._shard is not None:
            import torch.distributed as dist
            world = self._shard[0]
            self._dist = dist
            self._snap_ring = [(torch.zeros(world, dtype=torch.float64, device=dev),
                                torch.zeros(world, dtype=torch.float64).pin_memory(),
                                torch.cuda.Event()) for _ in range(self._P + 2 + 2 * _LAG)]
            self._snap_next = 0
        for _ in range(self._P + 2 if self._P > 0 else 2):
            info = native.alloc_sample_info(self._rows)
            fields = self._t.fields
            bufs = [None] * len(fields)
            # Transition items (o_tm1, a_tm1, r_t, d_t, o_t, ...): the two observations share
            # one [2, B, row] allocation, so o_t directly follows o_tm1 and the DQN learner
            # reads both as one frame array without a packing copy.
            if (len(fields) >= 5 and fields[0].row_bytes == fields[4].row_bytes
                    and fields[0].dtype == fields[4].dtype and fields[0].shape == fields[4].shape):
                pair = torch.empty(2, self._rows, fields[0].row_bytes, dtype=torch.uint8,
                                   device=dev)
                bufs[0], bufs[4] = pair[0], pair[1]
            bufs = [b if b is not None else
                    torch.empty(self._rows, f.row_bytes, dtype=torch.uint8, device=dev)
                    for b, f in zip(bufs, fields)]
            data = tree.unflatten_as(self._t._structure, [self._typed(b, f)  # noqa: SLF001
                                                          for b, f in zip(bufs, self._t.fields)])
            sample = replay.ReplaySample(
                info=replay.SampleInfo(key=info["keys"], probability=info["probabilities"],
                                       table_size=info["table_size"], priority=info["priorities"]),
                data=data)
            # Raw device pointers for the two per-step native calls (the views above alias
            # these buffers, so the returned sample never needs rebuilding).
            ptrs = (ctypes.c_void_p * len(bufs))(*[b.data_ptr() for b in bufs])
            raw = tuple(info[k].data_ptr() for k in ("slots", "keys", "probabilities",
                                                      "table_size", "priorities"))
            # `info` and `bufs` own the device memory behind `raw` / `ptrs` (the sampled
            # slots have no other reference): keep them alive with the slot set.
            self._slots.append((raw, ptrs, sample, info, bufs))
            self._fb.append(torch.empty(2 * self._rows, fields[0].row_bytes, dtype=torch.int16,
                                        device=dev) if self._f16_frames() else None)
        self._which = 0

    def _open_pipe(self) -> None:
        """Pipelined draws (round 6, acme_replay_sample_gather_pipe): a prefetched batch's rows
        are copied by the NEXT draw's launch, beside that draw's tree descent, so its ready
        event is recorded after that launch.  Same draws, keys and rows as the unpipelined
        path; single-table transition layouts only (not shards, FrameTable or the f16 copy),
        and prefetch_size >= 2 (at 1 the batch handed out would wait for the launch issued
        in the same next() call).  ACME_REPLAY_PIPE=0 turns it off (A/B)."""
        self._pipe = None
        self._pending = None  # buffer slot whose rows the next launch copies
        if (self._P < 2 or self._shard is not None
                or isinstance(self._t, (replay.FrameTable, replay.QueueTable))
                or self._f16_frames() or os.environ.get("ACME_REPLAY_PIPE", "1") == "0"):
            return
        import ctypes
        from acme_amd._lib import check, lib
        pid = ctypes.c_int32()
        check(lib().acme_replay_pipe_open(self._t.native.handle, ctypes.byref(pid)), "replay pipe")
        self._pipe = pid.value
        self._pipe_native = self._t.native  # closed before the table is destroyed

    def __del__(self):
        pipe = getattr(self, "_pipe", None)
        if pipe is not None:
            try:
                from acme_amd._lib import lib
                h = self._pipe_native.handle
                if h is not None and h.value:
                    lib().acme_replay_pipe_close(h, pipe)
            except Exception:  # interpreter shutdown
                pass
            self._pipe = None

    def _f16_frames(self) -> bool:
        """The fused kernel's f16 copy applies to uint8 transition tables whose only large
        fields are the two observations (fields 0 and 4); a shard's copy holds its share."""
        if isinstance(self._t, (replay.FrameTable, replay.QueueTable)):
            return False
        # Off by default since round 5: the DQN learner's conv1 reads the batch's uint8 frames
        # directly (half the bytes, and no 57.8 MB copy per B = 512 batch); ACME_DATASET_F16=1
        # brings back the copy (the round-4 path; bit-identical steps, tests/test_dp.py).
        if os.environ.get("ACME_DATASET_F16", "0") != "1":
            return False
        f = self._t.fields
        big = [i for i, x in enumerate(f) if x.row_bytes >= 1024]
        return (big == [0, 4] and f[0].dtype == np.uint8 and f[0].row_bytes == f[4].row_bytes
                and f[0].row_bytes % 16 == 0)

    def _typed(self, buf, f, rows=None):
        B = self._rows if rows is None else rows
        x = buf[:B] if f.nbytes == f.row_bytes else buf[:B, :f.nbytes]
        if f.dtype == np.bool_:
            return x.view(torch.bool).reshape((B,) + f.shape)
        return x.view(_TORCH[np.dtype(f.dtype)]).reshape((B,) + f.shape)

    @property
    def batch_size(self) -> int:
        return self._B

    def __iter__(self):
        return self

    def _draw(self, L, h, raw, ptrs, st, stream=None, fb=None):
        """Sample + gather of one batch as a unit: no insert lands between the draw and the
        row copy (actor threads may be inserting), so each row is that of its reported key.
        Returns the number of items drawn."""
        from acme_amd._lib import check
        t = self._t
        step = t.next_draw() & 0xFFFFFFFFFFFFFFFF
        if self._shard is not None:
            n, scale = self._shares(step)
            if fb is not None:
                check(L.acme_replay_sample_share_frames(h, n, step, scale, *raw, ptrs,
                                                        fb.data_ptr(), st), "replay sample")
            else:
                check(L.acme_replay_sample_share(h, n, step, scale, *raw, ptrs, st),
                      "replay sample")
            self._snapshot(L, h, step, st, stream)
            return n
        if isinstance(t, replay.FrameTable):  # stacks rebuilt from stored frames
            with t._mu:  # noqa: SLF001  (inserts commit under the table lock)
                check(L.acme_replay_sample(h, self._B, step, *raw, st), "replay sample")
                t.gather_into(raw[0], self._B, ptrs, st)
        elif fb is not None:
            check(L.acme_replay_sample_gather_frames(h, self._B, step, *raw, ptrs, fb.data_ptr(),
                                                     st), "replay sample")
        elif stream is not None and getattr(self, "_pipe", None) is not None:
            check(L.acme_replay_sample_gather_pipe(h, self._pipe, self._B, step, *raw, ptrs, st),
                  "replay sample")
        else:
            check(L.acme_replay_sample_gather(h, self._B, step, *raw, ptrs, st),
                  "replay sample")
        return self._B

    # -- global-probability sampling over shards (acme_amd.replay.sharding)
    def _shares(self, step: int):
        """(this rank's share n_r, probability scale n_r / (N B)) of draw `step`, from the
        mass snapshot taken after draw step - LAG (equal shares before the first one)."""
        world, rank = self._shard
        NB = world * self._B
        snap = self._snaps.pop(step - _LAG, None)
        if snap is None:
            n = self._B
        else:
            host, ev = snap
            ev.synchronize()  # issued LAG draws ago: normally long complete
            n = allocate_shares(host.tolist(), NB, cap=self._rows)[rank]
        return n, n / NB

    def _snapshot(self, L, h, step: int, st: int, stream) -> None:
        from acme_amd._lib import check
        world, rank = self._shard
        dev_vec, host, ev = self._snap_ring[self._snap_next]
        self._snap_next = (self._snap_next + 1) % len(self._snap_ring)
        s = stream if stream is not None else torch.cuda.current_stream(self._t.native.device)
        with torch.cuda.stream(s):
            dev_vec.zero_()
            check(L.acme_replay_total(h, dev_vec[rank:].data_ptr(), st), "replay total")
            self._dist.all_reduce(dev_vec)  # SUM of one-hot masses: exact, identical on ranks
            host.copy_(dev_vec, non_blocking=True)
            ev.record(s)
        self._snaps[step] = (host, ev)

    def _sample_view(self, i: int, n: int) -> replay.ReplaySample:
        """The first n rows of buffer slot i as a ReplaySample (shard draws vary in size)."""
        raw, ptrs, sample, info, bufs = self._slots[i]
        if n == self._rows:
            return sample
        data = tree.unflatten_as(self._t._structure, [self._typed(b, f, n)  # noqa: SLF001
                                                      for b, f in zip(bufs, self._t.fields)])
        return replay.ReplaySample(
            info=replay.SampleInfo(key=info["keys"][:n], probability=info["probabilities"][:n],
                                   table_size=info["table_size"][:n],
                                   priority=info["priorities"][:n]),
            data=data)

    def __next__(self) -> replay.ReplaySample:
        from acme_amd._lib import check, lib, stream_ptr
        t = self._t
        t.wait_for(self._B, self._timeout)
        t.flush_for_sampling(self._B)
        if self._slots is None:
            self._alloc()
        L, h = lib(), t.native.handle
        if self._P == 0:
            i = self._which
            raw, ptrs = self._slots[i][:2]
            self._which ^= 1
            n = self._draw(L, h, raw, ptrs, stream_ptr(), fb=self._fb[i])
            self.last_frames_f16 = self._fb[i]
            return self._sample_view(i, n)
        # Prefetch: order the dataset stream after everything queued so far on the caller's
        # stream (inserts, earlier learner steps and their priority updates), top the queue
        # up to P + 1 batches, hand out the oldest.
        from acme_amd._lib import profiling
        main = torch.cuda.current_stream(self._t.native.device)
        # Under the section profiler the batches are issued on the caller's stream, so no
        # profiled kernel shares the GPU with a prefetch (same draws, same order).
        side = main if profiling() else self._stream
        self._issued.record(main)
        side.wait_event(self._issued)
        st = stream_ptr(side)
        while len(self._queue) < self._P + 1:
            i = self._next_slot
            self._next_slot = (i + 1) % (self._P + 2)
            raw, ptrs = self._slots[i][:2]
            self._share[i] = self._draw(L, h, raw, ptrs, st, side, fb=self._fb[i])
            # Pipelined: this launch completed the previous batch's rows; the new batch's
            # event is recorded after the launch that copies them.
            done = i
            if self._pipe is not None:
                done = i if self._pending is None else self._pending
                self._pending = i
            self._ready[done].record(side)
            self._queue.append(i)
            t.set_reader_event(self._ready[done])
        i = self._queue.pop(0)
        # A batch issued P steps ago has normally landed: ordering the caller's stream
        # after a completed event is a no-op, and skipping the wait saves its queue-side
        # cost (each event wait / record on a stream leaves ~7 us before the next kernel).
        if not self._ready[i].query():
            main.wait_event(self._ready[i])
        # The batch is complete at its ready event (recorded on the dataset's stream): a
        # learner may start work on another stream of its own from it.
        self.last_inputs_event = self._ready[i] if side is not main else None
        self.last_frames_f16 = self._fb[i]
        return self._sample_view(i, self._share[i])


class _QueueIterator(_TableIterator):
    """Batches of a QueueTable: each next() consumes the next B items (FIFO, once) and
    gathers their rows from the HBM ring on the GPU (keys = insertion indices, probability
    and priority 1, table_size = items still queued)."""

    def __init__(self, table: replay.QueueTable, batch: int, timeout: float):
        super().__init__(table, batch, timeout, prefetch=0, shard=None)

    def __next__(self) -> replay.ReplaySample:
        from acme_amd._lib import check, lib, stream_ptr
        t = self._t
        if self._slots is None:
            t.wait_for(1, self._timeout)  # the first item fixes the layout the slots need
            self._alloc()
        i = self._which
        self._which ^= 1
        raw, ptrs, sample, info, _ = self._slots[i]

        def read(first: int) -> None:
            # Issued under the table lock, before pop_slots frees the slots to writers.
            dev = t.native.device
            idx = torch.arange(first, first + self._B, dtype=torch.int64, device=dev)
            info["keys"].copy_(idx.view(torch.uint64))
            info["probabilities"].fill_(1.0)
            info["priorities"].fill_(1.0)
            info["table_size"].fill_(t.size() - self._B)
            slots = idx % t.max_size
            check(lib().acme_replay_gather(t.native.handle, slots.data_ptr(), self._B, ptrs,
                                           stream_ptr()), "queue gather")
            self._keep = slots  # the launch reads it on the stream

        t.pop_slots(self._B, self._timeout, read=read)
        return sample


def make_reverb_dataset(server_address, environment_spec=None, batch_size: Optional[int] = None,
                        prefetch_size: Optional[int] = None, sequence_length: Optional[int] = None,
                        extra_spec=None, transition_adder: bool = False,
                        table: str = adders.DEFAULT_PRIORITY_TABLE,
                        parallel_batch_optimization: bool = True,
                        convert_zero_size_to_none: bool = False,
                        using_deprecated_adder: bool = False,
                        global_sampling: Optional[bool] = None) -> ReplayDataset:
    """Same arguments as the reference.  `prefetch_size` issues that many batches ahead on
    the dataset's stream (module docstring); the parallel-batch knob of the tf.data pipeline
    has no equivalent.  The environment / extra specs, transition_adder, sequence_length and
    convert_zero_size_to_none define `element_spec` as the reference's shapes and dtypes do
    (datasets/reverb.py:141-198); the rows themselves come from the table's layout (a
    sequence table stores T-step items, yielded [B, T, ...]), which is checked against the
    spec when both are known.  The GPU table stores fixed-shape rows, so items whose zero-size
    dimensions vary in length are refused at insert time."""
    del parallel_batch_optimization, using_deprecated_adder
    server = _server_of(server_address)
    if table not in server.tables:
        raise ValueError(f"unknown table {table!r}")
    t = server.tables[table]
    data_spec = None
    if environment_spec is not None:
        data_spec = _element_shapes(_adder_spec(transition_adder, environment_spec, extra_spec),
                                    sequence_length, convert_zero_size_to_none, batch_size)
        if isinstance(t, replay.Table) and t.fields is not None:
            leaves = tree.flatten(data_spec)
            if len(leaves) != len(t.fields):
                raise ValueError("environment_spec does not match the table's item layout")
            nb = 1 if batch_size else 0
            for x, f in zip(leaves, t.fields):
                want = tuple(x.shape[nb:])
                if None not in want and (want != tuple(f.shape) or np.dtype(x.dtype) != f.dtype):
                    raise ValueError(f"environment_spec leaf {want} {np.dtype(x.dtype)} does not "
                                     f"match the table's {tuple(f.shape)} {f.dtype}")
    return ReplayDataset(t, batch_size, prefetch=prefetch_size or 0,
                         global_sampling=global_sampling, data_spec=data_spec)


make_dataset = make_reverb_dataset
