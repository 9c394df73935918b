"""FrameTable: a Table whose stacked uint8 observations are stored one frame at a time.

SURVEY.md §8(f) row 4.  The reference's transition item carries two whole stacked
observations (acme/adders/reverb/transition.py:147-152: o_t and o_{t+n}), each built by
acme/wrappers/frame_stacking.py:78-83 as np.stack(last S frames, axis=-1) with zero frames
before the first one of an episode.  Consecutive stacks share S - 1 frames and o_{t+n} is a
later stack of the same episode, so storing stacks whole keeps every frame about 2 S times
(56,448 B per Atari transition; 56 GB per 1M slots).  Here each distinct frame is kept once
in an HBM ring [max_frames][H*W] and the item stores S int32 ring positions per stacked
field; the rest of the item is stored as by Table.  Sampling is unchanged (same sum tree,
same draws, same keys and probabilities); the dataset rebuilds the stacks of a sampled
batch with acme_frames_expand (csrc/frames.hip), so ReplaySample.data is bit-identical to
what a Table would return.

Deduplication is exact: a frame reuses a stored one only if its bytes are equal (hash
lookup over a window of recently stored frames, then a byte comparison).  Ring position 0
holds the all-zero frame (the padding of episode starts) and is never overwritten.  A frame
position is recycled only after every live item that references it has been evicted (FIFO);
a max_frames too small for that raises instead of corrupting an item.
"""

from __future__ import annotations

import collections
from typing import Optional, Sequence

import numpy as np

from acme_amd.utils import tree


def _make_frame_table(Table, _Field, _layout_from_signature):
    class FrameTable(Table):
        """Table(name, sampler, remover, max_size, rate_limiter, signature, ...) with the
        uint8 [H, W, S] leaves `stacked_fields` (flattened-leaf indices; default the two
        observations of a transition item) stored as deduplicated frames."""

        def __init__(self, name: str, sampler, remover, max_size: int, rate_limiter=None,
                     signature=None, seed: int = 1234, device=None, flush_every: int = 256,
                     stacked_fields: Sequence[int] = (0, 4), max_frames: Optional[int] = None,
                     window: int = 64):
            if signature is None:
                raise ValueError("FrameTable needs the item signature")
            outer = _layout_from_signature(signature)
            self._stacked = tuple(int(i) for i in stacked_fields)
            shapes = {outer[i].shape for i in self._stacked}
            if len(shapes) != 1:
                raise ValueError("stacked fields must share one [H, W, S] shape")
            shape = shapes.pop()
            for i in self._stacked:
                if outer[i].dtype != np.uint8 or len(outer[i].shape) != 3:
                    raise ValueError(f"field {i} is not a uint8 [H, W, S] stack")
            self._H, self._W, self._S = shape
            self._px = self._H * self._W
            if (self._px * self._S) % 4:
                # Dataset rows are padded to 4 bytes (_row_bytes) while the expand kernel
                # writes packed H*W*S rows: only unpadded stacks are supported.
                raise ValueError(f"stacked fields need H*W*S to be a multiple of 4, got "
                                 f"{self._H}x{self._W}x{self._S}")
            inner = [(_Field((self._S,), np.dtype(np.int32), 4 * self._S, 4 * self._S)
                      if i in self._stacked else f) for i, f in enumerate(outer)]
            super().__init__(name, sampler, remover, max_size, rate_limiter, signature=None,
                             seed=seed, device=device, flush_every=flush_every)
            self._outer_fields = outer
            self._init_layout(signature, inner)
            import torch
            self._F = int(max_frames) if max_frames else 2 * self.max_size + 1024
            if self._F < 2:
                raise ValueError("max_frames must be >= 2")
            dev = self._native.device
            self._frames = torch.zeros(self._F, self._px, dtype=torch.uint8, device=dev)
            self._g = 0                       # frames ever stored (ring position 1 + g % (F-1))
            self._recent = collections.OrderedDict()  # hash -> [(global index, bytes)]
            self._window = int(window)
            self._pending_frames = []         # (ring position, bytes) not yet on the device
            # Per live item (FIFO order): the oldest global frame index it references, and a
            # monotone deque of the same values for the sliding minimum.
            self._live_min = collections.deque()
            self._live_mono = collections.deque()
            self._idx_tmp = {}

        # -- layout seen by the dataset: the expanded items
        @property
        def fields(self):
            return self._outer_fields

        @property
        def stored_bytes_per_item(self) -> int:
            return sum(f.row_bytes for f in self._fields)

        @property
        def frames_stored(self) -> int:
            return self._g

        def _pos(self, g: int) -> int:
            return 1 + g % (self._F - 1)

        def _frame_index(self, frame: np.ndarray, live_floor: int) -> tuple:
            """(ring position, global index or None for the zero frame) of one frame."""
            if not frame.any():  # episode-start padding: the reserved zero frame
                return 0, None
            b = frame.tobytes()
            h = hash(b)
            for g, stored in self._recent.get(h, ()):
                if stored == b and g >= self._g - (self._F - 1):
                    return self._pos(g), g
            g = self._g
            # Recycling position pos(g) overwrites frame g - (F - 1): it must be older than
            # every frame a live item references.
            if g - (self._F - 1) >= live_floor:
                raise ValueError(f"FrameTable '{self.name}': max_frames={self._F} is too small "
                                 f"for the live items (a frame still referenced would be "
                                 f"overwritten); use a larger max_frames")
            self._g += 1
            pos = self._pos(g)
            self._pending_frames.append((pos, b))
            self._recent.setdefault(h, []).append((g, b))
            while len(self._recent) > self._window:
                self._recent.popitem(last=False)
            return pos, g

        def insert(self, item, priority: float) -> None:
            with self._mu:
                leaves = tree.flatten(item)
                if len(leaves) != len(self._outer_fields):
                    raise ValueError(f"item has {len(leaves)} leaves, table expects "
                                     f"{len(self._outer_fields)}")
                for i in self._stacked:
                    if np.shape(leaves[i]) != (self._H, self._W, self._S):
                        raise ValueError(f"leaf shape {np.shape(leaves[i])} does not match "
                                         f"table signature {(self._H, self._W, self._S)}")
                # The item about to be inserted evicts the oldest one when the table is full.
                # Everything below is undone if a frame cannot be placed (max_frames too
                # small), so a failed insert leaves the bookkeeping as it was.
                evicted = mono_evicted = None
                if len(self._live_min) >= self.max_size:
                    evicted = self._live_min.popleft()
                    if self._live_mono and self._live_mono[0] == evicted:
                        mono_evicted = self._live_mono.popleft()
                floor = self._live_mono[0] if self._live_mono else 1 << 62
                g0, npend = self._g, len(self._pending_frames)
                out, used = list(leaves), []
                try:
                    for i in self._stacked:
                        a = np.asarray(leaves[i], np.uint8)
                        idx = np.empty(self._S, np.int32)
                        for s in range(self._S):
                            pos, g = self._frame_index(np.ascontiguousarray(a[..., s]),
                                                       min(floor, *(used or [1 << 62])))
                            idx[s] = pos
                            if g is not None:
                                used.append(g)
                        out[i] = idx
                except ValueError:
                    self._g = g0
                    del self._pending_frames[npend:]
                    for h in list(self._recent):
                        kept = [e for e in self._recent[h] if e[0] < g0]
                        if kept:
                            self._recent[h] = kept
                        else:
                            del self._recent[h]
                    if mono_evicted is not None:
                        self._live_mono.appendleft(mono_evicted)
                    if evicted is not None:
                        self._live_min.appendleft(evicted)
                    raise
                m = min(used) if used else 1 << 62
                self._live_min.append(m)
                while self._live_mono and self._live_mono[-1] > m:
                    self._live_mono.pop()
                self._live_mono.append(m)
                super().insert(tree.unflatten_as(self._structure, out), priority)

        def flush(self) -> None:
            with self._mu:
                if self._pending_frames:
                    import torch
                    self._after_readers()  # a queued expand may still read these positions
                    pos = torch.as_tensor([p for p, _ in self._pending_frames], dtype=torch.int64)
                    data = np.frombuffer(bytearray(b"".join(b for _, b in self._pending_frames)),
                                         np.uint8).reshape(-1, self._px)
                    dev = self._frames.device
                    self._frames.index_copy_(0, pos.to(dev), torch.as_tensor(data).to(dev))
                    self._pending_frames = []
                super().flush()

        # -- checkpointing: the base table's items (ring positions) plus the frame ring and the
        # bookkeeping that decides when a ring position may be recycled.  The dedup window
        # is a cache: a restored table starts it empty (a repeated frame may be stored
        # twice; the samples are the same).
        def save(self):
            with self._mu:
                state = super().save()  # flushes the pending frames too
                state["frames"] = self._frames.cpu().numpy()
                state["frames_stored"] = np.int64(self._g)
                state["live_min"] = np.asarray(self._live_min, np.int64)
                state["live_mono"] = np.asarray(self._live_mono, np.int64)
                return state

        def restore(self, state) -> None:
            import torch
            with self._mu:
                if "frames" not in state:
                    raise ValueError(f"FrameTable '{self.name}': the checkpoint holds no "
                                     f"frame ring (saved by a plain Table?)")
                frames = np.asarray(state["frames"], np.uint8)
                if frames.shape != tuple(self._frames.shape):
                    raise ValueError(f"FrameTable '{self.name}': checkpoint frame ring "
                                     f"{frames.shape} != {tuple(self._frames.shape)}")
                super().restore(state)
                self._after_readers()
                self._frames.copy_(torch.as_tensor(frames).to(self._frames.device))
                self._g = int(state["frames_stored"])
                self._live_min = collections.deque(int(x) for x in state["live_min"])
                self._live_mono = collections.deque(int(x) for x in state["live_mono"])
                self._recent = collections.OrderedDict()
                self._pending_frames = []

        def gather_into(self, slots_ptr: int, batch: int, out_ptrs, stream: int) -> None:
            """Gather the sampled items into the dataset's (expanded) field buffers."""
            import ctypes

            import torch

            from acme_amd._lib import check, lib
            L = lib()
            tmp = self._idx_tmp.get(batch)
            if tmp is None:
                tmp = [torch.empty(batch, self._S, dtype=torch.int32, device=self._frames.device)
                       for _ in self._stacked]
                self._idx_tmp[batch] = tmp
            inner = (ctypes.c_void_p * len(self._fields))(*list(out_ptrs))
            for t, i in zip(tmp, self._stacked):
                inner[i] = t.data_ptr()
            check(L.acme_replay_gather(self._native.handle, slots_ptr, batch, inner, stream),
                  "replay gather")
            for t, i in zip(tmp, self._stacked):
                check(L.acme_frames_expand(self._frames.data_ptr(), self._F, self._px, self._S,
                                           t.data_ptr(), batch, out_ptrs[i], stream),
                      "frames expand")

    return FrameTable
