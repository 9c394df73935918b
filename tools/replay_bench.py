"""Where the fused draw + gather's time goes (round 6): the configs[1] table (1M slots, uint8
Atari transitions, prioritized), B = 512, timed alone with HIP events over 50 launches each:
the fused sample + gather (acme_replay_sample_gather), the pipelined launch
(acme_replay_sample_gather_pipe: this batch's draw + the previous batch's rows), the draw alone (acme_replay_sample),
the gather alone (acme_replay_gather of the draw's slots) and a device-to-device copy of the
same bytes (torch), plus the priority update alone.

  python tools/replay_bench.py
"""

import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(b) / n


def main():
    from acme_amd._lib import check, lib, stream_ptr
    from acme_amd.native import NativeReplay
    B, cap, row = 512, 1_000_000, 84 * 84 * 4
    r = NativeReplay(cap, [row, 4, 4, 4, row], prioritized=True, priority_exponent=0.6,
                     seed=1234, device=torch.device("cuda", 0))
    r.fill_synthetic(cap, layout=0, num_actions=18, seed=0)
    info = r.alloc_sample_info(B)
    outs = [torch.empty(B, n, dtype=torch.uint8, device="cuda") for n in (row, 4, 4, 4, row)]
    ptrs = (ctypes.c_void_p * 5)(*[o.data_ptr() for o in outs])
    raw = [info[k].data_ptr() for k in ("slots", "keys", "probabilities", "table_size",
                                        "priorities")]
    step = [0]

    def fused():
        step[0] += 1
        check(lib().acme_replay_sample_gather(r.handle, B, step[0], *raw, ptrs, stream_ptr()))

    def draw():
        step[0] += 1
        r.sample(B, step[0], out=info)

    def gather():
        r.gather(info["slots"], outs)

    # The pipelined launch (acme_replay_sample_gather_pipe): two buffer sets in rotation, each
    # launch draws one batch and copies the rows of the one before.
    pid = ctypes.c_int32()
    check(lib().acme_replay_pipe_open(r.handle, ctypes.byref(pid)))
    sets = []
    for _ in range(2):
        inf = r.alloc_sample_info(B)
        o = [torch.empty(B, n, dtype=torch.uint8, device="cuda") for n in (row, 4, 4, 4, row)]
        sets.append(([inf[k].data_ptr() for k in ("slots", "keys", "probabilities", "table_size",
                                                  "priorities")],
                     (ctypes.c_void_p * 5)(*[x.data_ptr() for x in o]), inf, o))

    def pipe():
        step[0] += 1
        rw, pt = sets[step[0] & 1][:2]
        check(lib().acme_replay_sample_gather_pipe(r.handle, pid.value, B, step[0], *rw, pt,
                                                   stream_ptr()))

    src = torch.empty(2 * B * row, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    prios = torch.rand(B, dtype=torch.float64, device="cuda") + 0.1

    def update():
        r.update_priorities(info["keys"], prios)

    mb = 2 * B * (2 * row + 12) / 1e6
    for name, fn in (("fused sample+gather", fused), ("pipelined sample+gather", pipe),
                     ("sample", draw), ("gather", gather),
                     ("torch d2d copy of the rows", lambda: dst.copy_(src)),
                     ("update_priorities", update)):
        us = timed(fn)
        print(f"{name:28s} {us:7.2f} us" + (f"  {mb / us:.2f} TB/s on {mb:.1f} MB"
                                             if name != "update_priorities" and name != "sample"
                                             else ""), flush=True)


if __name__ == "__main__":
    main()
