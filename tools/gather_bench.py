"""Replay row gather in isolation (acme_replay_gather): the 1M-slot Atari table of BASELINE
configs[1], batches of 512 prioritized draws, per-launch time by HIP events over many
launches with fresh draws (no cache reuse between launches), for the kernel variants
selected by acme_tune_set("GATH" / "GATHG").  Checks every variant against the reference
row-per-workgroup kernel bit for bit.  Usage: python tools/gather_bench.py [capacity]."""

import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from acme_amd._lib import lib
    from acme_amd.native import NativeReplay
    cap = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    B, n_draws = 512, 64
    fb = [28224, 4, 4, 4, 28224]
    r = NativeReplay(cap, fb, prioritized=True, priority_exponent=0.6, seed=3)
    r.fill_synthetic(cap, 0, num_actions=18, seed=1)
    slots = [r.sample(B, s)["slots"].clone() for s in range(n_draws)]
    outs = [torch.empty(B, b, dtype=torch.uint8, device="cuda") for b in fb]
    algo = 2 * B * (2 * 28224 + 12) + 8 * B
    L = lib()
    res = {}

    def run(variant, reps=4):
        for k, v in variant.items():
            L.acme_tune_set(k.encode(), v)
        for s in slots[:4]:
            r.gather(s, outs)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            for s in slots:
                r.gather(s, outs)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (reps * len(slots))
        for k in variant:
            L.acme_tune_set(k.encode(), 0)
        return us

    def snapshot(s):
        r.gather(s, outs)
        torch.cuda.synchronize()
        return [o.clone() for o in outs]

    L.acme_tune_set(b"GATH", 1)
    ref = snapshot(slots[7])
    L.acme_tune_set(b"GATH", 0)
    got = snapshot(slots[7])
    assert all(torch.equal(a, b) for a, b in zip(ref, got)), "pieces gather differs"
    variants = {"rowblock (GATH=1)": {"GATH": 1}}
    for g in (1024, 4096):
        variants[f"pieces grid<={g} (GATH=2)"] = {"GATH": 2, "GATHG": g}
    variants["pair (default)"] = {}
    for gv in (2,):
        L.acme_tune_set(b"GATH", gv)
        got = snapshot(slots[9])
        L.acme_tune_set(b"GATH", 1)
        ref9 = snapshot(slots[9])
        assert all(torch.equal(a, b) for a, b in zip(ref9, got)), f"GATH={gv} differs"
    L.acme_tune_set(b"GATH", 0)
    for name, v in variants.items():
        us = run(v)
        res[name] = dict(us=round(us, 2), TBps=round(algo / us / 1e6, 3))
        print(f"{name:24s} {us:8.2f} us  {algo / us / 1e6:6.3f} TB/s", flush=True)
    # Sample + gather: the two launches (SGF=1) and the fused kernel (default), fresh draws.
    keys_b = torch.empty(B, dtype=torch.int64, device="cuda")
    h = r.handle
    import ctypes
    ptrs = (ctypes.c_void_p * len(outs))(*[o.data_ptr() for o in outs])
    info = r.alloc_sample_info(B)
    raw = [info[k].data_ptr() for k in ("slots", "keys", "probabilities", "table_size",
                                          "priorities")]
    for name, sgf in (("sample+gather (2 launches)", 1), ("sample+gather (fused)", 0)):
        L.acme_tune_set(b"SGF", sgf)
        for s in range(4):
            L.acme_replay_sample_gather(h, B, s, *raw, ptrs, None)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for s in range(4 * n_draws):
            L.acme_replay_sample_gather(h, B, 1000 + s, *raw, ptrs, None)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (4 * n_draws)
        res[name] = dict(us=round(us, 2), TBps=round(algo / us / 1e6, 3))
        print(f"{name:24s} {us:8.2f} us  {algo / us / 1e6:6.3f} TB/s", flush=True)
    L.acme_tune_set(b"SGF", 0)
    del keys_b
    # The same bytes as a contiguous device copy (torch copy_ of a [2, B, 28224] block).
    src = torch.empty(n_draws, 2 * B * 28224, dtype=torch.uint8, device="cuda")
    dst = torch.empty(2 * B * 28224, dtype=torch.uint8, device="cuda")
    for i in range(3):
        dst.copy_(src[i])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n_draws):
        dst.copy_(src[i])
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n_draws
    res["contiguous copy (torch)"] = dict(us=round(us, 2), TBps=round(algo / us / 1e6, 3))
    print(f"{'contiguous copy (torch)':24s} {us:8.2f} us  {algo / us / 1e6:6.3f} TB/s", flush=True)
    print(json.dumps(dict(capacity=cap, batch=B, algo_bytes=algo, variants=res)))


if __name__ == "__main__":
    main()
