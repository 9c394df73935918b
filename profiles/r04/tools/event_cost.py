"""GPU-side cost of HIP event records and cross-stream waits between small kernels: a long
sleep kernel first, so the host queues every launch before the GPU reaches them; then
per-mode kernel gaps from a rocprofv3 kernel trace (tools/event_cost.py <trace.csv>)."""
import csv
import sys

import torch

if len(sys.argv) > 1:  # analysis of the trace: main-stream kernel gaps per spin segment
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    q_main = next(r["Queue_Id"] for r in rows if "spin" in r["Kernel_Name"])
    segs, cur = [], []
    for r in rows:
        if r["Queue_Id"] != q_main:
            continue
        if "spin" in r["Kernel_Name"]:
            if cur:
                segs.append(cur)
            cur = []
        else:
            cur.append(r)
    segs.append(cur)
    for m, s in enumerate(segs[-5:]):
        g = sorted((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000
                   for a, b in zip(s, s[1:]))
        print(f"mode {m}: {len(s)} kernels, median gap {g[len(g) // 2]:.2f} us, "
              f"p90 {g[9 * len(g) // 10]:.2f} us")
    sys.exit(0)
x = torch.zeros(1024, device="cuda")
s2 = torch.cuda.Stream()
e_other = torch.cuda.Event()
with torch.cuda.stream(s2):
    x.add_(0)
e_other.record(s2)
torch.cuda.synchronize()
evs = [torch.cuda.Event() for _ in range(4)]
# mode 4: the waited event is recorded on s2 after the host queued it but long before
# the main stream reaches the wait (the DQN dataset's case: the host runs steps ahead).
ev4 = [torch.cuda.Event() for _ in range(400)]
for mode in range(5):
    torch.cuda._sleep(200_000_000)
    if mode == 4:
        with torch.cuda.stream(s2):
            for i in range(400):
                x.add_(0)
                ev4[i].record(s2)
    for i in range(400):
        x.add_(1)
        if mode == 1:
            evs[i % 4].record()
        elif mode == 2:
            torch.cuda.current_stream().wait_event(e_other)
        elif mode == 3:
            evs[i % 4].record()
            s2.wait_event(evs[i % 4])
        elif mode == 4:
            torch.cuda.current_stream().wait_event(ev4[i])
    torch.cuda.synchronize()
print("done")
