#!/bin/bash
# Round-6 call 23: where the priority write-back's 24 us in the two-stream trace go: the
# workgroups' s_memrealtime stamps (100 MHz) of the last launch against the kernel trace's
# start / end of that launch, in one run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g23; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/raw -- python3 tools/update_stamps.py --steady --abs > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 3; }
grep -v amdgpu $O/stamps.log
f=$(find $O/raw -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "prio_update_fused" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-3:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("trace start", s, "end", e, "dur_us", (e - s) / 1e3)
PY
