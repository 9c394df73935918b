#!/bin/bash
# Round-6 call 44: a two-stream trace of the split-Adam schedule (ACME_V_SADAM=1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g44; mkdir -p $O/trace
ACME_V_SADAM=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace/raw -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > $O/trace/bench.json 2> $O/trace/bench.err || exit 5
f=$(find $O/trace/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_abs.py "$f" 20 > $O/trace/step_abs.txt
cat $O/trace/step_abs.txt
