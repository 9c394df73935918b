#!/bin/bash
# Round-6 call 26: conv1's weight gradient on the single-role kernel (two 20-KB stages, 40 KB of
# LDS: fits beside the target forward's fused conv kernel, 121 KB) instead of the
# warp-specialised one (three stages, 60 KB): A/B of the step (ACME_V_C1S=1), then a trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g26; mkdir -p $O/trace
A="" B="ACME_V_C1S=1" EXTRA="--no-staged" timeout -k 10 900 bash tools/ab_env.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 4; }
cat $O/ab.log
ACME_V_C1S=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace/raw -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > $O/trace/bench.json 2> $O/trace/bench.err || { tail -5 $O/trace/bench.err; exit 5; }
f=$(find $O/trace/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_abs.py "$f" 20 > $O/trace/step_abs.txt
tail -8 $O/trace/step_abs.txt
