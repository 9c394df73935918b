#!/bin/bash
# Round-6 call 24: the next step's early target forward (the fused conv1 -> conv2 kernel, one
# block per CU) ordered after this step's priority write-back (ACME_V_TAU=1), so it no longer
# shares the GPU with the main stream's conv1 weight gradient and write-back: A/B of the
# step, then a two-stream trace with it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g24; mkdir -p $O/trace
A="" B="ACME_V_TAU=1" EXTRA="--no-staged" timeout -k 10 900 bash tools/ab_env.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 4; }
cat $O/ab.log
ACME_V_TAU=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace/raw -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > $O/trace/bench.json 2> $O/trace/bench.err || { tail -5 $O/trace/bench.err; exit 5; }
f=$(find $O/trace/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_abs.py "$f" 20 > $O/trace/step_abs.txt
cat $O/trace/step_abs.txt
