#!/bin/bash
# Round-6 call 22: non-temporal slab stores (kernel-end L2 writeback experiment): A/B of the
# DQN step, base vs nt1 (conv / fc weight-gradient slabs) vs nt3 (+ fc_fwd's split-K slab),
# then a two-stream trace of nt3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g22; mkdir -p $O/trace
VARS="nt1 nt3" W=dqn timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 4; }
cat $O/ab.log
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_nt3.so timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace/raw -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > $O/trace/bench.json 2> $O/trace/bench.err || { tail -5 $O/trace/bench.err; exit 5; }
f=$(find $O/trace/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_abs.py "$f" 20 > $O/trace/step_abs.txt
cat $O/trace/step_abs.txt
