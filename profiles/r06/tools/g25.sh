#!/bin/bash
# Round-6 call 25: the priority write-back's small form (R = 2: 21 KB LDS, 56 VGPRs, fits beside
# the target forward's fused conv kernel): replay / headline / guard tests, A/B of the step
# against the previous library, and a two-stream trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g25; mkdir -p $O/trace
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_replay_gpu.py \
  tests/test_dqn_headline_gpu.py tests/test_step_guard_gpu.py tests/test_dp_bench_gpu.py -k "not long_horizon" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
VARS="prev" W=dqn timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 4; }
cat $O/ab.log
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace/raw -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > $O/trace/bench.json 2> $O/trace/bench.err || { tail -5 $O/trace/bench.err; exit 5; }
f=$(find $O/trace/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_abs.py "$f" 20 > $O/trace/step_abs.txt
tail -6 $O/trace/step_abs.txt
