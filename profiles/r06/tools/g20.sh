#!/bin/bash
# Round-6 call 20: a two-stream kernel trace of the DQN step (tools/trace_abs.py, 20 steps),
# then the D4PG counter passes and kernel stats (tools/pmc_passes.sh d4pg).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g20; mkdir -p $O/trace
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace/raw -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > $O/trace/bench.json 2> $O/trace/bench.err || { tail -5 $O/trace/bench.err; exit 4; }
f=$(find $O/trace/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_abs.py "$f" 20 > $O/trace/step_abs.txt
cat $O/trace/step_abs.txt
bash tools/pmc_passes.sh d4pg > $O/pmc_d4pg.log 2>&1 || { tail -20 $O/pmc_d4pg.log; exit 5; }
tail -25 $O/pmc_d4pg.log
