#!/bin/bash
# Round-6 call 54: the final code: the whole -m gpu suite, smoke(), the
# driver's command line, a 200-step DQN line, the D4PG and IMPALA learner lines, the DQN
# counter passes + kernel stats, and a two-stream trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g54; mkdir -p $O/trace
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 13
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 14
timeout -k 10 600 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_dqn.json 2> $O/bench_dqn.err || exit 15
timeout -k 10 600 python3 bench.py --workload d4pg > $O/bench_d4pg.json 2> $O/bench_d4pg.err || exit 16
timeout -k 10 600 python3 bench.py --workload impala > $O/bench_impala.json 2> $O/bench_impala.err || exit 17
python3 -c "
import json
for f in ('bench_driver', 'bench_dqn', 'bench_d4pg', 'bench_impala'):
    d = json.load(open('$O/%s.json' % f)); print(f, d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"
bash tools/pmc_passes.sh dqn > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 18; }
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace/raw -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > $O/trace/bench.json 2> $O/trace/bench.err || exit 19
f=$(find $O/trace/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_abs.py "$f" 20 > $O/trace/step_abs.txt
echo done
