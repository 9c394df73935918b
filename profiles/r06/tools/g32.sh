#!/bin/bash
# Round-6 call 32: rehearsal on the current code: the whole -m gpu suite, smoke(), the driver's
# bench command line, a 200-step bench line, then the DQN counter passes and kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g32; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 13
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 14
timeout -k 10 600 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_dqn.json 2> $O/bench_dqn.err || exit 15
python3 -c "
import json
for f in ('bench_driver', 'bench_dqn'):
    d = json.load(open('$O/%s.json' % f)); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'])"
bash tools/pmc_passes.sh dqn > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 16; }
tail -22 $O/pmc.log
