#!/bin/bash
# Round-6 rehearsal: the 6-seed drift test (printed), the rest of the -m gpu suite, smoke(),
# the driver's bench command, and a 200-step bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g15; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
  tests/test_step_guard_gpu.py -k long_horizon_drift > $O/drift.log 2>&1 || exit 11
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "not long_horizon_drift" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 13
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 14
timeout -k 10 600 python3 bench.py --gpus 1 --steps 200 --warmup 20 > $O/bench_dqn.json 2> $O/bench_dqn.err || exit 15
echo done
