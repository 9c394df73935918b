#!/bin/bash
# Round-6 call 18: D4PG critic head + loss in one launch: the D4PG parity tests, then an A/B of
# the step (base = this tree, prev = the previous commit's library), alternating 300-step runs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g18; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_d4pg_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
VARS="prev" W=d4pg timeout -k 10 600 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 4; }
cat $O/ab.log
