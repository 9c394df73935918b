#!/bin/bash
# Round-6 call 19: weight-gradient kernels with deeper register staging (RS sets in flight):
# DQN parity tests on the base build (RS 4/4/4), then an A/B of the step against rs2 (the
# previous depth), rs3 (conv2/3 3, conv1 6, fc 3) and rs8 (conv2/3 3, conv1 8, fc 2).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g19; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dqn_gpu.py \
  tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
VARS="rs2 rs3 rs8" W=dqn timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 4; }
cat $O/ab.log
