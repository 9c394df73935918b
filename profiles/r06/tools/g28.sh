#!/bin/bash
# Round-6 call 28: non-temporal plane stores for the convolution forward outputs (ntf) and the
# input-gradient planes (ntd) against the tree's build: the headline parity test on each, then
# three alternating 300-step runs of each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g28; mkdir -p $O
for v in ntf ntd; do
  ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_headline_gpu.py > $O/tests_$v.log 2>&1 || { tail -5 $O/tests_$v.log; exit 3; }
  tail -1 $O/tests_$v.log
done
VARS="ntf ntd" W=dqn timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 4; }
cat $O/ab.log
