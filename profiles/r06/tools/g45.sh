#!/bin/bash
# Round-6 call 45: the pipelined draw's row copies stored non-temporally (ntr: the learner reads
# them four steps later), replay tests on it, then six alternating pairs against the tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g45; mkdir -p $O
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_ntr.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_replay_gpu.py -k "pipelined or fused_sample or prefetched" > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for r in 1 2; do
VARS="ntr" W=dqn timeout -k 10 600 bash tools/ab_libs.sh $O/ab$r > $O/ab$r.log 2>&1 || { tail -5 $O/ab$r.log; exit 4; }
head -6 $O/ab$r.log
done
tail -2 $O/ab2.log | cut -c1-200
