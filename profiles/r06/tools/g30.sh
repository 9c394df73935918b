#!/bin/bash
# Round-6 call 30: the target network's fc_fwd (side stream, slack of ~100 us before the loss)
# on smaller-LDS configurations so the main stream's conv1 / conv2 forward blocks can share its
# CUs: TFC=1 128x128 single-role (64 KB, split-K 8), TFC=2 128x128 producer/consumer (96 KB,
# split-K 8), TFC=3 256x128 single-role (96 KB, split-K 16); the kept one is 256x128
# producer/consumer (147 KB).  Alternating 300-step runs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g30; mkdir -p $O
timeout -k 10 300 env ACME_V_TFC=1 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for t in 1 2 3; do
A="" B="ACME_V_TFC=$t" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$t > $O/t$t.log 2>&1 || { tail -5 $O/t$t.log; exit 4; }
head -6 $O/t$t.log
done
