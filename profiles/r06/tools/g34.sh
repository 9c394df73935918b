#!/bin/bash
# Round-6 call 34: the target fc_fwd (side stream, slack before the loss) at split-K 8 (128
# blocks: half the CUs, half the partial tile bytes) and 4 (64 blocks) on its 256x128
# producer/consumer tiles, against split-K 16 (256 blocks): headline test at 8, then three
# alternating 300-step pairs each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g34; mkdir -p $O
ACME_V_TSPLIT=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for t in 8 4; do
A="" B="ACME_V_TSPLIT=$t" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$t > $O/t$t.log 2>&1 || { tail -5 $O/t$t.log; exit 4; }
head -6 $O/t$t.log
done
