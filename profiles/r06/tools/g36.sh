#!/bin/bash
# Round-6 call 36: the fused target conv1 -> conv2 (gemm_p3c12, one block per CU) with at most
# 256 / 128 workgroups looping over the 512 frames (ACME_V_C12G), so that it leaves CUs to the
# main stream it runs beside: DQN tests at 128, then three alternating pairs each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g36; mkdir -p $O
ACME_V_C12G=128 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1 || { tail -8 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for t in 256 128; do
A="" B="ACME_V_C12G=$t" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$t > $O/t$t.log 2>&1 || { tail -5 $O/t$t.log; exit 4; }
head -6 $O/t$t.log
done
