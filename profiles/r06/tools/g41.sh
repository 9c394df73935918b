#!/bin/bash
# Round-6 call 41: conv3's (CWS=1), conv2's (CWS=2) or both (CWS=3) weight gradients on the side
# stream at split-K 64 instead of 128 (half the workgroups, twice the k per workgroup), so they
# leave CUs to the main stream's input-gradient chain they run beside (the side chain has
# ~35 us of slack): DQN tests at 3, then three alternating pairs each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g41; mkdir -p $O
ACME_V_CWS=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1 || { tail -8 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for t in 1 2 3; do
A="" B="ACME_V_CWS=$t" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$t > $O/t$t.log 2>&1 || { tail -5 $O/t$t.log; exit 4; }
head -6 $O/t$t.log
done
