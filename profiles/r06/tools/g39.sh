#!/bin/bash
# Round-6 call 39: Adam's dense part with two float4 per thread (all eight loads issued before
# the first store; half the workgroups; ACME_V_ADAM2=1): DQN tests, then six alternating pairs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g39; mkdir -p $O
ACME_V_ADAM2=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1 || { tail -8 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for r in 1 2; do
A="" B="ACME_V_ADAM2=1" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$r > $O/t$r.log 2>&1 || { tail -5 $O/t$r.log; exit 4; }
head -6 $O/t$r.log
done
tail -2 $O/t2.log | cut -c1-120
