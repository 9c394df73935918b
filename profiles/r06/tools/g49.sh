#!/bin/bash
# Round-6 call 49: the priority write-back (with the step's rescale) on a stream of its own,
# forked after conv2's input gradient so it runs beside conv1's weight gradient, joined before
# Adam (ACME_V_USTR=1): DQN / guard tests with it, then six alternating pairs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g49; mkdir -p $O
ACME_V_USTR=1 timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py tests/test_dp_bench_gpu.py tests/test_step_guard_gpu.py tests/test_replay_gpu.py -k "not long_horizon" > $O/tests.log 2>&1 || { tail -12 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for r in 1 2; do
A="" B="ACME_V_USTR=1" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$r > $O/t$r.log 2>&1 || { tail -5 $O/t$r.log; exit 4; }
head -6 $O/t$r.log
done
