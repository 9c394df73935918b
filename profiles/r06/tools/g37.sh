#!/bin/bash
# Round-6 call 37: the dataset's pipelined draw + row copy (sample_gather_pipe, 512 workgroups,
# four steps of slack) with at most 256 / 128 workgroups looping over the rows (ACME_V_SGG), so
# its 58 MB burst shares HBM and CUs more gently with the online forward it runs beside:
# replay / prefetch tests at 128, then three alternating pairs each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g37; mkdir -p $O
ACME_V_SGG=128 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_replay_gpu.py tests/test_prefetch_order_gpu.py tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1 || { tail -8 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for t in 256 128; do
A="" B="ACME_V_SGG=$t" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$t > $O/t$t.log 2>&1 || { tail -5 $O/t$t.log; exit 4; }
head -6 $O/t$t.log
done
