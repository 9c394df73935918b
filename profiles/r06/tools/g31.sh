#!/bin/bash
# Round-6 call 31: the target fc_fwd on 128x128 producer/consumer tiles at split-K 8 (TFC=2), six
# more alternating 300-step pairs against the kept 256x128 / split-K 16.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g31; mkdir -p $O
for r in 1 2; do
A="" B="ACME_V_TFC=2" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$r > $O/t$r.log 2>&1 || { tail -5 $O/t$r.log; exit 4; }
head -6 $O/t$r.log
done
tail -2 $O/t2.log
