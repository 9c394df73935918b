#!/bin/bash
# Round-6 call 42: the side stream's conv3 / conv2 weight gradients reserve 56 KB or 80 KB of LDS
# per block (ACME_V_WLDS, KB) instead of their 48 KB, so at most two / one of them share a CU
# and the main stream's conv2 input gradient (94.7 KB, 16 waves) fits beside one: three
# alternating pairs each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g42; mkdir -p $O
for t in 56 80; do
A="" B="ACME_V_WLDS=$t" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$t > $O/t$t.log 2>&1 || { tail -5 $O/t$t.log; exit 4; }
head -6 $O/t$t.log
done
