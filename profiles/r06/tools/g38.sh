#!/bin/bash
# Round-6 call 38: sample_gather_pipe capped at 128 workgroups, six more pairs; then 64 (three).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g38; mkdir -p $O
for t in 128 128b 64; do
A="" B="ACME_V_SGG=${t%b}" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$t > $O/t$t.log 2>&1 || { tail -5 $O/t$t.log; exit 4; }
head -6 $O/t$t.log
done
