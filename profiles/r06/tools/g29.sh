#!/bin/bash
# Round-6 call 29: the side stream (target forward, weight gradients) confined by a CU mask to
# 3 of every 4 CUs (m3) or half of them (m2), so the main stream's critical path always has
# CUs of its own: alternating 300-step runs against no mask.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g29; mkdir -p $O
A="" B="ACME_V_SIDEMASK=3" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/m3 > $O/m3.log 2>&1 || { tail -5 $O/m3.log; exit 4; }
head -6 $O/m3.log
A="" B="ACME_V_SIDEMASK=2" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/m2 > $O/m2.log 2>&1 || { tail -5 $O/m2.log; exit 4; }
head -6 $O/m2.log
