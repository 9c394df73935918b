#!/bin/bash
# Round-6 call 27: non-temporal stores for the weight-gradient slabs (nt1) against the tree's
# build, on the step with the small write-back and the single-role conv1 weight gradient:
# six alternating 300-step pairs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g27; mkdir -p $O
for r in 1 2; do
VARS="nt1" W=dqn timeout -k 10 600 bash tools/ab_libs.sh $O/ab$r > $O/ab$r.log 2>&1 || { tail -5 $O/ab$r.log; exit 4; }
head -6 $O/ab$r.log
done
tail -2 $O/ab2.log
