#!/bin/bash
# Round-6 call 51: the write-back's verdict poll.  Stamps (steps back to back) for the in-tree
# library and three variants: nvf (no early poll: the verdict loaded after the LDS work), vlds
# (the stale-key check read back from LDS, not the round-2 load's register), both; then
# alternating 300-step pairs of all four.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g51; mkdir -p $O
for v in base nvf vlds both; do
  if [ $v = base ]; then L=""; else L=$PWD/acme_amd/libacme_hip_$v.so; fi
  ACME_LIB_PATH=$L timeout -k 10 200 python3 tools/update_stamps.py --steady > $O/stamps_$v.log 2>&1 || { tail -5 $O/stamps_$v.log; exit 3; }
  echo "== $v"; tail -10 $O/stamps_$v.log
done
VARS="nvf vlds both" timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 4; }
cat $O/ab.log
