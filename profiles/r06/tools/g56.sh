#!/bin/bash
# Round-6 call 56: the write-back's phase stamps kept in registers and stored at exit
# (libacme_hip_sreg.so, -DACME_STAMPS_REG=1), against the in-tree stores-as-you-go stamps,
# steps back to back: the LDS phase without the stamps' own store waits.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g56; mkdir -p $O
for v in base sreg; do
  if [ $v = base ]; then L=""; else L=$PWD/acme_amd/libacme_hip_$v.so; fi
  ACME_LIB_PATH=$L timeout -k 10 200 python3 tools/update_stamps.py --steady > $O/stamps_$v.log 2>&1 || { tail -5 $O/stamps_$v.log; exit 3; }
  echo "== $v"; tail -10 $O/stamps_$v.log
done
