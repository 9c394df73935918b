#!/bin/bash
# Round-6 call 50: the write-back's phase stamps with a stamp before the verdict wait (phase
# "lds"), isolated steps and steps back to back.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g50; mkdir -p $O
timeout -k 10 200 python3 tools/update_stamps.py > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 3; }
timeout -k 10 200 python3 tools/update_stamps.py --steady > $O/stamps_steady.log 2>&1 || { tail -5 $O/stamps_steady.log; exit 4; }
tail -12 $O/stamps.log; tail -12 $O/stamps_steady.log
