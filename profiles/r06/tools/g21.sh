#!/bin/bash
# Round-6 call 21: priority write-back phase stamps with the steps synchronised and back to
# back (the bench's steady state), to locate the 24 us the launch takes in the two-stream
# trace against its 11 us workgroup span.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g21; mkdir -p $O
timeout -k 10 200 python3 tools/update_stamps.py > $O/stamps_sync.log 2>&1 || { tail -5 $O/stamps_sync.log; exit 3; }
timeout -k 10 200 python3 tools/update_stamps.py --steady > $O/stamps_steady.log 2>&1 || { tail -5 $O/stamps_steady.log; exit 3; }
grep -v amdgpu $O/stamps_sync.log | tail -10; grep -v amdgpu $O/stamps_steady.log
