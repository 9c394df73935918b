# Phase stamps of the fused priority write-back in the DQN step (tools/update_stamps.py).
set -u
O=gpurun_out/r05g37; mkdir -p $O
timeout -k 10 300 python3 tools/update_stamps.py > $O/stamps.log 2>&1; rc=$?
grep -v amdgpu.ids $O/stamps.log | tail -60
exit $rc
