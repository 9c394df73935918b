# Fill/drain cost of short timed windows of the DQN step (tools/window_fill.py).
set -u
O=gpurun_out/r05g42; mkdir -p $O
timeout -k 10 300 python3 tools/window_fill.py breakdown > $O/window.log 2>&1; rc=$?
grep -v amdgpu.ids $O/window.log | tail -30
exit $rc
