# Phase stamps of the DQN forward GEMMs / convolutions (tools/gemm_stamps.py), then the DQN tests.
set -u
O=gpurun_out/r05g20; mkdir -p $O
timeout -k 10 200 python3 tools/gemm_stamps.py > $O/stamps.log 2>&1; rc=$?; grep -v "amdgpu.ids" $O/stamps.log | tail -24
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_gpu.py tests/test_frames_f16_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; exit $rc
