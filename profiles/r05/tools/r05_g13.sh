# Round 5: MFMA issue rate; the image-resident kernels' fenced loop with three weight
# register sets (default) against the round-4 loop (p3i0) and fences with two sets (p3i1).
set -u
O=gpurun_out/r05g13; mkdir -p $O
timeout -k 10 60 tools/mfma_rate > $O/mfma_rate.log 2>&1; cat $O/mfma_rate.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dqn_gpu.py tests/test_frames_f16_gpu.py tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
VARS="p3i0 p3i1" timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1; cat $O/ab.log
