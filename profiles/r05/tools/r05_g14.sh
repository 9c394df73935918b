# Round 5: MFMA chain rate, fc_fwd phase stamps, WS bitwise tests after the stamps change.
set -u
O=gpurun_out/r05g14; mkdir -p $O
timeout -k 10 60 tools/mfma_rate > $O/mfma_rate.log 2>&1; cat $O/mfma_rate.log
timeout -k 10 200 python3 tools/gemm_stamps.py > $O/stamps.log 2>&1; rc=$?; grep -v "Warning\|warn" $O/stamps.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dqn_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -5
exit $rc
