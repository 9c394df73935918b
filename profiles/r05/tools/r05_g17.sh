# Round 5: R2D2 checkpoint format / scale state, the reverted D4PG and f32 engine.
set -u
O=gpurun_out/r05g17; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_r2d2_agent_gpu.py tests/test_r2d2_learner_gpu.py tests/test_d4pg_gpu.py tests/test_impala_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -10
exit $rc
