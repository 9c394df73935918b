set -u
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_replay_gpu.py tests/test_frames_f16_gpu.py tests/test_step_guard_gpu.py tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py tests/test_checkpoint_gpu.py tests/test_dp.py tests/test_dp_bench_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|B=|passed|failed" $O/tests.log | tail -60
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $rc -eq 0 ]; then
EXTRA=--no-staged A="" B="ACME_V_F16FRAMES=1 ACME_DATASET_F16=1" timeout -k 10 900 bash tools/ab_env.sh $O/ab_u8 > $O/ab_u8.log 2>&1; cat $O/ab_u8.log
fi
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_d4pg_gpu.py > $O/tests_d4pg.log 2>&1
rc2=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests_d4pg.log | tail -20
if [ $rc2 -ne 0 ]; then grep -E "Error|assert" $O/tests_d4pg.log | head -20; exit $rc2; fi
exit $rc
