# Round 5: the f32 engine's register ring (F32_RING 4, default) against the round-4 loop
# (r0), with the D4PG row kernels' batched loads: tests, then D4PG / DQN / IMPALA A/B.
set -u
O=gpurun_out/r05g15; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_d4pg_gpu.py tests/test_impala_gpu.py tests/test_dqn_gpu.py tests/test_r2d2_learner_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -10
if [ $rc -ne 0 ]; then exit $rc; fi
W=d4pg VARS="r0" timeout -k 10 600 bash tools/ab_libs.sh $O/ab_d4pg > $O/ab_d4pg.log 2>&1; cat $O/ab_d4pg.log
W=impala VARS="r0" timeout -k 10 600 bash tools/ab_libs.sh $O/ab_impala > $O/ab_impala.log 2>&1; cat $O/ab_impala.log
