# Round 5: DQN frames / learner tests, the uint8-frames A/B, the D4PG tests, then the DQN PMC
# passes (tools/pmc_passes.sh).
set -u
O=gpurun_out/r05g9; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_frames_f16_gpu.py tests/test_dqn_gpu.py tests/test_d4pg_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
EXTRA=--no-staged A="" B="ACME_V_F16FRAMES=1 ACME_DATASET_F16=1" timeout -k 10 900 bash tools/ab_env.sh $O/ab_u8 > $O/ab_u8.log 2>&1; cat $O/ab_u8.log
timeout -k 10 900 bash tools/pmc_passes.sh dqn > $O/pmc.log 2>&1; rc=$?; tail -5 $O/pmc.log
exit $rc
