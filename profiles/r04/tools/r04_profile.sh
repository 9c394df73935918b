# Round 4 profile refresh: R2D2 tests after the LSTM chunk change, then rocprof kernel
# stats and PMC traffic passes for every learner workload.
mkdir -p gpurun_out/r04p
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_r2d2_learner_gpu.py > gpurun_out/r04p/r2d2_tests.log 2>&1
rc=$?; echo "r2d2 tests rc=$rc"; tail -3 gpurun_out/r04p/r2d2_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/profile_round.sh dqn || exit $?
bash tools/profile_round.sh d4pg || exit $?
bash tools/profile_round.sh impala || exit $?
STEPS=10 PSTEPS=3 bash tools/profile_round.sh r2d2 || exit $?
for w in dqn d4pg impala r2d2; do
  f=$(find gpurun_out/prof_$w -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/r04p/rocprof_${w}_kernel_stats.csv
  find gpurun_out/prof_$w -name '*kernel_trace.csv' -delete
done
echo all done
