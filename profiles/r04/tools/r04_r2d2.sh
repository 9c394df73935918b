# R2D2 after the OAR split-K change: the R2D2 GPU tests, the profile refresh (kernel stats,
# PMC traffic) and the bench line.
mkdir -p gpurun_out/r2fin
B=gpurun_out/r2fin
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_r2d2_learner_gpu.py tests/test_r2d2_agent_gpu.py tests/test_r2d2_replay_gpu.py > $B/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $B/tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $B/tests.log | head; exit $rc; fi
STEPS=10 PSTEPS=3 bash tools/profile_round.sh r2d2 || exit $?
f=$(find gpurun_out/prof_r2d2 -name '*kernel_stats.csv' | head -1); cp "$f" $B/rocprof_r2d2_kernel_stats.csv
find gpurun_out/prof_r2d2 -name '*kernel_trace.csv' -delete
