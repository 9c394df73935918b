# Round 4: the R2D2 learner's GPU tests (+ the IMPALA tests sharing lstm.h and the plane
# policy step), then a short bench run of the r2d2 workload.
mkdir -p gpurun_out/r04r
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_r2d2_learner_gpu.py tests/test_impala_gpu.py tests/test_impala_agent_gpu.py > gpurun_out/r04r/gpu.log 2>&1
rc=$?; echo "gpu rc=$rc"; tail -14 gpurun_out/r04r/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --workload r2d2 --steps 10 --warmup 3 --cpu-baseline-seconds 5 > gpurun_out/r04r/bench.json 2> gpurun_out/r04r/bench.err || exit $?
tail -32 gpurun_out/r04r/bench.err; head -c 400 gpurun_out/r04r/bench.json
