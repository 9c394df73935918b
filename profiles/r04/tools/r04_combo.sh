# Round 4: R2D2 / IMPALA GPU tests, an r2d2 bench line, then a kernel trace of the DQN step.
mkdir -p gpurun_out/r04r gpurun_out/trace
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_r2d2_learner_gpu.py tests/test_impala_gpu.py tests/test_impala_agent_gpu.py > gpurun_out/r04r/gpu.log 2>&1
rc=$?; echo "gpu rc=$rc"; tail -14 gpurun_out/r04r/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --workload r2d2 --steps 10 --warmup 3 --cpu-baseline-seconds 5 > gpurun_out/r04r/bench.json 2> gpurun_out/r04r/bench.err || exit $?
tail -32 gpurun_out/r04r/bench.err; head -c 300 gpurun_out/r04r/bench.json; echo
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace/raw -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > gpurun_out/trace/bench.json 2> gpurun_out/trace/bench.err || exit $?
f=$(find gpurun_out/trace/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_abs.py "$f" 20 > gpurun_out/trace/abs.txt
cp "$f" gpurun_out/trace/kernel_trace.csv
echo trace done
