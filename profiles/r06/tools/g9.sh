# Round-6 call 9: (wgrads unsplit) drift test + gradient test, then a two-stream kernel trace.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g9; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread "tests/test_step_guard_gpu.py::test_long_horizon_drift" "tests/test_step_guard_gpu.py::test_gradient_error_matches_f32_engine" > $O/drift.log 2>&1
rc=$?; grep -E "B=|FAILED|passed|failed|Error|plane " $O/drift.log | tail -36; [ $rc -eq 0 ] || exit $rc
mkdir -p $O/trace
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace/raw -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > $O/trace/bench.json 2> $O/trace/bench.err || { tail -5 $O/trace/bench.err; exit 4; }
f=$(find $O/trace/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_abs.py "$f" 20 > $O/trace/step_abs.txt
cp "$f" $O/trace/kernel_trace.csv
cat $O/trace/step_abs.txt
