# Round-6 call 8: step-time A/B/C (split accumulators / one accumulator / wgrads unsplit), the
# gradient-accuracy test on base and wgns, the multi-seed drift test.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g8; mkdir -p $O
VARS="onacc wgns" timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 3; }
cat $O/ab.log
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread "tests/test_step_guard_gpu.py::test_gradient_error_matches_f32_engine" > $O/grad_base.log 2>&1
grep -E "plane|passed|failed" $O/grad_base.log | tail -16
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_wgns.so timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread "tests/test_step_guard_gpu.py::test_gradient_error_matches_f32_engine" > $O/grad_wgns.log 2>&1
grep -E "plane|passed|failed" $O/grad_wgns.log | tail -16
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread "tests/test_step_guard_gpu.py::test_long_horizon_drift" > $O/drift.log 2>&1
rc=$?; grep -E "B=|FAILED|passed|failed|Error" $O/drift.log | tail -20; exit $rc
