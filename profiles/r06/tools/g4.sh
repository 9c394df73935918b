# Round-6 call 4: drift at B=64/256/512 (split accumulators), then the whole -m gpu suite.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g4; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread "tests/test_step_guard_gpu.py::test_long_horizon_drift" > $O/drift.log 2>&1
rc=$?; grep -E "B=|FAILED|ERROR|passed|failed|assert" $O/drift.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect "tests/test_step_guard_gpu.py::test_long_horizon_drift" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; exit $rc
