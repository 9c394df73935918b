# Round-6 call 3: split accumulators -- gradient error structure at B=64, the DQN GPU tests, drift.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g3; mkdir -p $O
timeout -k 10 300 python -u tools/grad_err_diag.py --B 64 --out $O > $O/graderr_B64.log 2>&1 || { tail -20 $O/graderr_B64.log; exit 4; }
grep -E "structure|wgrad|plane:|f32:|conv2_d|hidden" $O/graderr_B64.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py tests/test_step_guard_gpu.py -k "not long_horizon" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread "tests/test_step_guard_gpu.py::test_long_horizon_drift" > $O/drift.log 2>&1
rc=$?; grep -E "B=|FAILED|ERROR|passed|failed|assert" $O/drift.log | tail -12; exit $rc
