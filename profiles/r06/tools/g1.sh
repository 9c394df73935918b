# Round-6 call 1: MFMA accumulation bias diagnostic, the ADVICE fixes' tests, the B=64 gradient
# error structure.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g1; mkdir -p $O
timeout -k 10 120 tools/mfma_bias > $O/mfma_bias.log 2>&1 || { cat $O/mfma_bias.log; exit 3; }
cat $O/mfma_bias.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_replay_gpu.py "tests/test_step_guard_gpu.py::test_learner_reissues_skipped_step" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/grad_err_diag.py --B 64 --out $O > $O/graderr_B64.log 2>&1 || { tail -20 $O/graderr_B64.log; exit 4; }
grep -E "structure|wgrad|plane:|f32:" $O/graderr_B64.log
