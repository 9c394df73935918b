# Leaves and node values computed before the verdict wait (stores only after): replay tests, stamps,
# then the DQN step A/B against the previous kernel (libacme_hip_updpar.so).
set -u
O=gpurun_out/r05g39; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_replay_gpu.py tests/test_step_guard_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/update_stamps.py > $O/stamps.log 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps.log | tail -10
W=dqn VARS=updpar timeout -k 10 900 bash tools/ab_libs.sh $O/ab_dqn > $O/ab_dqn.log 2>&1; cat $O/ab_dqn.log
