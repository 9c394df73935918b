# The fused head + loss + dZ kernel reading its loss inputs from LDS / prefetched registers:
# the DQN GPU tests, then the DQN step A/B against the previous kernel (libacme_hip_hlold.so).
set -u
O=gpurun_out/r05g47; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py tests/test_step_guard_gpu.py tests/test_agent_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
W=dqn VARS=hlold timeout -k 10 900 bash tools/ab_libs.sh $O/ab_dqn > $O/ab_dqn.log 2>&1; cat $O/ab_dqn.log
