# The priority write-back (with the step's rescale) on the side stream beside conv1's weight
# gradient (ACME_V_TAILSIDE=1) against after it on the main stream: DQN tests with the
# switch, then alternating 300-step runs and a kernel trace of the switched step.
set -u
O=gpurun_out/r05g48; mkdir -p $O
ACME_V_TAILSIDE=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_gpu.py tests/test_step_guard_gpu.py tests/test_agent_gpu.py tests/test_replay_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
A="" B="ACME_V_TAILSIDE=1" timeout -k 10 900 bash tools/ab_env.sh $O/ab > $O/ab.log 2>&1; cat $O/ab.log
