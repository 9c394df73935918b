# Round 5: the consumers' read threading (WS_FENCE 2, default) against no fences (0) and
# plain fences (1): DQN tests, then alternating step-time runs.
set -u
O=gpurun_out/r05g12; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
VARS="wsf0 wsf1" timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1; cat $O/ab.log
