# Tests, then an A/B of library builds on the DQN step (and optionally another workload).
# Usage (under gpurun): OUT=name VARS="v1 ..." [W2=impala] bash tools/ab_run.sh test_file.py ...
set -u
O=gpurun_out/$OUT; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread "$@" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 bash tools/ab_libs.sh $O/ab_dqn > $O/ab_dqn.log 2>&1; cat $O/ab_dqn.log
if [ -n "${W2:-}" ]; then
  W=$W2 timeout -k 10 600 bash tools/ab_libs.sh $O/ab_$W2 > $O/ab_$W2.log 2>&1; cat $O/ab_$W2.log
fi
