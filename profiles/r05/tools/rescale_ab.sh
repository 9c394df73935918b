# The end-of-step rescale with one round of loads (guard inputs with the records, verdict
# first): the whole -m gpu suite, then the DQN step A/B against the previous rescale.
set -u
O=gpurun_out/r05g40; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/tests.log | head; tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/update_stamps.py > $O/stamps.log 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps.log | tail -10
W=dqn VARS=rsold timeout -k 10 900 bash tools/ab_libs.sh $O/ab_dqn > $O/ab_dqn.log 2>&1; cat $O/ab_dqn.log
