# conv3_fwd at 6 waves per SIMD (P3I_OCC, default) against the unconstrained registers (occ0):
# DQN tests, then DQN and IMPALA step time.
set -u
O=gpurun_out/r05g19; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_gpu.py tests/test_impala_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
VARS="occ0" timeout -k 10 600 bash tools/ab_libs.sh $O/ab_dqn > $O/ab_dqn.log 2>&1; cat $O/ab_dqn.log
W=impala VARS="occ0" timeout -k 10 600 bash tools/ab_libs.sh $O/ab_impala > $O/ab_impala.log 2>&1; cat $O/ab_impala.log
