# The online forward's o_t rows through the fused conv1 -> conv2 (c12ot) against conv1 + conv2:
# DQN tests on the variant, then step time.
set -u
O=gpurun_out/r05g23; mkdir -p $O
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_c12ot.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
VARS="c12ot" timeout -k 10 600 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1; cat $O/ab.log
