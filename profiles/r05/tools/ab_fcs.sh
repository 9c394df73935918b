# The online fc_fwd at split-K 4 / 6 against 8: tests on fcs4, then step time.
set -u
O=gpurun_out/r05g24; mkdir -p $O
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_fcs4.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
VARS="fcs4 fcs6" timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1; cat $O/ab.log
