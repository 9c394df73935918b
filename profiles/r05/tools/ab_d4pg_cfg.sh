# D4PG dense-layer f32-engine configurations: tests on the bk32 build, then step time of the
# default (BK 16, 8 k-groups) against bk32, wk16 and bk32wk4.
set -u
O=gpurun_out/r05g22; mkdir -p $O
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_bk32.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_d4pg_gpu.py > $O/tests_bk32.log 2>&1
rc=$?; tail -2 $O/tests_bk32.log
W=d4pg VARS="bk32 wk16 bk32wk4" timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1; cat $O/ab.log
exit $rc
