set -u
O=gpurun_out/r05g25; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_d4pg_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
W=d4pg VARS=d4old timeout -k 10 600 bash tools/ab_libs.sh $O/ab_d4pg > $O/ab_d4pg.log 2>&1; cat $O/ab_d4pg.log
