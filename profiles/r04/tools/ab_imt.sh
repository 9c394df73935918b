# (Round-4 record: ACME_V_IMT was removed after this A/B; both changes slower.)
# A/B: IMPALA's embedding gradient on 128x64 tiles (3 x 121 blocks) and the OAR projection at
# split-K 16 (ACME_V_IMT=1) against 128x128 tiles (3 x 61) and split-K 8.
mkdir -p gpurun_out/imt
O=gpurun_out/imt
ACME_V_IMT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_impala_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests (IMT=1) rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" $O/tests.log | head; exit $rc; fi
for i in 1 2 3; do
  for v in base imt; do
    unset ACME_V_IMT
    if [ $v = imt ]; then export ACME_V_IMT=1; fi
    timeout -k 10 200 python3 bench.py --workload impala --no-cpu-baseline > $O/${v}_$i.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));k={x['name']:x['avg_us'] for x in d['kernels']};print('$v $i',d['value'],d['ms_per_step'],'dgrad',k.get('impala_feat_dgrad'),'oar',k.get('impala_oar_fwd'),'red',k.get('impala_oar_reduce'))"
  done
done
unset ACME_V_IMT
