# (Round-4 record: ACME_V_IMR1 was removed after this A/B; one row per row group is the default up to 16 rows.)
# A/B: IMPALA's one-launch LSTM with one row per row group (ACME_V_IMR1=1) against two (the
# default at B <= 32): the IMPALA tests on the variant, then alternating bench runs.
mkdir -p gpurun_out/imr1
O=gpurun_out/imr1
ACME_V_IMR1=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_impala_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests (IMR1=1) rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" $O/tests.log | head; exit $rc; fi
for i in 1 2 3; do
  for v in r2 r1; do
    unset ACME_V_IMR1
    if [ $v = r1 ]; then export ACME_V_IMR1=1; fi
    timeout -k 10 200 python3 bench.py --workload impala --no-cpu-baseline > $O/${v}_$i.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));l=d['lstm'];print('$v $i',d['value'],d['ms_per_step'],l['lstm_fwd']['us_per_launch'],l['lstm_bwd']['us_per_launch'])"
  done
done
unset ACME_V_IMR1
