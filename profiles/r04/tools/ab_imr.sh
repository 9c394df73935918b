# (Round-4 record: ACME_V_IMR4 was removed after this A/B; two rows per row group is the default.)
# A/B: IMPALA's one-launch LSTM with two rows per row group (the default up to 32 rows)
# against four (ACME_V_IMR4=1): the IMPALA tests on the default, then alternating bench runs.
mkdir -p gpurun_out/imr
O=gpurun_out/imr
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_impala_gpu.py tests/test_impala_agent_gpu.py tests/test_r2d2_learner_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" $O/tests.log | head; exit $rc; fi
for i in 1 2 3; do
  for v in r2 r4; do
    unset ACME_V_IMR4
    if [ $v = r4 ]; then export ACME_V_IMR4=1; fi
    timeout -k 10 200 python3 bench.py --workload impala --no-cpu-baseline > $O/${v}_$i.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));print('$v $i',d['value'],d['ms_per_step'],d['lstm'])"
  done
done
unset ACME_V_IMR4
