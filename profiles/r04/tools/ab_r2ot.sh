# (Round-4 record: ACME_V_R2OT was removed after this A/B; the tall OAR tile is the default.)
# A/B: R2D2's OAR projection on 256x128 tiles at split-K 4 (ACME_V_R2OT=1) against 128x128
# at split-K 8: the Atari parity test with the variant, then alternating bench runs.
mkdir -p gpurun_out/r2ot
O=gpurun_out/r2ot
ACME_V_R2OT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_r2d2_learner_gpu.py -k atari > $O/tests.log 2>&1
rc=$?; echo "tests (R2OT=1) rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E  " $O/tests.log | head; exit $rc; fi
for i in 1 2; do
  for v in base tall; do
    unset ACME_V_R2OT
    if [ $v = tall ]; then export ACME_V_R2OT=1; fi
    timeout -k 10 200 python3 bench.py --workload r2d2 --no-cpu-baseline > $O/${v}_$i.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$O/${v}_$i.json'));k={x['name']:x['avg_us'] for x in d['kernels']};print('$v $i',d['value'],d['ms_per_step'],'oar',k.get('r2d2_oar_fwd'),'reduce',k.get('r2d2_oar_reduce'))"
  done
done
unset ACME_V_R2OT
timeout -k 10 400 python3 bench.py > $O/bench_dqn.json 2> $O/bench_dqn.err || exit $?
echo "dqn $(python3 -c "import json;d=json.load(open('$O/bench_dqn.json'));print(d['value'],d['ms_per_step'],d['roofline'])")"
