# (Round-4 record: the OARS hook was removed after this A/B; split-K 2 kept.)
# A/B: R2D2's OAR projection split-K (ACME_V_OARS) 2 and 1 against 4: the R2D2 oracle tests
# at 2 and 1, then alternating 20-step bench runs.
mkdir -p gpurun_out/oars
O=gpurun_out/oars
for s in 2 1; do
  ACME_V_OARS=$s timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_r2d2_learner_gpu.py -k atari > $O/tests_$s.log 2>&1
  rc=$?; echo "tests ($s) rc=$rc"; tail -1 $O/tests_$s.log
  if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" $O/tests_$s.log | head; exit $rc; fi
done
for i in 1 2; do
  for s in 4 2 1; do
    export ACME_V_OARS=$s
    timeout -k 10 200 python3 bench.py --workload r2d2 --steps 20 --warmup 3 --profile-steps 5 --no-cpu-baseline > $O/s${s}_$i.json 2>/dev/null || exit $?
    python3 -c "
import json
d=json.load(open('$O/s${s}_$i.json')); k={x['name']:x['avg_us'] for x in d['kernels']}
print('$s $i', d['ms_per_step'], 'oar', k.get('r2d2_oar_fwd'), 'red', k.get('r2d2_oar_reduce'))"
  done
done
unset ACME_V_OARS
