# (Round-4 record: the C1WS / C1WT hooks were removed after this A/B; WS 256x32 at 512 splits kept.)
# A/B round 2: conv1 weight-gradient split-K 512 / 256 / 128 / 384 (WS 256x32 tile),
# the oracle test at 128 and 384, then three alternating bench runs.
mkdir -p gpurun_out/c1w2
O=gpurun_out/c1w2
for s in 128 384; do
  ACME_V_C1WS=$s timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_dqn_gpu.py -k "forward_backward_matches_oracle" > $O/tests_$s.log 2>&1
  rc=$?; echo "tests ($s) rc=$rc"; tail -1 $O/tests_$s.log
  if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" $O/tests_$s.log | head; exit $rc; fi
done
for i in 1 2 3; do
  for s in 512 256 128 384; do
    export ACME_V_C1WS=$s
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-staged > $O/s${s}_$i.json 2>/dev/null || exit $?
    python3 -c "
import json
d=json.load(open('$O/s${s}_$i.json')); k={x['name']:x['avg_us'] for x in d['kernels']}
print('$s $i', d['ms_per_step'], 'c1w', k.get('conv1_wgrad'), 'adam', k.get('adam'))"
  done
done
unset ACME_V_C1WS
