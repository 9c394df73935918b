# (Round-4 record: the C1WS / C1WT hooks were removed after this A/B; WS 256x32 at 512 splits kept.)
# A/B: conv1 weight-gradient split-K (ACME_V_C1WS) and tile (ACME_V_C1WT: 1 = WS 128x32,
# 2 = single-role 128x32) against WS 256x32 at 512 splits: the oracle DQN test at each
# variant, then alternating bench runs.
mkdir -p gpurun_out/c1w
O=gpurun_out/c1w
for cfg in "256 0" "512 1" "1024 1" "512 2"; do
  set -- $cfg
  ACME_V_C1WS=$1 ACME_V_C1WT=$2 timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_dqn_gpu.py -k "forward_backward_matches_oracle" > $O/tests_$1_$2.log 2>&1
  rc=$?; echo "tests ($1 $2) rc=$rc"; tail -1 $O/tests_$1_$2.log
  if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" $O/tests_$1_$2.log | head; exit $rc; fi
done
for i in 1 2; do
  for cfg in "512 0" "256 0" "512 1" "1024 1" "512 2"; do
    set -- $cfg
    export ACME_V_C1WS=$1 ACME_V_C1WT=$2
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-staged > $O/s$1_$2_$i.json 2>/dev/null || exit $?
    python3 -c "
import json
d=json.load(open('$O/s$1_$2_$i.json')); k={x['name']:x['avg_us'] for x in d['kernels']}
print('$1 $2 $i', d['ms_per_step'], 'c1w', k.get('conv1_wgrad'), 'adam', k.get('adam'))"
  done
done
unset ACME_V_C1WS ACME_V_C1WT
