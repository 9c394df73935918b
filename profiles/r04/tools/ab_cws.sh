# (Round-4 record: the C2WS / C3WS hooks were removed after this A/B; 128 splits kept.)
# A/B: conv2 / conv3 weight-gradient split-K (ACME_V_C2WS / ACME_V_C3WS) at 64 and 256
# against 128: the bitwise fused/staged and oracle DQN tests at 64, then alternating runs.
mkdir -p gpurun_out/cws
O=gpurun_out/cws
ACME_V_C2WS=64 ACME_V_C3WS=64 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_dqn_gpu.py -k "fused_step_equals_staged or forward_backward_matches_oracle" > $O/tests.log 2>&1
rc=$?; echo "tests (64) rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" $O/tests.log | head; exit $rc; fi
for i in 1 2; do
  for v in 128 64 256; do
    export ACME_V_C2WS=$v ACME_V_C3WS=$v
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-staged > $O/s${v}_$i.json 2>/dev/null || exit $?
    python3 -c "
import json
d=json.load(open('$O/s${v}_$i.json')); k={x['name']:x['avg_us'] for x in d['kernels']}
print('$v $i', d['ms_per_step'], 'c3w', k.get('conv3_wgrad'), 'c2w', k.get('conv2_wgrad'), 'adam', k.get('adam'))"
  done
done
unset ACME_V_C2WS ACME_V_C3WS
