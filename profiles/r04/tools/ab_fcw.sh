# A/B: the online fc_fwd on 256x128 WS tiles with split-K 8 (ACME_V_FCW=1) against the 128x128 WS
# kernel: the B=512 headline parity test with the variant, then alternating bench runs.
mkdir -p gpurun_out/fcw
O=gpurun_out/fcw
ACME_V_FCW=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_dqn_headline_gpu.py > $O/headline.log 2>&1
rc=$?; echo "headline (FCT=1) rc=$rc"; tail -2 $O/headline.log
if [ $rc -ne 0 ]; then grep -E "^E  " $O/headline.log | head; exit $rc; fi
for i in 1 2 3; do
  for v in base fct; do
    unset ACME_V_FCW
    if [ $v = fct ]; then export ACME_V_FCW=1; fi
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-staged > $O/s_${v}_$i.json 2>/dev/null || exit $?
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-staged --steps 20 --warmup 5 --profile-steps 0 > $O/w_${v}_$i.json 2>/dev/null || exit $?
    python3 -c "
import json
d=json.load(open('$O/s_${v}_$i.json')); w=json.load(open('$O/w_${v}_$i.json'))
k={x['name']:x['avg_us'] for x in d['kernels']}
print('$v $i', d['ms_per_step'], w['ms_per_step'], 'fc_fwd', k.get('fc_fwd'), 'loss_head_dz', k.get('loss_head_dz'), 'fc_head_fwd', k.get('fc_head_fwd'), d['roofline']['frac'])"
  done
done
unset ACME_V_FCW
