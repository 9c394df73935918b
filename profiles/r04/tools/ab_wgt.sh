# (Round-4 record: ACME_V_WGT was removed after this A/B; kept for R2D2 only.)
# A/B: the dense weight gradients (DQN fc_wgrad, IMPALA / R2D2 W_i) on 256x128 warp-
# specialised tiles (ACME_V_WGT=1) against 128x128 single-role at BK 16: oracle tests on the
# variant, then alternating bench runs of the three learners.
mkdir -p gpurun_out/wgt
O=gpurun_out/wgt
ACME_V_WGT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_dqn_gpu.py tests/test_impala_gpu.py tests/test_r2d2_learner_gpu.py -k "oracle or atari" > $O/tests.log 2>&1
rc=$?; echo "tests (WGT=1) rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" $O/tests.log | head; exit $rc; fi
for i in 1 2; do
  for v in base wgt; do
    unset ACME_V_WGT
    if [ $v = wgt ]; then export ACME_V_WGT=1; fi
    for w in dqn impala r2d2; do
      timeout -k 10 200 python3 bench.py --workload $w --no-cpu-baseline --no-staged > $O/${w}_${v}_$i.json 2>/dev/null || exit $?
    done
    python3 -c "
import json
out=[]
for w,k in (('dqn','fc_wgrad'),('impala','impala_wi_wgrad'),('r2d2','r2d2_wi_wgrad')):
    d=json.load(open('$O/'+w+'_${v}_$i.json')); ks={x['name']:x['avg_us'] for x in d['kernels']}
    out.append(f'{w} {d[\"ms_per_step\"]} {k} {ks.get(k)}')
print('$v $i', ' | '.join(out))"
  done
done
unset ACME_V_WGT
