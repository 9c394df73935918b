# A/B of two builds of the library on the DQN step: the current acme_amd/libacme_hip.so
# ("new") against acme_amd/libacme_hip_old.so ("old", built beforehand from the baseline
# commit), selected through ACME_LIB_PATH; alternating step-time runs, then one profiled run
# each.  Run under gpurun; delete libacme_hip_old.so afterwards.
set -e
mkdir -p gpurun_out/ab
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_old.so; else unset ACME_LIB_PATH; fi
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 0 > gpurun_out/ab/s_${v}_$i.json 2>/dev/null
    echo "$v $i $(python3 -c "import json;print(json.load(open('gpurun_out/ab/s_${v}_$i.json'))['ms_per_step'])")"
  done
done
for v in new old; do
  if [ $v = old ]; then export ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_old.so; else unset ACME_LIB_PATH; fi
  timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 100 --warmup 20 > gpurun_out/ab/p_${v}.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/ab/p_${v}.json'))
print('$v', {k['name']:k['avg_us'] for k in d['kernels'] if k['name'] in ('loss_head_dz','fc_head_fwd')})"
done
