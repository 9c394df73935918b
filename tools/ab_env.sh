# A/B of two environment settings on a workload's step (same library): alternating 300-step
# runs, then one profiled run each.  Usage: A="..." B="..." [W=d4pg] bash tools/ab_env.sh OUTDIR
#   e.g. A="" B="ACME_DATASET_F16=1"
set -e
O=${1:-gpurun_out/abe}; mkdir -p $O
for i in 1 2 3; do
  for v in A B; do
    eval "E=\$$v"
    env $E timeout -k 10 150 python3 bench.py --workload ${W:-dqn} --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 0 $EXTRA > $O/s_${v}_$i.json 2>$O/s_${v}_$i.err
    echo "$v $i $(python3 -c "import json;print(json.load(open('$O/s_${v}_$i.json'))['ms_per_step'])")"
  done
done
for v in A B; do
  eval "E=\$$v"
  env $E timeout -k 10 150 python3 bench.py --workload ${W:-dqn} --no-cpu-baseline --steps 100 --warmup 20 $EXTRA > $O/p_${v}.json 2>$O/p_${v}.err
  python3 -c "
import json;d=json.load(open('$O/p_${v}.json'))
print('$v', {k['name']:k['avg_us'] for k in d['kernels'][:14]})"
done
