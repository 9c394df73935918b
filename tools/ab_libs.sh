# A/B/C of library builds on a workload's step: the in-tree library ("base") and variant
# builds acme_amd/libacme_hip_<v>.so (ACME_EXTRA_CFLAGS / ACME_BUILD_OUT), alternating
# 300-step runs, then one profiled run each.  Usage: VARS="wsf0 wsf1" [W=dqn] bash tools/ab_libs.sh OUT
set -e
O=${1:-gpurun_out/abl}; mkdir -p $O
for i in 1 2 3; do
  for v in base $VARS; do
    if [ $v = base ]; then L=""; else L=$PWD/acme_amd/libacme_hip_$v.so; fi
    ACME_LIB_PATH=$L timeout -k 10 150 python3 bench.py --workload ${W:-dqn} --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 0 --no-staged > $O/s_${v}_$i.json 2>$O/s_${v}_$i.err
    echo "$v $i $(python3 -c "import json;print(json.load(open('$O/s_${v}_$i.json'))['ms_per_step'])")"
  done
done
for v in base $VARS; do
  if [ $v = base ]; then L=""; else L=$PWD/acme_amd/libacme_hip_$v.so; fi
  ACME_LIB_PATH=$L timeout -k 10 150 python3 bench.py --workload ${W:-dqn} --no-cpu-baseline --steps 100 --warmup 20 --no-staged > $O/p_${v}.json 2>$O/p_${v}.err
  python3 -c "
import json;d=json.load(open('$O/p_${v}.json'))
print('$v', {k['name']:k['avg_us'] for k in d['kernels'][:14]})"
done
