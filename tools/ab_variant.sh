# A/B of the in-tree library against a variant build (acme_amd/libacme_hip_$VAR.so, built
# with ACME_EXTRA_CFLAGS / ACME_BUILD_OUT): alternating 300-step runs, then one profiled
# run each.  Usage: VAR=fm bash tools/ab_variant.sh
set -e
mkdir -p gpurun_out/abv
for i in 1 2 3; do
  for v in base $VAR; do
    if [ $v = base ]; then unset ACME_LIB_PATH; else export ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_$v.so; fi
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 0 --no-staged > gpurun_out/abv/s_${v}_$i.json 2>/dev/null
    echo "$v $i $(python3 -c "import json;print(json.load(open('gpurun_out/abv/s_${v}_$i.json'))['ms_per_step'])")"
  done
done
for v in base $VAR; do
  if [ $v = base ]; then unset ACME_LIB_PATH; else export ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_$v.so; fi
  timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 100 --warmup 20 --no-staged > gpurun_out/abv/p_${v}.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/abv/p_${v}.json'))
print('$v', {k['name']:k['avg_us'] for k in d['kernels'][:12]})"
done
