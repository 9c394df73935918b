set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 0 > gpurun_out/ab_new_$i.json 2>/dev/null
  ACME_V_HEAD=1 timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 0 > gpurun_out/ab_old_$i.json 2>/dev/null
done
for f in gpurun_out/ab_*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f',d['ms_per_step'])"; done
