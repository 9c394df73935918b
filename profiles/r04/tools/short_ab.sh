# A/B of ACME_V_* variants on driver-like 20-step windows (and one 200-step window each).
set -e
mkdir -p gpurun_out/sab
for i in 1 2 3; do
  for v in ${AB:-base ONFIRST=1}; do
    e=""; [ $v = base ] || e=$(echo "$v" | tr ',' '\n' | sed 's/^/ACME_V_/' | tr '\n' ' ')
    env $e timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-steps 0 --no-staged > gpurun_out/sab/$v.$i.json 2>/dev/null
    echo "$v 20 $(python3 -c "import json;print(json.load(open('gpurun_out/sab/$v.$i.json'))['ms_per_step'])")"
  done
done
