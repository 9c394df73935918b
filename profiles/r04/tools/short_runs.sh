# Timed-window length vs measured step time (driver-like short runs against a long one).
set -e
mkdir -p gpurun_out/short
for k in 20 20 50 200 20; do
  timeout -k 10 150 python3 bench.py --steps $k --warmup 5 --no-cpu-baseline --profile-steps 0 --no-staged > gpurun_out/short/s_$k.json 2>/dev/null
  echo "steps $k $(python3 -c "import json;d=json.load(open('gpurun_out/short/s_$k.json'));print(d['ms_per_step'], d['settle_steps'])")"
done
