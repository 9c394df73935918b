# Two default bench runs with section profiles: step time and the fused loss / head-dZ kernel.
# Run under gpurun.
set -e
mkdir -p gpurun_out
run() { timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 150 --warmup 20 --profile-steps 30 > gpurun_out/lh_$1.json 2>/dev/null; }
for t in a b; do run $t; done
for t in a b; do python3 -c "
import json;d=json.load(open('gpurun_out/lh_$t.json'));k={x['name']:x['avg_us'] for x in d['kernels']}
print('$t', d['ms_per_step'], k.get('loss_head_dz'))"; done
