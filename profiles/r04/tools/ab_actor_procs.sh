# IMPALA configs[3] end to end: actor process counts 12 / 16 / 14, alternating (round 4).
mkdir -p gpurun_out/actors
for i in 1 2; do
  for p in 12 16 14; do
    timeout -k 10 200 python3 bench.py --workload impala_actors --steps 300 --warmup 20 --no-cpu-baseline --actor-procs $p > gpurun_out/actors/p${p}_$i.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/actors/p${p}_$i.json'));print('$p $i',d['value'],d['actors']['driver_us_per_act'])"
  done
done
