# IMPALA configs[3] end to end with the vectorised actor pool (1, 2, 4 host threads) and
# the thread-per-actor pool (0); learned frames/s and environment steps/s.
set -e
mkdir -p gpurun_out
for th in 1 2 4 0; do
  timeout -k 10 240 python3 bench.py --workload impala_actors --steps 30 --warmup 3 --actor-threads $th > gpurun_out/act_$th.json 2> gpurun_out/act_$th.err
  python3 -c "import json;d=json.load(open('gpurun_out/act_$th.json'));print($th, d['value'], d['actors'])"
done
