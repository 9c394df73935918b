# Round-4 first GPU pass: the IMPALA end-to-end record, then the ONFIRST A/B on 20-step windows.
set -e
mkdir -p gpurun_out/r04a
timeout -k 10 240 python3 bench.py --workload impala_actors --steps 300 --warmup 20 > gpurun_out/r04a/bench_impala_actors.json 2> gpurun_out/r04a/impala_actors.log
cat gpurun_out/r04a/bench_impala_actors.json
AB="base ONFIRST=1" bash profiles/r04/tools/short_ab.sh
