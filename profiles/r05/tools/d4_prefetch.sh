# D4PG with the reference agent's prefetch_size 4 against no prefetch: alternating runs.
set -u
O=gpurun_out/r05g46; mkdir -p $O
for i in 1 2 3; do
  for pf in 0 4; do
    timeout -k 10 150 python3 bench.py --workload d4pg --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 0 --prefetch $pf > $O/s_${pf}_$i.json 2> $O/s_${pf}_$i.err || exit 1
    echo "prefetch $pf run $i $(python3 -c "import json;print(json.load(open('$O/s_${pf}_$i.json'))['ms_per_step'])")"
  done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_d4pg_agent_gpu.py tests/test_d4pg_gpu.py > $O/tests.log 2>&1; tail -1 $O/tests.log
