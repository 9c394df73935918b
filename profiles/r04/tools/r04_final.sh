# Round 4 final: the whole -m gpu suite, the DQN profile refresh (kernel stats, PMC traffic
# passes), then the DQN bench line and three 20-step windows.
mkdir -p gpurun_out/fin
B=gpurun_out/fin
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $B/smoke.log 2>&1 || { tail -5 $B/smoke.log; exit 1; }
echo "smoke ok: $(tail -1 $B/smoke.log)"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $B/gpu.log 2>&1
rc=$?; echo "gpu rc=$rc"; tail -2 $B/gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $B/gpu.log | head; exit $rc; fi
bash tools/profile_round.sh dqn || exit $?
f=$(find gpurun_out/prof_dqn -name '*kernel_stats.csv' | head -1); cp "$f" $B/rocprof_dqn_kernel_stats.csv
find gpurun_out/prof_dqn -name '*kernel_trace.csv' -delete
timeout -k 10 400 python3 bench.py > $B/bench_dqn.json 2> $B/bench_dqn.err || exit $?
echo "dqn $(python3 -c "import json;d=json.load(open('$B/bench_dqn.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_us'])")"
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-steps 0 --no-staged > $B/w20_$i.json 2>/dev/null || exit $?
  echo "w20 $i $(python3 -c "import json;d=json.load(open('$B/w20_$i.json'));print(d['value'],d['ms_per_step'])")"
done
