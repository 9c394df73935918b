# Round 4 last run after the second stream's priority change: smoke, the whole -m gpu suite,
# the DQN profile refresh (kernel stats, PMC traffic), then every bench line.
mkdir -p gpurun_out/fin4
B=gpurun_out/fin4
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $B/smoke.log 2>&1 || { tail -5 $B/smoke.log; exit 1; }
echo "smoke: $(tail -1 $B/smoke.log)"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $B/gpu.log 2>&1
rc=$?; echo "gpu rc=$rc"; tail -1 $B/gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $B/gpu.log | head; exit $rc; fi
bash tools/profile_round.sh dqn || exit $?
f=$(find gpurun_out/prof_dqn -name '*kernel_stats.csv' | head -1); cp "$f" $B/rocprof_dqn_kernel_stats.csv
find gpurun_out/prof_dqn -name '*kernel_trace.csv' -delete
bash profiles/r04/tools/r04_bench.sh
