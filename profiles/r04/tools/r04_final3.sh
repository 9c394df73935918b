# Round 4 last run: smoke, the whole -m gpu suite, the R2D2 profile refresh (kernel stats,
# PMC traffic) after its weight-gradient changes, then every bench line (profiles/r04/tools/r04_bench.sh).
mkdir -p gpurun_out/fin3
B=gpurun_out/fin3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $B/smoke.log 2>&1 || { tail -5 $B/smoke.log; exit 1; }
echo "smoke: $(tail -1 $B/smoke.log)"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $B/gpu.log 2>&1
rc=$?; echo "gpu rc=$rc"; tail -1 $B/gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $B/gpu.log | head; exit $rc; fi
STEPS=10 PSTEPS=3 bash tools/profile_round.sh r2d2 || exit $?
f=$(find gpurun_out/prof_r2d2 -name '*kernel_stats.csv' | head -1); cp "$f" $B/rocprof_r2d2_kernel_stats.csv
find gpurun_out/prof_r2d2 -name '*kernel_trace.csv' -delete
bash profiles/r04/tools/r04_bench.sh
