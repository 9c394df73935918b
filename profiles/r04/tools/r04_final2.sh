# Round 4 closing run: smoke, the whole -m gpu suite, profile refresh (kernel stats + PMC
# traffic) for IMPALA and R2D2 after their LSTM / tile changes, then every bench line.
mkdir -p gpurun_out/fin2
B=gpurun_out/fin2
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $B/smoke.log 2>&1 || { tail -5 $B/smoke.log; exit 1; }
echo "smoke: $(tail -1 $B/smoke.log)"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $B/gpu.log 2>&1
rc=$?; echo "gpu rc=$rc"; tail -1 $B/gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $B/gpu.log | head; exit $rc; fi
bash tools/profile_round.sh impala || exit $?
STEPS=10 PSTEPS=3 bash tools/profile_round.sh r2d2 || exit $?
for w in impala r2d2; do
  f=$(find gpurun_out/prof_$w -name '*kernel_stats.csv' | head -1); cp "$f" $B/rocprof_${w}_kernel_stats.csv
  find gpurun_out/prof_$w -name '*kernel_trace.csv' -delete
done
echo profiles done
