# Round 4: the -m gpu suite, then every bench line (profiles/r04/tools/r04_bench.sh).
mkdir -p gpurun_out/r04b
B=gpurun_out/r04b
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $B/gpu.log 2>&1
rc=$?; echo "gpu rc=$rc"; tail -4 $B/gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $B/gpu.log | head; exit $rc; fi
bash profiles/r04/tools/r04_bench.sh
