# Round 4: the -m gpu suite, one process, each test bounded.
mkdir -p gpurun_out/r04t
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04t/gpu.log 2>&1
rc=$?; echo "gpu rc=$rc"; tail -15 gpurun_out/r04t/gpu.log
exit $rc
