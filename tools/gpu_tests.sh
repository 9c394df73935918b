# A selection of the -m gpu tests in one process, each test bounded (usage under gpurun:
# bash tools/gpu_tests.sh OUTDIR test_file.py [...]).
set -u
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -10
exit $rc
