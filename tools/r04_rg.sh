# One-launch LSTM unroll for R2D2: its tests, IMPALA's (the kernels moved to lstm.h), the
# R2D2 bench line; then the first-step host issue diagnosis of the DQN window.
mkdir -p gpurun_out/rg
B=gpurun_out/rg
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_r2d2_learner_gpu.py tests/test_impala_gpu.py > $B/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error" $B/tests.log | tail -40
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --workload r2d2 > $B/bench_r2d2.json 2> $B/bench_r2d2.err || exit $?
python3 -c "import json;d=json.load(open('$B/bench_r2d2.json'));print('r2d2',d['value'],d['ms_per_step']);[print(k['name'],k['launches'],k['avg_us']) for k in d['kernels'][:12]]"
timeout -k 10 240 python3 tools/first_step.py 20 5 > $B/first_step.txt 2>&1 || exit $?
grep -v amdgpu.ids $B/first_step.txt
