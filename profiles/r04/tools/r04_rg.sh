# One-launch LSTM unroll: the R2D2 and IMPALA GPU tests, the per-step phase trace, then the
# R2D2 and IMPALA bench lines.
mkdir -p gpurun_out/rg
B=gpurun_out/rg
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_r2d2_learner_gpu.py tests/test_impala_gpu.py > $B/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $B/tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" $B/tests.log | head -20; exit $rc; fi
timeout -k 10 200 python3 tools/rg_trace.py 2>&1 | grep -v amdgpu.ids || exit $?
for w in r2d2 impala; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > $B/bench_$w.json 2> $B/bench_$w.err || exit $?
  python3 -c "import json;d=json.load(open('$B/bench_$w.json'));k={x['name']:x['avg_us'] for x in d['kernels']};print('$w',d['value'],d['ms_per_step'],{n:v for n,v in k.items() if 'lstm' in n})"
done
