# Round-end check: the whole -m gpu suite, smoke(), then the default bench line.
set -u
mkdir -p gpurun_out/check
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/check/tests.log 2>&1
rc=$?
tail -3 gpurun_out/check/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/check/smoke.log 2>&1 || { tail -5 gpurun_out/check/smoke.log; exit 3; }
tail -1 gpurun_out/check/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/check/bench_driver_like.json 2> gpurun_out/check/bench.err
python3 -c "import json;d=json.load(open('gpurun_out/check/bench_driver_like.json'));print('bench(20/5)', d['value'], d['ms_per_step'], d.get('settle_steps'))"
exit $rc
