# Round 4: the step-guard tests, the whole -m gpu suite, the plane diagnostics, a bench.
mkdir -p gpurun_out/r04d
run() {  # run <name> <seconds> <cmd...>; a pytest status 1 (failures) continues
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/r04d/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 gpurun_out/r04d/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run guard 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_step_guard_gpu.py
run gpu 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ --deselect tests/test_step_guard_gpu.py
run diag 300 python tools/plane_diag.py overflow
run bench 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline
