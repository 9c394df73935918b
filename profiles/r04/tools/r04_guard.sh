# Round 4: the step-guard tests, then the whole -m gpu suite, then a short DQN bench.
# A pytest exit status of 1 (test failures) continues; anything else (a crash, a time
# limit) stops the script.
mkdir -p gpurun_out/r04b
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/r04b/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -3 gpurun_out/r04b/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run guard 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_step_guard_gpu.py
run gpu 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/
run bench 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline
