# One GPU call: the -m gpu tests (or a subset), then (only if pytest ended with passes or
# plain test failures, never after a crash, abort or time limit) the default bench line.
# Usage (under gpurun): bash tools/gpu_run.sh OUT "pytest selection" "bench args"|none
set -u
out=gpurun_out/$1
mkdir -p "$out"
sel=${2:-"tests -m gpu"}
timeout -k 10 900 python -u -m pytest $sel -x -q --timeout 200 --timeout-method thread \
  > "$out/tests.log" 2>&1
rc=$?
tail -3 "$out/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
  echo "pytest exited $rc: no further GPU work in this call"
  exit $rc
fi
if [ "${3:-}" != "none" ]; then
  timeout -k 10 300 python bench.py ${3:-} > "$out/bench.json" 2> "$out/bench.err"
  brc=$?
  python3 -c "import json;d=json.load(open('$out/bench.json'));print('bench', d['value'], d['ms_per_step'])" || true
  exit $brc
fi
exit $rc
