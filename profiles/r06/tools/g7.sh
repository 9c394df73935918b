# Round-6 call 7: replay + DP rehearsal tests, the bench (split accumulators, two-round update),
# multi-seed drift split vs one accumulator.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g7; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_replay_gpu.py tests/test_dp_bench_gpu.py tests/test_step_guard_gpu.py -k "not long_horizon" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err || { tail -5 $O/bench20.err; exit 5; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench200.json 2> $O/bench200.err || { tail -5 $O/bench200.err; exit 6; }
python3 - <<'PY'
import json
for n in ("bench20", "bench200"):
    d = json.load(open(f"gpurun_out/r06g7/{n}.json"))
    print(n, d["value"], d["ms_per_step"], d["roofline"]["frac"], d.get("step_guard"))
    for k in d["kernels"][:24]: print("  %-22s %8.2f %s" % (k["name"], k["avg_us"], k.get("frac")))
PY
timeout -k 10 500 python -u tools/drift_seeds.py --seeds 4 --out $O/split > $O/split.log 2>&1 || { tail -20 $O/split.log; exit 4; }
grep -v amdgpu $O/split.log
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_onacc.so timeout -k 10 500 python -u tools/drift_seeds.py --seeds 4 --out $O/onacc > $O/onacc.log 2>&1 || { tail -20 $O/onacc.log; exit 5; }
grep -v amdgpu $O/onacc.log
