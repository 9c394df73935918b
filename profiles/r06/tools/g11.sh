# Round-6 call 11: owner-thread update kernel: replay/DQN/DP tests, stamps, bench.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g11; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_replay_gpu.py tests/test_dqn_headline_gpu.py tests/test_prefetch_order_gpu.py tests/test_dp_bench_gpu.py tests/test_step_guard_gpu.py tests/test_r2d2_replay_gpu.py -k "not long_horizon" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/update_stamps.py > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 3; }
grep -v amdgpu $O/stamps.log | tail -10
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench200.json 2> $O/bench200.err || { tail -5 $O/bench200.err; exit 6; }
python3 -c "
import json; d=json.load(open('$O/bench200.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k in d['kernels'][:22]: print('  %-22s %8.2f %s' % (k['name'], k['avg_us'], k.get('frac')))"
