# Round-6 call 12: update kernel (bounded loops): tests + stamps; sample_gather vs replay size.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g12; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_replay_gpu.py tests/test_dqn_headline_gpu.py tests/test_step_guard_gpu.py -k "not long_horizon" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/update_stamps.py > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 3; }
grep -v amdgpu $O/stamps.log | tail -10
for RS in 1000000 16384; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-staged --replay-size $RS > $O/bench_$RS.json 2> $O/bench_$RS.err || { tail -5 $O/bench_$RS.err; exit 6; }
python3 -c "
import json; d=json.load(open('$O/bench_$RS.json')); print('$RS', d['value'], d['ms_per_step'])
for k in d['kernels']:
  if k['name'] in ('replay_sample_gather','replay_update','fc_fwd'): print('  %-22s %8.2f %s' % (k['name'], k['avg_us'], k.get('frac')))"
done
