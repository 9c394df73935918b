#!/bin/bash
# Round-6 call 16: the rescale workgroup's loads in one round (verdict earlier): replay / guard
# tests, update phase stamps, a 200-step bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g16; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_replay_gpu.py \
  tests/test_dqn_headline_gpu.py tests/test_step_guard_gpu.py -k "not long_horizon" > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/update_stamps.py > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 3; }
grep -v amdgpu $O/stamps.log | tail -10
timeout -k 10 400 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 6; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'])
for k in d['kernels']:
  if k['name'] in ('replay_sample_gather','replay_update','fc_fwd'): print('  %-22s %8.2f %s' % (k['name'], k['avg_us'], k.get('frac')))"
