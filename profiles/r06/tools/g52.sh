#!/bin/bash
# Round-6 call 52: the sum tree's totals by a DPP / swizzle butterfly (wave_total64) instead of
# the lane-63 value of the LDS-permute scan: replay / DQN parity tests, write-back stamps and
# the isolated replay bench for both builds (old = the scan, libacme_hip_old.so), then
# alternating 300-step pairs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g52; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_replay_gpu.py tests/test_r2d2_replay_gpu.py tests/test_dqn_gpu.py tests/test_step_guard_gpu.py -k "not long_horizon" > $O/tests.log 2>&1 || { tail -12 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for v in base old; do
  if [ $v = base ]; then L=""; else L=$PWD/acme_amd/libacme_hip_$v.so; fi
  ACME_LIB_PATH=$L timeout -k 10 200 python3 tools/update_stamps.py --steady > $O/stamps_$v.log 2>&1 || { tail -5 $O/stamps_$v.log; exit 4; }
  echo "== $v"; tail -10 $O/stamps_$v.log
  ACME_LIB_PATH=$L timeout -k 10 200 python3 tools/replay_bench.py > $O/replay_bench_$v.log 2>&1 || { tail -5 $O/replay_bench_$v.log; exit 5; }
  grep -v amdgpu $O/replay_bench_$v.log
done
VARS="old" timeout -k 10 600 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 6; }
cat $O/ab.log
