#!/bin/bash
# Round-6 call 53: the draw's prefix scan with DPP wave shifts for rounds 1..8 (the same
# additions; LDS permutes only for 16 and 32), libacme_hip_dpp.so: replay / R2D2 / DQN parity
# tests on it, the isolated replay bench for both builds, then alternating 300-step pairs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g53; mkdir -p $O
D=$PWD/acme_amd/libacme_hip_dpp.so
ACME_LIB_PATH=$D timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_replay_gpu.py tests/test_r2d2_replay_gpu.py tests/test_dqn_gpu.py -k "not long_horizon" > $O/tests.log 2>&1 || { tail -12 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for v in base dpp; do
  if [ $v = base ]; then L=""; else L=$D; fi
  ACME_LIB_PATH=$L timeout -k 10 200 python3 tools/replay_bench.py > $O/replay_bench_$v.log 2>&1 || { tail -5 $O/replay_bench_$v.log; exit 5; }
  echo "== $v"; grep -v amdgpu $O/replay_bench_$v.log
done
VARS="dpp" timeout -k 10 600 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 6; }
cat $O/ab.log
