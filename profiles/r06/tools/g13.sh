# Round-6 call 13: replay micro-benchmark (fused / draw / gather / d2d / update) and update stamps.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g13; mkdir -p $O
timeout -k 10 200 python3 tools/replay_bench.py > $O/replay_bench.log 2>&1 || { tail -5 $O/replay_bench.log; exit 3; }
grep -v amdgpu $O/replay_bench.log
timeout -k 10 200 python3 tools/update_stamps.py > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 4; }
grep -v amdgpu $O/stamps.log | tail -10
