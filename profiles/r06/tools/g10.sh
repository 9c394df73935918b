# Round-6 call 10: update-kernel phase stamps, then the whole -m gpu suite.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g10; mkdir -p $O
timeout -k 10 200 python3 tools/update_stamps.py > $O/stamps.log 2>&1 || { tail -5 $O/stamps.log; exit 3; }
grep -v amdgpu $O/stamps.log | tail -30
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8; exit $rc
