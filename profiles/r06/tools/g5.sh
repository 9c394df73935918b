# Round-6 call 5: where the step-1 loss error comes from (update diagnosis), B=256 and 512.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g5; mkdir -p $O
for B in 256 512; do
timeout -k 10 300 python -u tools/update_diag.py --B $B > $O/update_B$B.log 2>&1 || { tail -20 $O/update_B$B.log; exit 4; }
cat $O/update_B$B.log | grep -v amdgpu.ids
done
