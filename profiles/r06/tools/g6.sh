# Round-6 call 6: drift over 4 seeds at B=64/256/512, split accumulators vs one accumulator.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g6; mkdir -p $O
timeout -k 10 500 python -u tools/drift_seeds.py --seeds 4 --out $O/split > $O/split.log 2>&1 || { tail -20 $O/split.log; exit 4; }
grep -v amdgpu $O/split.log
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_onacc.so timeout -k 10 500 python -u tools/drift_seeds.py --seeds 4 --out $O/onacc > $O/onacc.log 2>&1 || { tail -20 $O/onacc.log; exit 5; }
grep -v amdgpu $O/onacc.log
