# Round 5: fc_fwd experiments -- the slab epilogue's share (a build without the slab stores,
# timing only) and 256x256 single-role tiles (ACME_V_FCT=1) against the 256x128 WS tiles.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05g11; mkdir -p $O
v=noslab
ACME_BENCH_ON_OVERFLOW=skip ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_$v.so timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --no-staged > $O/p_$v.json 2>$O/p_$v.err || { echo $v failed; tail -3 $O/p_$v.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/p_$v.json'))
print('$v', {k['name']:k['avg_us'] for k in d['kernels'][:16]})"
EXTRA=--no-staged A="" B="ACME_V_FCT=1" timeout -k 10 900 bash tools/ab_env.sh $O/ab_fct > $O/ab_fct.log 2>&1; cat $O/ab_fct.log
