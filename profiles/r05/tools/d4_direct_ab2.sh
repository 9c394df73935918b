# D4PG direct engine (strided buffer loads, all loads before the products): parity tests,
# A/B against the staged engine, then a kernel trace of the step.
set -u
O=gpurun_out/${OUT:-r05g27}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_d4pg_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
W=d4pg VARS=${VARS:-d4old} timeout -k 10 600 bash tools/ab_libs.sh $O/ab_d4pg > $O/ab_d4pg.log 2>&1; cat $O/ab_d4pg.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/raw -- python3 bench.py --workload d4pg --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > $O/bench.json 2> $O/bench.err || exit 1
f=$(find $O/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_step.py "$f" 20 clip_adam > $O/step.txt
cp "$f" $O/kernel_trace.csv; rm -rf $O/raw
cat $O/step.txt
