# D4PG: parity tests, the bench line (with its CPU baseline), rocprofv3 kernel stats.
set -u
O=gpurun_out/${OUT:-r05g32}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_d4pg_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py --workload d4pg > $O/bench_d4pg.json 2> $O/bench_d4pg.err || exit 1
tail -c 600 $O/bench_d4pg.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 bench.py --workload d4pg --no-cpu-baseline --steps 200 --warmup 20 --profile-steps 0 --no-staged > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$f" $O/rocprof_d4pg_kernel_stats.csv
find $O/prof -name '*kernel_trace.csv' -delete
echo done
