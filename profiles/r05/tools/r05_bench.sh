# Round 5 bench records: the driver's command line, the default run, and a rocprofv3 kernel
# trace + stats of the driver's command (no CPU baseline) for the roofline kernel.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05bench; mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driverlike.json 2> $O/bench_driverlike.err || { tail -5 $O/bench_driverlike.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_driverlike.json'));print('20/5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline'])"
timeout -k 10 600 python3 bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('200/20', d['value'], d['ms_per_step'], d['roofline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -5 $O/prof_bench.err; exit 1; }
echo prof done
