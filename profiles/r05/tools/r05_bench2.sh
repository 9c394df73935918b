# Round 5: the driver's command line with the bounded CPU baseline, and a rocprofv3 summary of
# the same command with every kernel on one stream (ACME_V_SIDE=1, as the bench's own
# profiled pass runs them), whose fc_fwd average is comparable with the bench's live one.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05bench2; mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driverlike.json 2> $O/bench_driverlike.err || { tail -5 $O/bench_driverlike.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_driverlike.json'));print('20/5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_us'], d['cpu_baseline'])"
ACME_V_SIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -5 $O/prof_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/prof_bench.json'));print('side', d['roofline']['avg_us'])"
echo prof done
