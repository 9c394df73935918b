# rocprofv3 kernel trace of the D4PG step (direct-engine build): per-launch durations and gaps.
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05g26; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/raw -- python3 bench.py --workload d4pg --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > $O/bench.json 2> $O/bench.err
f=$(find $O/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_step.py "$f" 20 clip_adam > $O/step.txt
cp "$f" $O/kernel_trace.csv
echo done
