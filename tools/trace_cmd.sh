set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/trace
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace/raw -- python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --profile-steps 0 --no-staged > gpurun_out/trace/bench.json 2> gpurun_out/trace/bench.err
f=$(find gpurun_out/trace/raw -name '*kernel_trace.csv' | head -1)
python3 tools/trace_step.py "$f" 20 > gpurun_out/trace/step.txt
cp "$f" gpurun_out/trace/kernel_trace.csv
echo done
