# Round-end DQN evidence: kernel trace + stats and PMC passes (tools/profile_round.sh), then
# the default bench line with its CPU baseline.
set -eo pipefail
bash tools/profile_round.sh dqn
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 bench.py > gpurun_out/bench_dqn_final.json 2> gpurun_out/bench_dqn_final.err
python3 -c "import json;d=json.load(open('gpurun_out/bench_dqn_final.json'));print('bench', d['value'], d['ms_per_step'], d['cpu_baseline'])"
