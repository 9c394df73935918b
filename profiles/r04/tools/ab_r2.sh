# A/B of tune variants on the DQN step: alternating step-time runs, then one profiled run each.
# Usage: bash profiles/r04/tools/ab_r2.sh "base HEAD=2,ADAMNT=1 ..." [rounds]
set -e
mkdir -p gpurun_out/ab
V=${1:-"base HEAD=2,ADAMNT=1"}
R=${2:-3}
envs() { [ $1 = base ] && return 0; echo "$1" | tr ',' '\n' | sed 's/^/ACME_V_/' | tr '\n' ' '; }
for i in $(seq 1 $R); do
  for v in $V; do
    env $(envs $v) timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 0 > gpurun_out/ab/step_${v}_$i.json 2>/dev/null
    echo "$v $i $(python3 -c "import json;print(json.load(open('gpurun_out/ab/step_${v}_$i.json'))['ms_per_step'])")"
  done
done
for v in $V; do
  env $(envs $v) timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 100 --warmup 20 > gpurun_out/ab/prof_${v}.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/ab/prof_${v}.json'))
print('$v', {k['name']:k['avg_us'] for k in d['kernels'] if k['name'].endswith('_reduce') or k['name'] in ('fc_head_fwd','adam')})"
done
