#!/bin/bash
# Round-6 call 55: the round-end code on another box: the driver's command line and a 200-step
# DQN line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g55; mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 14
timeout -k 10 600 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_dqn.json 2> $O/bench_dqn.err || exit 15
python3 -c "
import json
for f in ('bench_driver', 'bench_dqn'):
    d = json.load(open('$O/%s.json' % f)); print(f, d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"
