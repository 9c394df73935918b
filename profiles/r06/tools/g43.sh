#!/bin/bash
# Round-6 call 43: split Adam (ACME_V_SADAM=1): the write-back (and the step's verdict) before
# conv1's weight gradient, the side stream's Adam over conv2 / conv3 / dense beside that weight
# gradient, conv1's Adam (with the tail) on the main stream after the join.  The DQN, guard,
# replay and checkpoint tests with it, then six alternating 300-step pairs and three driver
# windows each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g43; mkdir -p $O
ACME_V_SADAM=1 timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py tests/test_step_guard_gpu.py tests/test_checkpoint_gpu.py tests/test_replay_gpu.py -k "not long_horizon" > $O/tests.log 2>&1 || { tail -12 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for r in 1 2; do
A="" B="ACME_V_SADAM=1" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$r > $O/t$r.log 2>&1 || { tail -5 $O/t$r.log; exit 4; }
head -6 $O/t$r.log
done
for i in 1 2 3; do
  for v in A B; do
    if [ $v = B ]; then E="ACME_V_SADAM=1"; else E=""; fi
    env $E timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/w_${v}_$i.json 2> $O/w_${v}_$i.err || exit 5
    echo "window $v $i $(python3 -c "import json;print(json.load(open('$O/w_${v}_$i.json'))['ms_per_step'])")"
  done
done
