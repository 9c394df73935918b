#!/bin/bash
# Round-6 call 35: target fc_fwd at split-K 8, confirmation: six alternating 300-step pairs, then
# three alternating pairs of the driver's window (20 timed steps after 5 warm-up steps).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g35; mkdir -p $O
for r in 1 2; do
A="" B="ACME_V_TSPLIT=8" EXTRA="--no-staged" timeout -k 10 600 bash tools/ab_env.sh $O/t$r > $O/t$r.log 2>&1 || { tail -5 $O/t$r.log; exit 4; }
head -6 $O/t$r.log
done
for i in 1 2 3; do
  for v in A B; do
    if [ $v = B ]; then E="ACME_V_TSPLIT=8"; else E=""; fi
    env $E timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/w_${v}_$i.json 2> $O/w_${v}_$i.err || exit 5
    echo "window $v $i $(python3 -c "import json;print(json.load(open('$O/w_${v}_$i.json'))['ms_per_step'])")"
  done
done
