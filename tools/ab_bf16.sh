# Same-box alternating A/B of the dataset's bf16 frame copy (ACME_DATASET_BF16=1, default:
# the fused gather writes it and the learner skips frames_bf16) against the learner's own
# conversion (=0); step time and the affected sections.
set -e
mkdir -p gpurun_out
run() { env $1 timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 20 > gpurun_out/bf_$2.json 2>/dev/null; }
for i in 1 2 3; do run ACME_DATASET_BF16=0 d$i; run ACME_DATASET_BF16=1 b$i; done
for t in d1 b1 d2 b2 d3 b3; do python3 -c "
import json;d=json.load(open('gpurun_out/bf_$t.json'));k={x['name']:x['avg_us'] for x in d['kernels']}
print('$t', d['ms_per_step'], k.get('replay_sample_gather'), k.get('frames_bf16'))"; done
