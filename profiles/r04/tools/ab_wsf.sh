# Same-box A/B of the warp-specialised plane GEMMs (fc_fwd, fc_dgrad, conv2_fwd, conv1_wgrad) against
# the single-role kernels (ACME_V_WSN=1): alternating bench runs with section profiles;
# prints step time and the affected kernels.  Run under gpurun.
set -e
mkdir -p gpurun_out
run() { env $1 timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 150 --warmup 20 --profile-steps 30 > gpurun_out/wsf_$2.json 2>/dev/null; }
run ACME_V_WSN=1 n1
run ACME_V_WSN=0 n0
run ACME_V_WSN=1 n1b
run ACME_V_WSN=0 n0b
for t in n1 n0 n1b n0b; do python3 -c "
import json;d=json.load(open('gpurun_out/wsf_$t.json'));k={x['name']:x['avg_us'] for x in d['kernels']}
print('$t', d['ms_per_step'], *[(n, k.get(n)) for n in ('fc_fwd','fc_dgrad','conv1_wgrad')])"; done
