set -e
mkdir -p gpurun_out
run() { env $1 timeout -k 10 150 python3 bench.py --workload impala --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/imp_$2.json 2>/dev/null; }
T="f:ACME_V_IMP3=1 p:ACME_V_IMP3=0 fb:ACME_V_IMP3=1 pb:ACME_V_IMP3=0"
for x in $T; do run ${x#*:} ${x%%:*}; done
for x in $T; do t=${x%%:*}; python3 -c "
import json;d=json.load(open('gpurun_out/imp_$t.json'));print('$t', d['value'], d['ms_per_step'])"; done
python3 -c "
import json;d=json.load(open('gpurun_out/imp_pb.json'))
for k in d['kernels']: print(k['name'], k['launches'], k['avg_us'])"
