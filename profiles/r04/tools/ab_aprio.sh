# (Round-4 record: the APRIO hook was removed after this A/B; the high priority kept.)
# A/B: the pipelined actor policy's stream at the default priority (ACME_V_APRIO=0) against
# the high priority (unset), IMPALA end to end, three alternating pairs.
mkdir -p gpurun_out/aprio
O=gpurun_out/aprio
for i in 1 2 3; do
  for v in hi 0; do
    if [ $v = 0 ]; then export ACME_V_APRIO=0; else unset ACME_V_APRIO; fi
    timeout -k 10 200 python3 bench.py --workload impala_actors --steps 300 --warmup 20 --no-cpu-baseline > $O/a${v}_$i.json 2>/dev/null || exit $?
    python3 -c "
import json
d=json.load(open('$O/a${v}_$i.json')); print('$v $i', d['value'], d.get('actors', {}).get('env_steps_per_s'))"
  done
done
unset ACME_V_APRIO
