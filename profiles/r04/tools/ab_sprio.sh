# (Round-4 record: the SPRIO hook was removed after this A/B; the default priority kept.)
# A/B: the DQN learner's second stream at the default priority (ACME_V_SPRIO=0) against
# the lowest (unset): 200-step runs and 20-step windows, three alternating pairs each.
mkdir -p gpurun_out/sprio
O=gpurun_out/sprio
for i in 1 2 3; do
  for v in low 0; do
    if [ $v = 0 ]; then export ACME_V_SPRIO=0; else unset ACME_V_SPRIO; fi
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-staged --no-profile > $O/s${v}_$i.json 2>/dev/null || exit $?
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-staged --no-profile --steps 20 --warmup 5 > $O/w${v}_$i.json 2>/dev/null || exit $?
    python3 -c "
import json
a=json.load(open('$O/s${v}_$i.json')); b=json.load(open('$O/w${v}_$i.json'))
print('$v $i', a['ms_per_step'], b['ms_per_step'])"
  done
done
unset ACME_V_SPRIO
