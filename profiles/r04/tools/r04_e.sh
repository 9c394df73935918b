# Round 4: tests, then step-time A/B: this tree (online head fused into the loss launch),
# the same library with the separate head (ACME_V_HEADSEP=1), and libacme_hip_old.so (the
# step guard commit, before the rescale fused into the priority write-back); 300-step and
# 20-step windows, alternating; then one profiled run each of new and sep.
mkdir -p gpurun_out/r04e
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04e/gpu.log 2>&1
rc=$?; echo "gpu rc=$rc"; tail -4 gpurun_out/r04e/gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  for v in new sep old; do
    unset ACME_LIB_PATH ACME_V_HEADSEP
    if [ $v = old ]; then export ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_old.so; fi
    if [ $v = sep ]; then export ACME_V_HEADSEP=1; fi
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 0 --no-staged > gpurun_out/r04e/s_${v}_$i.json 2>/dev/null || exit $?
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 0 --no-staged > gpurun_out/r04e/w_${v}_$i.json 2>/dev/null || exit $?
    echo "$v $i 300:$(python3 -c "import json;print(json.load(open('gpurun_out/r04e/s_${v}_$i.json'))['ms_per_step'])") 20:$(python3 -c "import json;print(json.load(open('gpurun_out/r04e/w_${v}_$i.json'))['ms_per_step'])")"
  done
done
unset ACME_LIB_PATH ACME_V_HEADSEP
for v in new sep; do
  if [ $v = sep ]; then export ACME_V_HEADSEP=1; fi
  timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 100 --warmup 20 --no-staged > gpurun_out/r04e/p_${v}.json 2>/dev/null || exit $?
  python3 -c "
import json;d=json.load(open('gpurun_out/r04e/p_${v}.json'))
print('$v', {k['name']:k['avg_us'] for k in d['kernels'][:14]})"
done
unset ACME_V_HEADSEP
