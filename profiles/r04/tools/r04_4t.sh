# Round 4: the guard tests on the default build; the free-running trajectory with the
# four-term build (ACME_LIB_PATH); step-time A/B of the two builds (alternating runs).
mkdir -p gpurun_out/r04c
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_step_guard_gpu.py > gpurun_out/r04c/guard.log 2>&1
rc=$?; echo "guard rc=$rc"; tail -5 gpurun_out/r04c/guard.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DIAG_TAG=_4t ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_4t.so timeout -k 10 300 python tools/plane_diag.py traj > gpurun_out/r04c/traj4t.log 2>&1 || exit $?
tail -3 gpurun_out/r04c/traj4t.log
for i in 1 2 3; do
  for v in base 4t; do
    if [ $v = 4t ]; then export ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_4t.so; else unset ACME_LIB_PATH; fi
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 300 --warmup 30 --profile-steps 0 --no-staged > gpurun_out/r04c/s_${v}_$i.json 2>/dev/null || exit $?
    echo "$v $i $(python3 -c "import json;print(json.load(open('gpurun_out/r04c/s_${v}_$i.json'))['ms_per_step'])")"
  done
done
unset ACME_LIB_PATH
