set -u
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_step_guard_gpu.py -k "not long_horizon" tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py tests/test_checkpoint_gpu.py tests/test_dp.py > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/grad_err_diag.py --out $O --B 64 --warm 0 2>&1 | grep -v "Warning\|Consider\|return {k\|amdgpu.ids" > $O/g64_0.log || { echo fail; tail -5 $O/g64_0.log; exit 1; }
cat $O/g64_0.log
timeout -k 10 400 python -u tools/drift_diag.py --out $O --tag t32 --B 64 --steps 100 --engines torch32,plane,f32 > $O/d64.log 2>&1 || { echo fail d; tail -5 $O/d64.log; exit 1; }
grep -v amdgpu $O/d64.log
timeout -k 10 400 python -u tools/drift_diag.py --out $O --tag t32 --B 512 --steps 20 --every 5 --engines torch32 > $O/d512.log 2>&1 || { echo fail d; tail -5 $O/d512.log; exit 1; }
grep -v amdgpu $O/d512.log
exit $rc
