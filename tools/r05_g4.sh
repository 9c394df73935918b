set -u
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 200 python -u tools/grad_err_diag.py --out $O --B 64 --warm 0 2>&1 | grep -v "Warning\|Consider\|return {k\|amdgpu.ids" > $O/g64_0.log || { echo fail; tail -5 $O/g64_0.log; exit 1; }
cat $O/g64_0.log
timeout -k 10 400 python -u tools/drift_diag.py --out $O --tag t32 --B 64 --steps 100 --engines torch32,plane,f32 > $O/d64.log 2>&1 || { echo fail d; tail -5 $O/d64.log; exit 1; }
grep -v amdgpu $O/d64.log
timeout -k 10 400 python -u tools/drift_diag.py --out $O --tag t32 --B 512 --steps 20 --every 5 --engines torch32 > $O/d512.log 2>&1 || { echo fail d; tail -5 $O/d512.log; exit 1; }
grep -v amdgpu $O/d512.log
