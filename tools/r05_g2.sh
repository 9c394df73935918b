set -u
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 200 python -u tools/grad_err_diag.py --out $O --B 64 --warm 0 > $O/g64_0.log 2>&1 || { echo fail; tail -5 $O/g64_0.log; exit 1; }
cat $O/g64_0.log | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/grad_err_diag.py --out $O --B 64 --warm 30 > $O/g64_30.log 2>&1 || { echo fail; tail -5 $O/g64_30.log; exit 1; }
cat $O/g64_30.log | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/grad_err_diag.py --out $O --B 512 --warm 10 > $O/g512_10.log 2>&1 || { echo fail; tail -5 $O/g512_10.log; exit 1; }
cat $O/g512_10.log | grep -v amdgpu.ids
