set -u
O=gpurun_out/r05c; mkdir -p $O
for w in 0 1 3 10; do
timeout -k 10 200 python -u tools/grad_err_diag.py --out $O --B 64 --warm $w 2>&1 | grep -v "Warning\|Consider\|return {k\|amdgpu.ids" > $O/g64_$w.log || { echo fail; tail -5 $O/g64_$w.log; exit 1; }
echo "== warm $w"; cat $O/g64_$w.log
done
