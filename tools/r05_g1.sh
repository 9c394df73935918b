set -u
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 300 python -u tools/drift_diag.py --out $O --tag 3t --B 64 --steps 100 > $O/d3_64.log 2>&1 || { echo fail d3; tail -5 $O/d3_64.log; exit 1; }
tail -3 $O/d3_64.log
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_4t.so timeout -k 10 300 python -u tools/drift_diag.py --out $O --tag 4t --B 64 --steps 100 --engines plane > $O/d4_64.log 2>&1 || { echo fail d4; tail -5 $O/d4_64.log; exit 1; }
tail -2 $O/d4_64.log
timeout -k 10 300 python -u tools/drift_diag.py --out $O --tag 3t --B 512 --steps 20 --every 5 > $O/d3_512.log 2>&1 || { echo fail d3b; tail -5 $O/d3_512.log; exit 1; }
tail -3 $O/d3_512.log
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_4t.so timeout -k 10 300 python -u tools/drift_diag.py --out $O --tag 4t --B 512 --steps 20 --every 5 --engines plane > $O/d4_512.log 2>&1 || { echo fail d4b; exit 1; }
tail -2 $O/d4_512.log
VAR=4t timeout -k 10 900 bash tools/ab_variant.sh > $O/ab4t.log 2>&1; tail -12 $O/ab4t.log
