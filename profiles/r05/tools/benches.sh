# The other workloads' bench lines at the end of round 5.
set -u
O=gpurun_out/r05_benches; mkdir -p $O
for w in impala r2d2 impala_actors; do
  timeout -k 10 420 python3 bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "$w failed"; tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w', d['value'], d['unit'], d['ms_per_step'])"
done
