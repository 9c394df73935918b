# Round 4 bench lines for every workload (the PMC traffic of profiles/r04 is in place), the
# driver-shaped 20-step DQN windows, and the per-step timing of a short window.
mkdir -p gpurun_out/r04b
B=gpurun_out/r04b
timeout -k 10 400 python3 bench.py > $B/bench_dqn.json 2> $B/bench_dqn.err || exit $?
echo "dqn $(python3 -c "import json;d=json.load(open('$B/bench_dqn.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['cpu_baseline']['value'])")"
for i in 1 2 3; do
  timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-steps 0 --no-staged > $B/w20_$i.json 2>/dev/null || exit $?
  echo "w20 $i $(python3 -c "import json;d=json.load(open('$B/w20_$i.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 200 python3 tools/window_steps.py 20 3 > $B/window_steps.txt 2>&1 || exit $?
cat $B/window_steps.txt | grep -v amdgpu
timeout -k 10 300 python3 bench.py --workload d4pg > $B/bench_d4pg.json 2> $B/bench_d4pg.err || exit $?
echo "d4pg $(python3 -c "import json;d=json.load(open('$B/bench_d4pg.json'));print(d['value'],d['ms_per_step'],d['roofline'])")"
timeout -k 10 300 python3 bench.py --workload impala > $B/bench_impala.json 2> $B/bench_impala.err || exit $?
echo "impala $(python3 -c "import json;d=json.load(open('$B/bench_impala.json'));print(d['value'],d['ms_per_step'],d['roofline'],d.get('lstm'))")"
timeout -k 10 300 python3 bench.py --workload r2d2 --steps 20 --warmup 3 --profile-steps 5 > $B/bench_r2d2.json 2> $B/bench_r2d2.err || exit $?
echo "r2d2 $(python3 -c "import json;d=json.load(open('$B/bench_r2d2.json'));print(d['value'],d['ms_per_step'],d['roofline'],d['cpu_baseline']['value'])")"
timeout -k 10 300 python3 bench.py --workload impala_actors --steps 300 --warmup 20 > $B/bench_impala_actors.json 2> $B/bench_impala_actors.err || exit $?
echo "actors $(python3 -c "import json;d=json.load(open('$B/bench_impala_actors.json'));print(d['value'],d.get('actors'))")"
