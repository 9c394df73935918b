# The DQN bench lines on the final round-5 code: the default 200-step run, then the driver's
# command line, on a fresh box.
set -u
O=gpurun_out/r05g45; mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench_dqn.json 2> $O/bench_dqn.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_dqn.json'));print('200 steps', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_dqn_20x5.json 2> $O/bench_dqn_20x5.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_dqn_20x5.json'));print('20x5', d['value'], d['ms_per_step'], d['roofline']['frac'])"
