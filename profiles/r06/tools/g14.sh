#!/bin/bash
# Pipelined sample + gather: parity tests, the isolated replay timing, the headline test.
set -o pipefail
mkdir -p gpurun_out/g14
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_replay_gpu.py -k "pipelined or fused_sample or prefetched_dataset" \
  > gpurun_out/g14/replay.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_insert_gpu.py tests/test_prefetch_order_gpu.py tests/test_dqn_headline_gpu.py \
  > gpurun_out/g14/insert.log 2>&1 &&
timeout -k 10 180 python -u tools/replay_bench.py > gpurun_out/g14/replay_bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 > gpurun_out/g14/bench.log 2>&1
