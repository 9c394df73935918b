# DQN step schedule changes: their tests, then A/B step time (ACME_V_* variants), then a trace.
set -eo pipefail
timeout -k 10 400 python -u -m pytest tests/test_dqn_gpu.py tests/test_dqn_headline_gpu.py tests/test_dp.py tests/test_insert_gpu.py tests/test_prefetch_order_gpu.py tests/test_checkpoint_gpu.py tests/test_golden_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/upd_tests.log 2>&1
tail -2 gpurun_out/upd_tests.log
bash profiles/r04/tools/ab_r2.sh "${AB:-base UPDQ=1}" 3
bash tools/trace_cmd.sh
python3 tools/trace_abs.py gpurun_out/trace/kernel_trace.csv 20 adam_slabs > gpurun_out/trace/abs.txt
