# Device-scope vs system-scope stream-order events: ordering tests, A/B step time, trace.
set -eo pipefail
timeout -k 10 400 python -u -m pytest tests/test_prefetch_order_gpu.py tests/test_dqn_headline_gpu.py tests/test_dqn_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ev_tests.log 2>&1
tail -2 gpurun_out/ev_tests.log
bash profiles/r04/tools/ab_r2.sh "${AB:-base DOORBELL=1}" 3
bash tools/trace_cmd.sh
python3 tools/trace_abs.py gpurun_out/trace/kernel_trace.csv 20 > gpurun_out/trace/abs.txt
