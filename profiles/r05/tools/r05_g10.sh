# Round 5: where the DQN step's time goes -- a two-stream kernel trace, the producer /
# consumer bottleneck builds (WS_EXP=1: producers idle, 2: consumers idle; timing only, the
# results are wrong), and an LDS / instruction-mix PMC pass.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05g10; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_replay_gpu.py tests/test_dqn_headline_gpu.py tests/test_dp_bench_gpu.py tests/test_checkpoint_gpu.py > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
#timeout -k 10 300 bash tools/trace_cmd.sh > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
#head -80 gpurun_out/trace/step.txt
for v in ws1 ws2; do
  ACME_BENCH_ON_OVERFLOW=skip ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_$v.so timeout -k 10 150 python3 bench.py --no-cpu-baseline --steps 60 --warmup 20 --no-staged > $O/p_$v.json 2>$O/p_$v.err || { echo $v failed; tail -3 $O/p_$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/p_$v.json'))
print('$v', {k['name']:k['avg_us'] for k in d['kernels'][:16]})"
done
ACME_V_SIDE=1 timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_lds_dqn \
  -- python3 bench.py --workload dqn --no-cpu-baseline --steps 20 --warmup 2 --profile-steps 3 \
  > $O/pmc_lds.log 2>&1 || { echo pmc failed; tail -5 $O/pmc_lds.log; exit 1; }
python3 tools/pmc_mfma.py dqn gpurun_out/pmc_lds_dqn gpurun_out/pmc_lds_dqn.json
