# MFMA-busy / stall counters (one pass) and the HBM-traffic passes for the DQN bench, each
# pass its own rocprofv3 run (MI355X_MICROARCH.md PMC slots), then the kernel trace + stats.
set -eo pipefail
W=${1:-dqn}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_mfma_$W gpurun_out/pmc_fetch_$W gpurun_out/pmc_write_$W gpurun_out/prof_$W
export ACME_V_SIDE=1
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_mfma_$W \
  -- python3 bench.py --workload $W --no-cpu-baseline --steps 20 --warmup 2 --profile-steps 3 \
  > gpurun_out/pmc_mfma_$W.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$W \
  -- python3 bench.py --workload $W --no-cpu-baseline --steps 20 --warmup 2 --profile-steps 3 \
  > gpurun_out/pmc_fetch_$W.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$W \
  -- python3 bench.py --workload $W --no-cpu-baseline --steps 20 --warmup 2 --profile-steps 3 \
  > gpurun_out/pmc_write_$W.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$W \
  -- python3 bench.py --workload $W --no-cpu-baseline --steps 100 --warmup 5 \
  > gpurun_out/prof_$W.log 2>&1
python3 tools/pmc_mfma.py $W gpurun_out/pmc_mfma_$W gpurun_out/pmc_mfma_$W.json
python3 tools/pmc_traffic.py $W gpurun_out/pmc_fetch_$W gpurun_out/pmc_write_$W gpurun_out/pmc_traffic_$W.json
echo "pmc $W done"
