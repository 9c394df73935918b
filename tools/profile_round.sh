#!/bin/bash
# GPU-box half of a profile refresh for one workload (run under gpurun):
#   kernel trace + stats, and separate FETCH_SIZE / WRITE_SIZE PMC passes
#   (MI355X_MICROARCH.md: one counter group per pass, --kernel-trace free).
# ACME_V_SIDE=1: every kernel on one stream, so each traced duration is the kernel's own
# (uncontended) time, as bench.py's live section profiler measures it; the timed region of a
# plain bench run overlaps the target forward / weight gradients on a second stream.
# STEPS / PSTEPS: steps of the trace run / of each PMC pass (defaults 100 / 20).
# Locally afterwards: tools/pmc_traffic.py <workload> gpurun_out/pmc_fetch_<w> \
#   gpurun_out/pmc_write_<w> profiles/<round>/pmc_traffic_<w>.json, then the bench line.
set -eo pipefail
W=${1:-dqn}
STEPS=${STEPS:-100}
PSTEPS=${PSTEPS:-20}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_$W gpurun_out/pmc_fetch_$W gpurun_out/pmc_write_$W
export ACME_V_SIDE=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$W \
  -- python3 bench.py --workload $W --no-cpu-baseline --steps $STEPS --warmup 5 \
  > gpurun_out/prof_$W.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$W \
  -- python3 bench.py --workload $W --no-cpu-baseline --steps $PSTEPS --warmup 2 --profile-steps 3 \
  > gpurun_out/pmc_fetch_$W.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$W \
  -- python3 bench.py --workload $W --no-cpu-baseline --steps $PSTEPS --warmup 2 --profile-steps 3 \
  > gpurun_out/pmc_write_$W.log 2>&1
echo "profile_round $W done"
