#!/bin/bash
# Round-6 call 17: the DQN counter passes (MFMA busy / stalls, FETCH_SIZE, WRITE_SIZE) and the
# kernel trace + stats, each its own rocprofv3 run (tools/pmc_passes.sh), then the LDS pass.
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/pmc_passes.sh dqn > gpurun_out/g17_pmc.log 2>&1 || { tail -20 gpurun_out/g17_pmc.log; exit 3; }
tail -3 gpurun_out/g17_pmc.log
