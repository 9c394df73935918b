#!/bin/bash
# Round-6 call 46: Adam's stores non-temporal beyond the moments: the parameters (nap), the
# parameter planes (nal), both (nab); headline test on nab, then three alternating rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g46; mkdir -p $O
ACME_LIB_PATH=$PWD/acme_amd/libacme_hip_nab.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dqn_headline_gpu.py > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 3; }
tail -1 $O/tests.log
VARS="nap nal nab" W=dqn timeout -k 10 900 bash tools/ab_libs.sh $O/ab > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 4; }
head -12 $O/ab.log
