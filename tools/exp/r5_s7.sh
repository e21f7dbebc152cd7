#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/exp/bwd_flags_diag.py > gpurun_out/r5_bwd_flags.log 2>&1; rc=$?
cat gpurun_out/r5_bwd_flags.log; exit $rc
