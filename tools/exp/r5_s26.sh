#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 200 python -u tools/exp/win_bwd_stamp.py 1 4 > $O/r5_winbwd_b1_stamps.log 2>&1; rc=$?
grep -v amdgpu.ids $O/r5_winbwd_b1_stamps.log; exit $rc
