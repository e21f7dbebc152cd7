#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
WPAIR=1 timeout -k 10 200 python -u tools/exp/win_stamp.py > $O/r5_winfwd_b1_stamps.log 2>&1; rc=$?
grep -v amdgpu.ids $O/r5_winfwd_b1_stamps.log; exit $rc
