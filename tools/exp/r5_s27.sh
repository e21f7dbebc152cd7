#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 300 python -u tools/exp/winbwd_pair_ab.py 1 2 3 4 > $O/r5_winbwd_pair_ab.log 2>&1; rc=$?
grep -v "amdgpu.ids" $O/r5_winbwd_pair_ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests/ -m gpu -k "windowed" -x -q --timeout 120 --timeout-method thread > $O/r5_win_tests_pair.log 2>&1; rc=$?
tail -3 $O/r5_win_tests_pair.log; exit $rc
