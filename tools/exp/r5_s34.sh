#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_B="1,2,4" timeout -k 10 300 python -u tools/ab_lib_win.py tools/exp/ab/libfa_win_prev.so flashattention.jl_amd/libfa_hip.so > $O/r5_winfwd_pairstore_ab.log 2>&1; rc=$?
grep -v "amdgpu.ids" $O/r5_winfwd_pairstore_ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests/ -m gpu -k "windowed" -x -q --timeout 120 --timeout-method thread > $O/r5_win_tests_pairstore.log 2>&1; rc=$?
tail -3 $O/r5_win_tests_pairstore.log; exit $rc
