#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -k "windowed or window or dpa or block" -x -q --timeout 120 --timeout-method thread > $O/r5_win_tests_split.log 2>&1; rc=$?
tail -2 $O/r5_win_tests_split.log; [ $rc -ne 0 ] && exit $rc
AB_B="1,32" timeout -k 10 300 python -u tools/ab_lib_win.py tools/exp/ab/libfa_win_prev.so flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_win_prev.so flashattention.jl_amd/libfa_hip.so > $O/r5_win_split_fwd_ab.log 2>&1; rc=$?
grep " us" $O/r5_win_split_fwd_ab.log; [ $rc -ne 0 ] && exit $rc
AB_B="1,32" timeout -k 10 300 python -u tools/ab_lib_winbwd.py tools/exp/ab/libfa_win_prev.so flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_win_prev.so flashattention.jl_amd/libfa_hip.so > $O/r5_win_split_bwd_ab.log 2>&1; rc=$?
grep " us" $O/r5_win_split_bwd_ab.log; exit $rc
