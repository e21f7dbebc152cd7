#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -k "dense or forward or golden or pers or p4" -x -q --timeout 120 --timeout-method thread > $O/r5_fwd_tests_trk.log 2>&1; rc=$?
tail -2 $O/r5_fwd_tests_trk.log; [ $rc -ne 0 ] && exit $rc
AB_DENSE_ONLY=1 AB_ROUNDS=10 timeout -k 10 300 python -u tools/ab_lib.py tools/exp/ab/libfa_fwd_base.so flashattention.jl_amd/libfa_hip.so > $O/r5_fwd_trackers_ab3.log 2>&1; rc=$?
grep "N=4096" $O/r5_fwd_trackers_ab3.log; exit $rc
