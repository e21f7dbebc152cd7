#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_ROUNDS=6 timeout -k 10 300 python -u tools/ab_bwd_libs.py tools/exp/ab/libfa_r4.so tools/exp/ab/libfa_walk.so flashattention.jl_amd/libfa_hip.so --shapes 8192,128,64 4096,64,64 > $O/r5_bwd_ab_earlypoll.log 2>&1; rc=$?
grep -v "rel err" $O/r5_bwd_ab_earlypoll.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/r5_bwd_tests_earlypoll.log 2>&1; rc=$?
tail -3 $O/r5_bwd_tests_earlypoll.log; exit $rc
