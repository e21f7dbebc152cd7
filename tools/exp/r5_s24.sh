#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/r5_bwd_tests_combine.log 2>&1; rc=$?
tail -5 $O/r5_bwd_tests_combine.log; [ $rc -ne 0 ] && exit $rc
AB_ROUNDS=8 timeout -k 10 300 python -u tools/ab_bwd_libs.py tools/exp/ab/libfa_prev.so flashattention.jl_amd/libfa_hip.so --shapes 8192,128,64 4096,64,64 > $O/r5_bwd_ab_combineknob.log 2>&1; rc=$?
grep -v "amdgpu.ids\|rel err" $O/r5_bwd_ab_combineknob.log; exit $rc
