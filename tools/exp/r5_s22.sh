#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_ROUNDS=10 timeout -k 10 300 python -u tools/ab_bwd_libs.py tools/exp/ab/libfa_prev.so flashattention.jl_amd/libfa_hip.so --shapes 8192,128,64 4096,64,64 > $O/r5_bwd_ab_prepass.log 2>&1; rc=$?
grep -v "amdgpu.ids" $O/r5_bwd_ab_prepass.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r5_prepass_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_bwd_libs.py $GRAFT_REPO_ROOT/flashattention.jl_amd/libfa_hip.so --shapes 8192,128,64 > $O/r5_prepass_prof.log 2>&1 || exit 4
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/r5_bwd_tests_prepass.log 2>&1; rc=$?
tail -3 $O/r5_bwd_tests_prepass.log; exit $rc
