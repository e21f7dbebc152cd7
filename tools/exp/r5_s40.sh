#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_DENSE_ONLY=1 AB_ROUNDS=10 timeout -k 10 300 python -u tools/ab_lib.py flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_p4_trk.so > $O/r5_p4_trackers_ab.log 2>&1; rc=$?
grep -v "amdgpu.ids" $O/r5_p4_trackers_ab.log; [ $rc -ne 0 ] && exit $rc
AB_ROUNDS=8 timeout -k 10 300 python -u tools/ab_bwd_libs.py flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_bwd_trk.so --shapes 8192,128,64 4096,64,64 > $O/r5_bwd_trackers_ab.log 2>&1; rc=$?
grep -v "amdgpu.ids\|rel err" $O/r5_bwd_trackers_ab.log; exit $rc
