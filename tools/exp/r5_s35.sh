#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_ROUNDS=8 timeout -k 10 300 python -u tools/ab_bwd_libs.py flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_bwd_maxilp.so --shapes 8192,128,64 4096,64,64 16384,128,64 > $O/r5_bwd_ab_maxilp2.log 2>&1; rc=$?
grep -v "amdgpu.ids\|rel err" $O/r5_bwd_ab_maxilp2.log; exit $rc
