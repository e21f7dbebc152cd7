#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_DENSE_ONLY=1 AB_ROUNDS=12 timeout -k 10 300 python -u tools/ab_lib.py flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_fwd_nounc.so flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_fwd_nounc.so > $O/r5_fwd_nounc_ab.log 2>&1; rc=$?
grep "N=4096" $O/r5_fwd_nounc_ab.log; exit $rc
