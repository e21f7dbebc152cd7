#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_ROUNDS=6 timeout -k 10 300 python -u tools/ab_bwd_libs.py tools/exp/ab/libfa_r4.so flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_onechain.so --shapes 8192,128,64 4096,64,64 > $O/r5_bwd_ab_onechain.log 2>&1; rc=$?
grep -v "rel err" $O/r5_bwd_ab_onechain.log; exit $rc
