#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_ROUNDS=8 timeout -k 10 400 python -u tools/ab_bwd_libs.py tools/exp/ab/libfa_r4.so flashattention.jl_amd/libfa_hip.so --shapes 8192,128,64 4096,64,64 > $O/r5_bwd_ab_r4b.log 2>&1; rc=$?
cat $O/r5_bwd_ab_r4b.log; exit $rc
