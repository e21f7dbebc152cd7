#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 200 python -u tools/exp/bwd_flags_diag.py > $O/r5_bwd_flags.log 2>&1; cat $O/r5_bwd_flags.log
AB_ROUNDS=8 timeout -k 10 500 python -u tools/ab_bwd_libs.py tools/exp/ab/libfa_r4.so flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_bwd_maxilp.so tools/exp/ab/libfa_bwd_maxmem.so --shapes 8192,128,64 4096,64,64 > $O/r5_bwd_ab_sched.log 2>&1; rc=$?
cat $O/r5_bwd_ab_sched.log; exit $rc
