#!/bin/bash
# round 5, session 5: backward A/B (round-4 library vs the two-chain hand-off), and the
# one-GPU two-rank bench rehearsal on the single pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_ROUNDS=8 timeout -k 10 400 python -u tools/ab_bwd_libs.py tools/exp/ab/libfa_r4.so flashattention.jl_amd/libfa_hip.so --shapes 8192,128,64 4096,64,64 16384,128,64 > $O/r5_bwd_ab_r4.log 2>&1 || { cat $O/r5_bwd_ab_r4.log; exit 1; }
cat $O/r5_bwd_ab_r4.log
FA_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --no-cpu > $O/r5_bench_2rank_gloo_one_gpu.log 2>&1; rc=$?
tail -c 3000 $O/r5_bench_2rank_gloo_one_gpu.log; exit $rc
