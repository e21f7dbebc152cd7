#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for L in tools/exp/ab/libfa_prev.so flashattention.jl_amd/libfa_hip.so; do
  n=$(basename $L .so)
  AB_ROUNDS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r5_prepass_prof_$n -o run -- python3 $R/tools/ab_bwd_libs.py $R/$L --shapes 8192,128,64 > $O/r5_prepass_prof_$n.log 2>&1 || exit 4
done
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/r5_bwd_tests_prepass.log 2>&1; rc=$?
tail -3 $O/r5_bwd_tests_prepass.log; exit $rc
