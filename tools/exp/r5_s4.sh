#!/bin/bash
# round 5, session 4: the two-chain backward hand-off after the asm hazard fix
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 200 python -u tools/exp/bwd_diag.py > $O/r5_bwd_diag.log 2>&1 || { cat $O/r5_bwd_diag.log; exit 1; }
cat $O/r5_bwd_diag.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_backward.py -x -v --timeout 150 --timeout-method thread > $O/r5_bwd_tests.log 2>&1 || { grep -E "FAIL|Error|error|^E " $O/r5_bwd_tests.log | tail -30; exit 1; }
grep -E "two-stream|passed|failed" $O/r5_bwd_tests.log | tail -5
timeout -k 10 400 python -u tools/exp/bwd_two_proc.py 100000 > $O/r5_bwd_two_proc.log 2>&1; rc=$?
cat $O/r5_bwd_two_proc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/exp/ab_fwd_libs.py flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_oaux2.so tools/exp/ab/libfa_oaux16.so tools/exp/ab/libfa_oaux17.so > $O/r5_fwd_oaux_ab.log 2>&1; rc=$?
cat $O/r5_fwd_oaux_ab.log; exit $rc
