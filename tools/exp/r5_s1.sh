#!/bin/bash
# round 5, session 1: persistent d<=64 forward (parity + A/B) and the two-chain backward hand-off
# (backward suite, two-process run)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense_pers.py -x -v --timeout 120 --timeout-method thread > $O/r5_pers_tests.log 2>&1 || { tail -40 $O/r5_pers_tests.log; exit 1; }
tail -2 $O/r5_pers_tests.log
timeout -k 10 240 python -u tools/ab_fwd.py --shapes 4096,64,64 4096,64,128 0 40 > $O/r5_pers_ab.log 2>&1 || { cat $O/r5_pers_ab.log; exit 1; }
cat $O/r5_pers_ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py -x -v --timeout 150 --timeout-method thread > $O/r5_bwd_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/r5_bwd_tests.log | tail -30; exit 1; }
grep -E "two-stream|passed|failed" $O/r5_bwd_tests.log | tail -5
timeout -k 10 400 python -u tools/exp/bwd_two_proc.py 100000 > $O/r5_bwd_two_proc.log 2>&1; rc=$?
cat $O/r5_bwd_two_proc.log; exit $rc
