#!/bin/bash
# round 5, session 2: forward launch timeline; the two-chain backward hand-off (suite, two processes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 120 python -u tools/exp/fwd_timeline.py run > $O/r5_fwd_timeline.log 2>&1 || { cat $O/r5_fwd_timeline.log; exit 1; }
cat $O/r5_fwd_timeline.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_backward.py -x -v --timeout 150 --timeout-method thread > $O/r5_bwd_tests.log 2>&1 || { grep -E "FAIL|Error|error|^E " $O/r5_bwd_tests.log | tail -30; exit 1; }
grep -E "two-stream|passed|failed" $O/r5_bwd_tests.log | tail -5
timeout -k 10 400 python -u tools/exp/bwd_two_proc.py 100000 > $O/r5_bwd_two_proc.log 2>&1; rc=$?
cat $O/r5_bwd_two_proc.log; exit $rc
