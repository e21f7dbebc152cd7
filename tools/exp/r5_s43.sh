#!/bin/bash
# round 5: persistent d<=64 forward — parity tests, then a same-process A/B vs the 8-wave kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense_pers.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5_pers_tests_trk.log 2>&1 || { tail -30 gpurun_out/r5_pers_tests.log; exit 1; }
tail -3 gpurun_out/r5_pers_tests_trk.log
timeout -k 10 240 python -u tools/ab_fwd.py --shapes 4096,64,64 4096,64,128 0 40 > gpurun_out/r5_pers_ab_trk.log 2>&1
rc=$?; cat gpurun_out/r5_pers_ab_trk.log; exit $rc
