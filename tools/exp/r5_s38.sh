#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_DENSE_ONLY=1 AB_ROUNDS=16 timeout -k 10 300 python -u tools/ab_lib.py tools/exp/ab/libfa_fwd_trk.so tools/exp/ab/libfa_fwd_base.so tools/exp/ab/libfa_fwd_trk.so tools/exp/ab/libfa_fwd_base.so > $O/r5_fwd_trackers_ab2.log 2>&1; rc=$?
grep -v "amdgpu.ids" $O/r5_fwd_trackers_ab2.log; exit $rc
