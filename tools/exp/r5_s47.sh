#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_B="1,32" timeout -k 10 300 python -u tools/ab_lib_winbwd.py flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_winbwd_ilp.so flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_winbwd_ilp.so > $O/r5_winbwd_ilp_ab.log 2>&1; rc=$?
grep -v amdgpu.ids $O/r5_winbwd_ilp_ab.log; exit $rc
