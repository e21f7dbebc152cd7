#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
AB_B="1,4,32" timeout -k 10 300 python -u tools/ab_lib_win.py flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_win_trk.so flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_win_trk.so > $O/r5_win_trackers_fwd_ab.log 2>&1; rc=$?
grep -v "amdgpu.ids" $O/r5_win_trackers_fwd_ab.log | grep " us"; [ $rc -ne 0 ] && exit $rc
AB_B="1,4,32" timeout -k 10 300 python -u tools/ab_lib_winbwd.py flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_win_trk.so flashattention.jl_amd/libfa_hip.so tools/exp/ab/libfa_win_trk.so > $O/r5_win_trackers_bwd_ab.log 2>&1; rc=$?
grep -v "amdgpu.ids" $O/r5_win_trackers_bwd_ab.log | grep " us"; exit $rc
