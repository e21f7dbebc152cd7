#!/bin/bash
# round 3: max-ILP machine scheduler on fa_bwd.hip / fa_windowed.hip (A/B vs the shipped build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_bwd_libs.py flashattention.jl_amd/libfa_hip.so tools/exp/abl/libfa_bwdilp.so --shapes 8192,128,64 4096,64,64 8192,128,64 > gpurun_out/flags_bwd_ab.log 2>&1 || exit 1
AB_B="1,32,128" timeout -k 10 300 python -u tools/ab_lib_winbwd.py flashattention.jl_amd/libfa_hip.so tools/exp/abl/libfa_winilp.so > gpurun_out/flags_winbwd_ab.log 2>&1 || exit 1
AB_B="1,32,128" timeout -k 10 300 python -u tools/ab_lib_win.py flashattention.jl_amd/libfa_hip.so tools/exp/abl/libfa_winilp.so > gpurun_out/flags_winfwd_ab.log 2>&1 || exit 1
