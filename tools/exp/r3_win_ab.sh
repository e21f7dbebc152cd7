#!/bin/bash
# round 3: windowed backward A/B (committed build vs working tree) + windowed GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AB_B="1,2,4,8,32" timeout -k 10 300 python -u tools/ab_lib_winbwd.py tools/exp/abl/libfa_head5.so flashattention.jl_amd/libfa_hip.so > gpurun_out/winbwd_ab.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_windowed.py tests/test_gpu_windowed_paths.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_win.log 2>&1 || exit 1
