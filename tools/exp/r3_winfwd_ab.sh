#!/bin/bash
# round 3: windowed strip forward epilogue wait (builtin instead of asm) A/B + windowed GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AB_B="1,8,32,128" timeout -k 10 300 python -u tools/ab_lib_win.py tools/exp/abl/libfa_head5.so flashattention.jl_amd/libfa_hip.so > gpurun_out/winfwd_ab.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_windowed.py tests/test_gpu_windowed_paths.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_win.log 2>&1 || exit 1
