#!/bin/bash
# round 3: backward A/B (committed build vs working tree) + backward GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_bwd_libs.py tools/exp/abl/libfa_head5.so flashattention.jl_amd/libfa_hip.so --shapes 8192,128,64 4096,64,64 8192,128,64 > gpurun_out/bwd_ab.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bwd.log 2>&1 || exit 1
