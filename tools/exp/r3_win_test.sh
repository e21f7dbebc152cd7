#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_windowed_paths.py -x -q -k "dynamic_deal or strip_full_size" --timeout 200 --timeout-method thread > gpurun_out/pytest_dyn.log 2>&1 || exit 1
