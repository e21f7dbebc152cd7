#!/bin/bash
# round-3 session 2: backward ablations (no next-slice DMA) + 2-rank gloo rehearsal of bench.py --gpus 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
FA_HIP_LIB=$PWD/tools/exp/abl/libfa_abl.so timeout -k 10 300 python -u tools/ab_bwd.py --shapes 8192,128,64 2 6 10 11 1 > gpurun_out/bwd_abl.log 2>&1 || exit 1
FA_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_2rank_gloo.log 2>&1 || exit 1
