#!/bin/bash
# round-4 GPU session 1c: p4 cross-seam prefetch vs the previous p4 (old) and the 8-wave
# default; strip-backward deal A/B (round-3 chip-wide deal vs XCD groups); p4 tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 150 python -u tools/exp/p4_abl.py 4096,64,64 old a0 a4 pf2 pf6 > $O/p4_abl2.log 2>&1 &&
timeout -k 10 150 python -u tools/exp/p4_abl.py 8192,128,64 old a0 a4 pf2 pf6 >> $O/p4_abl2.log 2>&1 &&
timeout -k 10 200 python -u tools/exp/ab_win_libs.py tools/exp/abl/libfa_r3deal.so flashattention.jl_amd/libfa_hip.so > $O/ab_win_deal.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense_p4.py -x -q --timeout 120 --timeout-method thread > $O/r4s1c_tests.log 2>&1
echo "tests rc=$?"
