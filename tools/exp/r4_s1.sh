#!/bin/bash
# round-4 GPU session: p4 ablations, windowed strip-backward timing + PMC (XCD-grouped deal),
# then the backward / p4 / windowed / dense GPU tests.  Every GPU step has its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 150 python -u tools/exp/p4_abl.py 4096,64,64 a0 a1 a2 a4 a8 a15 pf2 pf6 > $O/p4_abl1.log 2>&1 &&
timeout -k 10 150 python -u tools/exp/p4_abl.py 8192,128,64 a0 a1 a2 a4 a8 a15 pf2 pf6 >> $O/p4_abl1.log 2>&1 &&
timeout -k 10 120 python -u tools/exp/win_bwd_time.py 1 32 > $O/win_bwd_time.log 2>&1 &&
timeout -k 10 150 python -u tools/exp/bwd_l2local_ab.py > $O/bwd_l2local.log 2>&1 &&
WPAIR=1 timeout -k 10 120 python -u tools/exp/win_stamp.py > $O/win_stamp_b1.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
pmc() { timeout -s KILL 60 rocprofv3 --pmc $2 -d $O/pmcw/$1 -o run --output-format csv -- python3 $R/tools/exp/win_bwd_run.py 32 5 > $O/pmcw_$1.log 2>&1; }
pmc f FETCH_SIZE && pmc w WRITE_SIZE && pmc s "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES" || exit 2
python3 $R/tools/exp/pmc_summary.py $O/pmcw > $O/pmcw_summary.txt
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_dense_p4.py tests/test_gpu_windowed_paths.py tests/test_gpu_windowed.py tests/test_gpu_dense.py -x -q -s --timeout 120 --timeout-method thread > $O/r4s1_tests.log 2>&1
echo "tests rc=$?"
