#!/bin/bash
# round-4 GPU session 1b: windowed B=1 forward stamps, strip-backward PMC (XCD-grouped
# deal), p4 vs 8-wave SQ/LDS counters at d=128, then the GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
WPAIR=1 timeout -k 10 120 python -u tools/exp/win_stamp.py > $O/win_stamp_b1.log 2>&1 || echo "stamp failed"
cd /tmp && export TMPDIR=/tmp
pmc() { timeout -s KILL 60 rocprofv3 --pmc $2 -d $O/pmcw/$1 -o run --output-format csv -- python3 $R/tools/exp/win_bwd_run.py 32 5 > $O/pmcw_$1.log 2>&1; }
pmc f FETCH_SIZE && pmc w WRITE_SIZE && pmc s "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES" || exit 2
python3 $R/tools/exp/pmc_summary.py $O/pmcw > $O/pmcw_summary.txt
pf() { FA_N=8192 FA_D=128 timeout -s KILL 60 rocprofv3 --pmc $2 -d $O/pmcp/$1 -o run --output-format csv -- python3 $R/tools/exp/fwd_run.py 5 30 > $O/pmcp_$1.log 2>&1; }
pf a "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" &&
pf b "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES" || exit 3
python3 $R/tools/exp/pmc_summary.py $O/pmcp > $O/pmcp_summary.txt
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_dense_p4.py tests/test_gpu_windowed_paths.py tests/test_gpu_windowed.py tests/test_gpu_dense.py -x -q -s --timeout 120 --timeout-method thread > $O/r4s1_tests.log 2>&1
echo "tests rc=$?"
