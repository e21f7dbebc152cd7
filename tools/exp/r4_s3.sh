#!/bin/bash
# round-4 session 3: strip-backward phase stamps (XCD-group deal) and LDS bank conflicts
# with / without the gradient image writes (WABL 64, timing-only).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/exp/bwd_strip_stamp.py > $O/bwd_strip_stamp.log 2>&1 &&
WABL=64 timeout -k 10 120 python -u tools/exp/bwd_strip_stamp.py >> $O/bwd_strip_stamp.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $O/pmcs/a0 -o run --output-format csv -- python3 $R/tools/exp/bwd_strip_stamp.py > $O/pmcs_a0.log 2>&1 &&
WABL=64 timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $O/pmcs/a64 -o run --output-format csv -- python3 $R/tools/exp/bwd_strip_stamp.py > $O/pmcs_a64.log 2>&1 || exit 2
python3 $R/tools/exp/pmc_summary.py $O/pmcs/a0 > $O/pmcs_summary.txt; python3 $R/tools/exp/pmc_summary.py $O/pmcs/a64 >> $O/pmcs_summary.txt
echo s3 done
