#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r5_fwd_pers_prof -o run -- python3 $R/tools/exp/fwd_pers_prof.py > $O/r5_fwd_pers_prof.log 2>&1; rc=$?
tail -3 $O/r5_fwd_pers_prof.log; exit $rc
