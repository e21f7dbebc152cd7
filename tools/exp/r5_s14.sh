#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
: > $O/r5_bwd_abl_r4_vs_cur.log
for m in 2 4 5 6; do
  echo "== mode $m" >> $O/r5_bwd_abl_r4_vs_cur.log
  AB_MODE=$m AB_ROUNDS=5 timeout -k 10 200 python -u tools/ab_bwd_libs.py tools/exp/ab/libfa_r4_abl.so tools/exp/ab/libfa_cur_abl.so --shapes 8192,128,64 4096,64,64 >> $O/r5_bwd_abl_r4_vs_cur.log 2>&1 || exit $?
done
grep -v "rel err" $O/r5_bwd_abl_r4_vs_cur.log
