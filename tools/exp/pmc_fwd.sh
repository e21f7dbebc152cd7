#!/bin/bash
# SQ counter passes over tools/exp/fwd_run.py (one counter group per rocprofv3 run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcf; mkdir -p $OUT
VARS="${VARS:-7 8}"
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 ${PMC_SCRIPT:-tools/exp/fwd_run.py} $VARS > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo done
