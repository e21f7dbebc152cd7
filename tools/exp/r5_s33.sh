#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 600 python -u tools/runcompare.py --dtype both > $O/r5_runcompare.log 2>&1; rc=$?
tail -40 $O/r5_runcompare.log; exit $rc
