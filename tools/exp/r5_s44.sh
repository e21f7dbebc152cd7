#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense_pers.py tests/test_gpu_dense.py -x -q --timeout 120 --timeout-method thread > $O/r5_final_pers_tests.log 2>&1 || { tail -5 $O/r5_final_pers_tests.log; exit 1; }
tail -2 $O/r5_final_pers_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" 2>&1 | tail -1
