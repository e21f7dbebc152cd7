#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/r5h_pytest_gpu.log 2>&1 || { tail -5 $O/r5h_pytest_gpu.log; exit 1; }
tail -2 $O/r5h_pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > $O/r5h_smoke.log 2>&1 || { tail -5 $O/r5h_smoke.log; exit 2; }
tail -1 $O/r5h_smoke.log
