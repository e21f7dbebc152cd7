#!/bin/bash
# r6 closing validation: GPU suite, smoke, default bench, per-config rocprof CSVs, forward PMC traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo tests failed; tail -30 $O/pytest_gpu.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || exit 3
for c in "cfg1:--no-cfg23 --no-cfg4" "cfg3:--no-cfg2 --no-cfg4" "cfg2:--no-cfg3 --no-cfg4" "cfg4:--no-cfg23"; do
  n=${c%%:*}; a=${c#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 bench.py --no-cpu $a > $O/prof_$n.log 2>&1 || exit 4
done
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$grp -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-cfg4 --no-cfg23 --settle-ms 50 > $O/pmc_$grp.log 2>&1 || exit 5
done
echo ALLOK
