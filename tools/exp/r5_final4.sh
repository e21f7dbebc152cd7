#!/bin/bash
# round-5 validation run: backward A/B against round 4 (longer), the two-process and
# one-GPU two-rank rehearsals of the two-chain hand-off, then the validation set (GPU
# suite, smoke, the default bench line, its rocprof kernel stats, PMC passes).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/r5j_pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > $O/r5j_smoke.log 2>&1 || { echo "smoke failed"; exit 2; }
timeout -k 10 300 python -u bench.py > $O/r5j_bench.log 2>&1 || { echo "bench failed"; exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r5j_prof -o run -- python3 $R/bench.py --no-cpu > $O/r5j_prof.log 2>&1 || { echo "rocprof failed"; exit 4; }
cd $R
PMC_CMD="python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-cfg23 --no-cfg4" timeout -k 10 200 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE > $O/r5j_pmc.log 2>&1 || { echo "pmc failed"; exit 5; }
echo final done
