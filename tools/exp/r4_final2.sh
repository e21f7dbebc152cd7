#!/bin/bash
# round-4 closing run: the two-process slab-placement A/B, then the validation set
# (GPU suite, smoke, the default bench line, its rocprof kernel stats, the configs[1]
# forward's HBM traffic from separate PMC passes).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 420 python -u tools/exp/bwd_two_proc_xcd.py > $O/bwd_two_proc_xcd.log 2>&1 || { echo "xcd a/b failed"; exit 9; }
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/final_pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > $O/final_smoke.log 2>&1 || { echo "smoke failed"; exit 2; }
timeout -k 10 300 python -u bench.py > $O/final_bench.log 2>&1 || { echo "bench failed"; exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/final_prof -o run -- python3 $R/bench.py --no-cpu > $O/final_prof.log 2>&1 || { echo "rocprof failed"; exit 4; }
cd $R
PMC_CMD="python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-cfg23 --no-cfg4" timeout -k 10 200 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE > $O/final_pmc.log 2>&1 || { echo "pmc failed"; exit 5; }
echo final done
