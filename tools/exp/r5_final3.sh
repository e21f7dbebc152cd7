#!/bin/bash
# round-5 validation run: backward A/B against round 4 (longer), the two-process and
# one-GPU two-rank rehearsals of the two-chain hand-off, then the validation set (GPU
# suite, smoke, the default bench line, its rocprof kernel stats, PMC passes).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/exp/bwd_two_proc.py 100000 > $O/r5i_bwd_two_proc.log 2>&1 || { echo "two-proc failed"; exit 9; }
FA_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --no-cpu > $O/r5i_bench_2rank_gloo_one_gpu.log 2>&1 || { echo "2rank failed"; exit 10; }
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/r5i_pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > $O/r5i_smoke.log 2>&1 || { echo "smoke failed"; exit 2; }
timeout -k 10 300 python -u bench.py > $O/r5i_bench.log 2>&1 || { echo "bench failed"; exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r5i_prof -o run -- python3 $R/bench.py --no-cpu > $O/r5i_prof.log 2>&1 || { echo "rocprof failed"; exit 4; }
cd $R
PMC_CMD="python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-cfg23 --no-cfg4" timeout -k 10 200 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE > $O/r5i_pmc.log 2>&1 || { echo "pmc failed"; exit 5; }
echo final done
