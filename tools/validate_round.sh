set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fwd -o fwd -- python3 bench.py --no-cpu > gpurun_out/prof_fwd.log 2>&1 || exit 4
PMC_CMD="python3 bench.py --steps 5 --warmup 2 --no-cpu --no-cfg4 --no-cfg23 --settle-ms 50" timeout -k 10 400 bash tools/pmc.sh FETCH_SIZE WRITE_SIZE > gpurun_out/pmc.log 2>&1 || exit 5
echo ALLOK
