#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench -> rocprof kernel trace.
# Every GPU step has its own time limit; steps chained with && (stop at first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${1:-all}"
run_tests() { timeout -k 10 ${T_TESTS:-900} python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; }
run_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; }
run_bench() { timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench.log 2>&1; }
run_prof()  { timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o fwd -- python3 bench.py --no-cpu ${PROF_ARGS:-} > gpurun_out/prof.log 2>&1; }
case "$STEPS" in
  all)   run_tests && run_smoke && run_bench && run_prof ;;
  tests) run_tests ;;
  bench) run_bench ;;
  prof)  run_prof ;;
  smoke) run_smoke ;;
  *)     eval "$STEPS" ;;
esac
rc=$?
echo "exit $rc"
for f in gpurun_out/*.log; do echo "== $f"; tail -n 5 "$f"; done
exit $rc
