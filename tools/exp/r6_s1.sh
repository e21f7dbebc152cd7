#!/bin/bash
# r6 session 1: bwd_fused traffic at configs[3] (default and L2-local hand-off), power probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6s1; mkdir -p $O
pass() {  # name env counters...
  local name=$1; shift; local envs=$1; shift
  echo "== $name: $*" 
  timeout -k 10 120 env $envs rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- python3 tools/exp/bwd_run.py 0 3 > $O/$name.log 2>&1
}
for v in "def:FA_L2LOCAL=0" "l2l:FA_L2LOCAL=1"; do
  n=${v%%:*}; e=${v#*:}
  pass ${n}_fetch "$e" FETCH_SIZE || exit 1
  pass ${n}_write "$e" WRITE_SIZE || exit 1
  pass ${n}_hit "$e" TCC_HIT_sum TCC_MISS_sum || exit 1
  pass ${n}_dram "$e" TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum || exit 1
  pass ${n}_ea "$e" TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum || exit 1
  timeout -k 10 120 env $e rocprofv3 --kernel-trace --stats --output-format csv -d $O/${n}_trace -o run -- python3 tools/exp/bwd_run.py 0 5 > $O/${n}_trace.log 2>&1 || exit 1
done
timeout -k 10 200 python3 tools/power_probe.py 8 fwd gemm bwd > $O/power.log 2>&1 || exit 1
echo done
