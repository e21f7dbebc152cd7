#!/bin/bash
# r6 session 2: Q/dO DMA cache policy x L2-local hand-off x chain offset, configs[3] backward
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6s2; mkdir -p $O
A=tools/exp/abr6
for cfg in "0 3" "1 3" "1 2" "0 2"; do
  set -- $cfg
  echo "== l2local=$1 hoff=$2" | tee -a $O/ab.log
  AB_L2LOCAL=$1 AB_HOFF=$2 AB_ROUNDS=5 timeout -k 10 200 python3 tools/ab_bwd_libs.py $A/libfa_base.so $A/libfa_nt.so $A/libfa_sc1.so --shapes 8192,128,64 >> $O/ab.log 2>&1 || exit 1
done
for v in "nt1:FA_HIP_LIB=$A/libfa_nt.so FA_L2LOCAL=1" "nt0:FA_HIP_LIB=$A/libfa_nt.so FA_L2LOCAL=0"; do
  n=${v%%:*}; e=${v#*:}
  timeout -k 10 120 env $e rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${n}_fetch -o run -- python3 tools/exp/bwd_run.py 0 3 > $O/${n}_fetch.log 2>&1 || exit 1
  timeout -k 10 120 env $e rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/${n}_hit -o run -- python3 tools/exp/bwd_run.py 0 3 > $O/${n}_hit.log 2>&1 || exit 1
done
echo done
