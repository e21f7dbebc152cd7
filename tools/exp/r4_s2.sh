#!/bin/bash
# round-4 GPU session 2: the default bench line with the node-wide CPU legs, then
# per-config rocprof kernel stats (configs[1]+[3] without cfg4; cfg4 without cfg2/3),
# so the d=128 forward kernel's average belongs to one config in each CSV.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 420 python -u bench.py --cpu-node > $O/bench_r4_cpunode.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg13 -o run -- python3 $R/bench.py --no-cfg4 --no-cpu > $O/prof_cfg13.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg4 -o run -- python3 $R/bench.py --no-cfg23 --no-cpu > $O/prof_cfg4.log 2>&1 || exit 2
echo s2 done
