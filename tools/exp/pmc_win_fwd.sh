set -e
# PMC passes for the configs[2] windowed forward at B images (default 32); one counter group per run.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B=${B:-32}
T=${TAG:-}
run() { timeout -s KILL 60 rocprofv3 --pmc $2 -d $R/gpurun_out/pmcf$T/$1 -o run --output-format csv -- python3 $R/tools/exp/win_run.py $B > $R/gpurun_out/pmcf${T}_$1.log 2>&1; }
run p1 "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum GRBM_GUI_ACTIVE"
run p2 "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
run p3 "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_WAIT_ANY"
run p4 "TCC_HIT_sum TCC_MISS_sum"
run p5 "FETCH_SIZE"
run p6 "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
run p7 "WRITE_SIZE"
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmcf$T/trace -o run --output-format csv -- python3 $R/tools/exp/win_run.py $B > $R/gpurun_out/pmcf${T}_trace.log 2>&1
echo done
