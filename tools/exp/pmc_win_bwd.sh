set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1 || echo "list failed"
R=$GRAFT_REPO_ROOT
run() { timeout -s KILL 60 rocprofv3 --pmc $2 -d $R/gpurun_out/pmcb/$1 -o run --output-format csv -- python3 $R/tools/exp/win_bwd_run.py 32 5 > $R/gpurun_out/pmcb_$1.log 2>&1 || echo "pass $1 failed"; }
run p1 "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
run p2 "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM"
run p3 "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE"
run p4 "FETCH_SIZE"
run p5 "WRITE_SIZE"
echo done
