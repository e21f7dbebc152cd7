set -e
# SQ / LDS counter passes for the configs[3] backward (single pass, mode 0; split passes, mode 1).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() { timeout -s KILL 90 rocprofv3 --pmc $2 -d $R/gpurun_out/pmcb/$1 -o run --output-format csv -- python3 $R/tools/exp/bwd_run.py $3 3 > $R/gpurun_out/pmcb_$1.log 2>&1; }
for m in ${MODES:-0 1}; do
run m${m}p1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" $m
run m${m}p2 "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE" $m
run m${m}p3 "SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM SQ_WAVES" $m
done
echo done
