set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcf/p1 -o run --output-format csv -- python3 $R/tools/exp/win_run.py 32 > $R/gpurun_out/pmcf_p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum -d $R/gpurun_out/pmcf/p2 -o run --output-format csv -- python3 $R/tools/exp/win_run.py 32 > $R/gpurun_out/pmcf_p2.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES -d $R/gpurun_out/pmcf/p3 -o run --output-format csv -- python3 $R/tools/exp/win_run.py 32 > $R/gpurun_out/pmcf_p3.log 2>&1
echo done
