# dev/pmc_cmp.sh -- memory-pipe counters for rs_scatter_lines vs the synthetic line-store scatter.
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCC_BUSY_avr TCC_EA0_WRREQ_STALL_sum -d $R/gpurun_out/pmc30a -o run -- $R/dev/scatter_lab 30 "k8 1024x16 lines16" > $R/gpurun_out/pmc30a.log 2>&1
timeout -k 10 200 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCC_BUSY_avr TCC_EA0_WRREQ_STALL_sum -d $R/gpurun_out/pmc30b -o run -- $R/dev/wc_lab 30 > $R/gpurun_out/pmc30b.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY -d $R/gpurun_out/pmc30c -o run -- $R/dev/scatter_lab 30 "k8 1024x16 lines16" > $R/gpurun_out/pmc30c.log 2>&1
