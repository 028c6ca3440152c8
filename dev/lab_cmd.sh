# dev/lab_cmd.sh -- one gpurun call: scatter_lab timings (+ phase stamps) and two PMC passes.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./dev/scatter_lab 30 "k8 512x32 count" > gpurun_out/lab10.log 2>&1
timeout -k 10 120 ./dev/scatter_lab_stamps 30 "k8 512x32 count" >> gpurun_out/lab10.log 2>&1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY -d $R/gpurun_out/pmc10a -o run -- $R/dev/scatter_lab 30 "k8 512x32 count" > $R/gpurun_out/pmc10a.log 2>&1
timeout -k 10 180 rocprofv3 --pmc TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU -d $R/gpurun_out/pmc10b -o run -- $R/dev/scatter_lab 30 "k8 512x32 count" > $R/gpurun_out/pmc10b.log 2>&1
timeout -k 10 180 rocprofv3 --pmc TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum -d $R/gpurun_out/pmc10c -o run -- $R/dev/wc_lab 30 > $R/gpurun_out/pmc10c.log 2>&1
