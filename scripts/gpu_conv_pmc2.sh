#!/bin/bash
# Per-kernel times (kernel trace) of every conv shape + PMC counters of one shape's fwd.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/cmb -o run -- python scripts/conv_microbench.py --iters 20 --ops fwd,dgrad,wgrad > gpurun_out/cmb.log 2>&1 || { tail -5 gpurun_out/cmb.log; exit 1; }
find gpurun_out/cmb -name "*kernel_stats.csv" -exec cp {} gpurun_out/cmb_kernel_stats.csv \;
SH=${SH:-4}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --output-format csv --pmc $grp -d gpurun_out/pmc2_$i -o run -- python scripts/conv_microbench.py --iters 10 --shape $SH --ops fwd > gpurun_out/pmc2_$i.log 2>&1 || { tail -5 gpurun_out/pmc2_$i.log; exit 1; }
done
python scripts/pmc_summary.py gpurun_out "pmc2_*" conv_halo
