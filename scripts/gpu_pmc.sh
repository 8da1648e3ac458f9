# PMC counters for one conv shape (fwd only), halo vs glds kernels.
set -x
[ -f mdistiller_ddp_amd/ops/_lib/libmda_hip.so ] || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SH=${SH:-2}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --output-format csv --pmc $grp -d gpurun_out/pmc_h$i -o run -- python scripts/conv_microbench.py --iters 10 --shape $SH --ops fwd > gpurun_out/pmc_h$i.log 2>&1 || { tail -5 gpurun_out/pmc_h$i.log; exit 1; }
  MDA_CONV_HALO=0 timeout -k 10 120 rocprofv3 --output-format csv --pmc $grp -d gpurun_out/pmc_g$i -o run -- python scripts/conv_microbench.py --iters 10 --shape $SH --ops fwd > gpurun_out/pmc_g$i.log 2>&1 || { tail -5 gpurun_out/pmc_g$i.log; exit 1; }
done
python scripts/pmc_summary.py gpurun_out "pmc_h*" conv_halo
python scripts/pmc_summary.py gpurun_out "pmc_g*" conv_glds
