set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_WR" "TCC_HIT_sum TCC_EA0_WRREQ_sum" "TCC_EA0_RDREQ_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --output-format csv --pmc $grp -d gpurun_out/pmc1_g$i -o run -- python scripts/conv_microbench.py --set imagenet --iters 10 --shape 1 --ops fwd > gpurun_out/pmc1_g$i.log 2>&1 || { tail -5 gpurun_out/pmc1_g$i.log; exit 1; }
  MDA_CONV_GLDS=0 timeout -s KILL 90 rocprofv3 --output-format csv --pmc $grp -d gpurun_out/pmc1_r$i -o run -- python scripts/conv_microbench.py --set imagenet --iters 10 --shape 1 --ops fwd > gpurun_out/pmc1_r$i.log 2>&1 || { tail -5 gpurun_out/pmc1_r$i.log; exit 1; }
done
python scripts/pmc_summary.py gpurun_out "pmc1_g*" conv_glds
python scripts/pmc_summary.py gpurun_out "pmc1_r*" conv_fwd
