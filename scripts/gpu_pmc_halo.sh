set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python scripts/conv_microbench.py --set cifar --graph --iters 30 --json gpurun_out/cmb_cifar.json > gpurun_out/cmb_cifar.log 2>&1 || { tail -5 gpurun_out/cmb_cifar.log; exit 1; }
for sh in 2 4 6; do
  for grp in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES" "SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"; do
    tag=$(echo $grp | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 90 rocprofv3 --output-format csv --pmc $grp -d gpurun_out/pmc_s${sh}_$tag -o run -- python scripts/conv_microbench.py --iters 10 --shape $sh --ops fwd > gpurun_out/pmc_s${sh}_$tag.log 2>&1 || { tail -5 gpurun_out/pmc_s${sh}_$tag.log; exit 1; }
  done
  python scripts/pmc_summary.py gpurun_out "pmc_s${sh}_*" conv_halo > gpurun_out/pmc_s${sh}.txt
  cat gpurun_out/pmc_s${sh}.txt
done
