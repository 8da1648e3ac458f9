set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
for p8 in 1 0; do
  grp="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES"
  MDA_HALO_PERM8=$p8 timeout -s KILL 90 rocprofv3 --output-format csv --pmc $grp -d gpurun_out/pmc8_p$p8 -o run -- python scripts/conv_microbench.py --iters 10 --shape 6 --ops fwd > gpurun_out/pmc8_p$p8.log 2>&1 || { tail -5 gpurun_out/pmc8_p$p8.log; exit 1; }
  python scripts/pmc_summary.py gpurun_out "pmc8_p$p8" conv_halo > gpurun_out/pmc8_p$p8.txt
  echo "== MDA_HALO_PERM8=$p8"; cat gpurun_out/pmc8_p$p8.txt
done
