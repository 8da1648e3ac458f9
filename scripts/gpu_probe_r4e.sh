set -o pipefail
mkdir -p gpurun_out; export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python scripts/conv_microbench.py --set imagenet --graph --iters 30 --json gpurun_out/cmb_imagenet.json > gpurun_out/cmb_imagenet.log 2>&1 || { tail -5 gpurun_out/cmb_imagenet.log; exit 1; }
timeout -k 10 400 python scripts/conv_microbench.py --set mv1 --graph --iters 30 --json gpurun_out/cmb_mv1.json > gpurun_out/cmb_mv1.log 2>&1 || { tail -5 gpurun_out/cmb_mv1.log; exit 1; }
echo done
