#!/bin/bash
# Kernel-level A/B of conv variants on the microbench shapes (kernel trace, no PMC).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/cab_$tag -o run -- python scripts/conv_microbench.py --iters 20 --ops fwd,dgrad > gpurun_out/cab_$tag.log 2>&1 || { tail -5 gpurun_out/cab_$tag.log; return 1; }
  echo "== $tag"; python scripts/kstats.py "gpurun_out/cab_$tag/*.db" --filter "conv_" --top 25
  rm -rf gpurun_out/cab_$tag
}
run base || exit 1
run nohalo2 MDA_CONV_HALO2=0 || exit 1
run nohalo MDA_CONV_HALO=0 || exit 1
