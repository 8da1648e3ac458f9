#!/bin/bash
# Kernel-level wgrad timings (rocprofv3 kernel trace) for a few shapes: SHAPES="set:idx ..."
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for sh in ${SHAPES:-imagenet:3 imagenet:12 cifar:2}; do
  set=${sh%%:*}; idx=${sh##*:}
  for cfg in "old MDA_WG_GLDS=0" "new X=1"; do
    set -- $cfg
    tag=wgp_${set}_${idx}_$1
    env $2 timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/$tag -o run -- python scripts/conv_microbench.py --set $set --shape $idx --iters 20 --ops wgrad > gpurun_out/$tag.log 2>&1 || { tail -5 gpurun_out/$tag.log; exit 1; }
    echo "== $set $idx $1: $(grep '^{' gpurun_out/$tag.log | cut -c1-60)"
    python scripts/kstats.py "gpurun_out/$tag/*.db" --filter "wgrad" --top 4
    rm -rf gpurun_out/$tag
  done
done
