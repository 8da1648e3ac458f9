#!/bin/bash
# A/B of the conv block-count target (split-K trigger) on step throughput.
set -o pipefail
mkdir -p gpurun_out
for t in 512 256 128; do
  MDA_CONV_TARGET=$t timeout -k 10 400 python benchmarks/throughput.py --configs ${CONFIGS:-dkd_cifar_res32x4_res8x4,reviewkd_imagenet_r34_r18} --steps 30 --warmup 10 > gpurun_out/tgt_$t.log 2>&1 || { tail -5 gpurun_out/tgt_$t.log; exit 1; }
  echo "== target $t"; grep '^{' gpurun_out/tgt_$t.log | cut -c1-110
done
