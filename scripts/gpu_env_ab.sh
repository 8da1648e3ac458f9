#!/bin/bash
# Generic env-var A/B on step throughput: VARS="A=1 B=2" ("base" = no override), CONFIGS=...
set -o pipefail
mkdir -p gpurun_out
for v in ${VARS:-base}; do
  if [ "$v" = base ]; then e=X_BASE=1; else e=$v; fi
  env $e timeout -k 10 400 python benchmarks/throughput.py --configs $CONFIGS --steps ${STEPS:-30} --warmup 10 > gpurun_out/envab_$v.log 2>&1 || { tail -5 gpurun_out/envab_$v.log; exit 1; }
  echo "== $v"; grep '^{' gpurun_out/envab_$v.log | sed 's/"images_per_s".*"ms_per_step"/ms/' | cut -c1-80
done
