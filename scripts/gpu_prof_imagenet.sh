#!/bin/bash
# Kernel profiles of the ImageNet-shape BASELINE configs (#4, #5) + flagship.
set -o pipefail
mkdir -p gpurun_out
CFG=configs/imagenet/r34_r18/reviewkd.yaml BATCH=32 TAG=reviewkd_r34_r18 TOP=45 bash scripts/gpu_prof_cfg.sh > /dev/null 2>&1 || exit 1
CFG=configs/imagenet/r50_mv1/dkd.yaml BATCH=64 TAG=dkd_r50_mv1 TOP=45 bash scripts/gpu_prof_cfg.sh > /dev/null 2>&1 || exit 1
CFG=configs/cifar100/dkd/res32x4_res8x4.yaml TAG=dkd_flagship TOP=45 bash scripts/gpu_prof_cfg.sh > /dev/null 2>&1 || exit 1
head -2 gpurun_out/prof_*_summary.md
