#!/bin/bash
# Round-2 measurements: RCCL capture probe, stream-overlap probe, teacher-stream A/B,
# flagship + ImageNet-shape kernel profiles.  Every GPU step time-limited; stop on failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python scripts/rccl_capture_probe.py > gpurun_out/rccl_capture_probe.log 2>&1; echo "rc=$?" >> gpurun_out/rccl_capture_probe.log
tail -2 gpurun_out/rccl_capture_probe.log
timeout -k 10 120 python scripts/graph_overlap_probe.py > gpurun_out/graph_overlap_probe.log 2>&1 || exit 1
cat gpurun_out/graph_overlap_probe.log
timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/ab_stream_on.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-teacher-stream > gpurun_out/ab_stream_off.log 2>&1 || exit 1
grep metric gpurun_out/ab_stream_on.log | cut -c1-200; grep metric gpurun_out/ab_stream_off.log | cut -c1-200
CFG=configs/cifar100/dkd/res32x4_res8x4.yaml TAG=dkd_flagship bash scripts/gpu_prof_cfg.sh || exit 1
CFG=configs/cifar100/dkd/res32x4_res8x4.yaml TAG=dkd_flagship_nostream EXTRA=--no-teacher-stream bash scripts/gpu_prof_cfg.sh || exit 1
CFG=configs/imagenet/r34_r18/reviewkd.yaml BATCH=32 TAG=reviewkd_r34_r18 bash scripts/gpu_prof_cfg.sh || exit 1
CFG=configs/imagenet/r50_mv1/dkd.yaml BATCH=64 TAG=dkd_r50_mv1 bash scripts/gpu_prof_cfg.sh || exit 1
exit 0
