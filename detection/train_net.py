#!/usr/bin/env python
"""Detection distillation entry point (reference `detection/train_net.py`).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        detection/train_net.py --config-file detection/configs/DKD/DKD-R18-R101.yaml \
        [--resume] [--eval-only] [--bench K] [KEY VALUE ...]

One process per GPU (``--num-gpus`` is accepted for CLI compatibility; the
launcher decides the world size).  ``SOLVER.IMS_PER_BATCH`` is global and
split across ranks.  Without ``RUNTIME.COCO_JSON`` the run uses COCO-shaped
synthetic data.  ``--bench K`` times K steps after ``--warmup`` untimed
ones and prints one JSON line (images/s over all ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def setup(args):
    from mdistiller_ddp_amd.detection.config import get_det_cfg, merge_det_file
    cfg = get_det_cfg()
    merge_det_file(cfg, args.config_file)
    if args.opts:
        cfg.merge_from_list(args.opts)
    return cfg


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--config-file", required=True)
    p.add_argument("--num-gpus", type=int, default=1)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--eval-only", action="store_true")
    p.add_argument("--bench", type=int, default=0)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("opts", nargs=argparse.REMAINDER)
    args = p.parse_args(argv)

    import torch
    from mdistiller_ddp_amd.detection.data import build_detection_data
    from mdistiller_ddp_amd.detection.engine import DetectionTrainer, dump_json
    from mdistiller_ddp_amd.detection.evaluation import build_evaluator, inference_on_dataset
    from mdistiller_ddp_amd.detection.tta import GeneralizedRCNNWithTTA
    from mdistiller_ddp_amd.detection.rcnn import build_model
    from mdistiller_ddp_amd.ops.backend import set_backend
    from mdistiller_ddp_amd.parallel.dist import barrier, get_rank, get_world_size, init_distributed, is_master

    info = init_distributed()
    cfg = setup(args)
    set_backend(cfg.RUNTIME.BACKEND)
    device = info.device
    torch.manual_seed(cfg.SEED if cfg.SEED >= 0 else 0)
    model = build_model(cfg).to(device)
    if cfg.MODEL.WEIGHTS and os.path.exists(cfg.MODEL.WEIGHTS):
        sd = torch.load(cfg.MODEL.WEIGHTS, map_location="cpu", weights_only=True)
        sd = sd.get("model", sd)
        missing, unexpected = model.load_state_dict(sd, strict=False)
        if is_master():
            print(f"loaded {cfg.MODEL.WEIGHTS}: {len(missing)} missing, {len(unexpected)} unexpected keys")
    ds, loader = build_detection_data(cfg, get_rank(), get_world_size(), train=True,
                                      device=device if cfg.RUNTIME.SYNTHETIC else "cpu")
    trainer = DetectionTrainer(cfg, model, loader, device)

    if args.bench:
        it = iter(loader)
        model.train()
        for _ in range(args.warmup):
            trainer.run_step(next(it))
        batches = [next(it) for _ in range(args.bench)]
        barrier()
        if device.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.time()
        for b in batches:
            total, _ = trainer.run_step(b)
        if device.type == "cuda":
            torch.cuda.synchronize()
        barrier()
        dt = time.time() - t0
        t = torch.tensor([dt], device=device)
        if get_world_size() > 1:
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
        ims = int(cfg.SOLVER.IMS_PER_BATCH) // get_world_size() * get_world_size()
        if is_master():
            print(json.dumps({"metric": "det_train_images_per_s", "value": round(ims * args.bench / dt, 2),
                              "ms_per_step": round(dt / args.bench * 1e3, 2), "n_gpus": get_world_size(),
                              "global_batch": ims, "config": os.path.basename(args.config_file),
                              "kd": cfg.KD.TYPE, "dtype": cfg.RUNTIME.DTYPE,
                              "final_loss": round(float(total), 4)}))
        return 0

    out_dir = cfg.OUTPUT_DIR
    start = trainer.resume(out_dir) if args.resume else 0
    if not args.eval_only:
        trainer.train(start_iter=start, ckpt_dir=out_dir)
    val_ds, _ = build_detection_data(cfg, train=False, device=device if cfg.RUNTIME.SYNTHETIC else "cpu")
    evaluator = build_evaluator(cfg.RUNTIME.EVALUATOR_TYPE, int(cfg.MODEL.ROI_HEADS.NUM_CLASSES),
                                mask_on=bool(cfg.MODEL.MASK_ON))
    res = inference_on_dataset(model, val_ds, evaluator, autocast=trainer.autocast)
    if cfg.TEST.AUG.ENABLED:  # reference train_net.py:106-117 (test_with_TTA)
        tta = build_evaluator(cfg.RUNTIME.EVALUATOR_TYPE, int(cfg.MODEL.ROI_HEADS.NUM_CLASSES))
        res_tta = inference_on_dataset(GeneralizedRCNNWithTTA(cfg, model), val_ds, tta,
                                       autocast=trainer.autocast)
        res.update({k + "_TTA": v for k, v in res_tta.items()})
    if is_master():
        for k, v in res.items():
            print(f"{k}:", json.dumps(v))
        os.makedirs(out_dir, exist_ok=True)
        dump_json(res, os.path.join(out_dir, "metrics.json"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
