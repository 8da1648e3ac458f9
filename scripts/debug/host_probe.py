"""Is the captured flagship step launch-bound?  Builds the bench step, then
measures with an idle GPU: the host cost of each part of ``TrainStep.step``
(input copies, graph launch) and the GPU time of one replay alone (events
around it), against the steady-state per-step time.

usage: python scripts/debug/host_probe.py [--batch 64]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--cfg", default="configs/cifar100/dkd/res32x4_res8x4.yaml")
    a = ap.parse_args()
    from mdistiller_ddp_amd.config import get_cfg
    from mdistiller_ddp_amd.engine.build import build_distiller
    from mdistiller_ddp_amd.engine.step import TrainStep
    from mdistiller_ddp_amd.engine.trainer import BATCH_KEYS
    from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
    from mdistiller_ddp_amd.benchmark import _calibrate_random_teacher
    dev = torch.device("cuda", 0)
    cfg = get_cfg()
    cfg.merge_from_file(a.cfg)
    cfg.DISTILLER.RANDOM_TEACHER = True
    cfg.freeze()
    d = build_distiller(cfg, num_classes=100, device=dev, num_data=50000)
    _calibrate_random_teacher(d, "cifar100", dev)
    step = TrainStep(d, cfg, dev, trainer=cfg.SOLVER.TRAINER, use_graph=True, dtype=torch.bfloat16,
                     batch_keys=BATCH_KEYS[cfg.SOLVER.TRAINER])
    d.train()
    step.set_epoch(10.0)
    it = iter(SyntheticLoader("cifar100", a.batch, dev, steps_per_epoch=10 ** 9, pool=4, seed=0,
                              channels_last=True))
    cur = next(it)
    for _ in range(30):
        nb = next(it)
        step.step(cur, next_batch=nb)
        cur = nb
    torch.cuda.synchronize()
    g1, g2 = step._graphs
    print("graphs:", step._graphs, "pipe:", step._pipe is not None)
    # GPU time of one replay alone, idle GPU before and after
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    gpu, launch = [], []
    for _ in range(20):
        torch.cuda.synchronize()
        e0.record()
        t0 = time.perf_counter()
        g1.replay()
        launch.append(time.perf_counter() - t0)
        e1.record()
        torch.cuda.synchronize()
        gpu.append(e0.elapsed_time(e1))
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(f"replay alone: gpu {1000 * med(gpu):.1f} us, host launch {1e6 * med(launch):.1f} us")
    # host cost of a whole step() call (idle GPU)
    hs = []
    for _ in range(20):
        torch.cuda.synchronize()
        nb = next(it)
        t0 = time.perf_counter()
        step.step(cur, next_batch=nb)
        hs.append(time.perf_counter() - t0)
        cur = nb
    torch.cuda.synchronize()
    print(f"step() host (idle GPU): {1e6 * med(hs):.1f} us")
    # steady state
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 200
    for _ in range(n):
        nb = next(it)
        step.step(cur, next_batch=nb)
        cur = nb
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(f"steady: {1e6 * t / n:.1f} us/step (host enqueue {1e6 * th / n:.1f} us/step)")
    # steady state of bare replays (no input copies / python)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        g1.replay()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(f"bare replays: {1e6 * t / n:.1f} us/step (host enqueue {1e6 * th / n:.1f} us/step)")


if __name__ == "__main__":
    main()
