"""Throughput measurement of a full distillation training step.

Shared by ``bench.py`` (the headline metric) and
``benchmarks/throughput.py`` (all BASELINE configs).  One timed step is the
framework's real ``TrainStep``: batch copy into the step's input buffers,
teacher forward (no grad, own stream), student forward, losses, backward,
gradient all-reduce (world > 1), optimizer update, BN running-stat updates
and on-device metrics (with the teacher look-ahead, the teacher forward a step
runs is that of the next batch -- still one teacher forward of fresh data
per step).  Timing: W untimed warm-up steps, then K steps
bracketed by a barrier and a device synchronisation on both sides; the
slowest rank's time is reported.
"""
from __future__ import annotations

import gc
import os
import time

import torch


TEACHER_LOGIT_STD = 4.0


def _calibrate_random_teacher(distiller, ds, dev) -> None:
    """Rescale a random-init teacher's classifier to a trained teacher's logit range.

    A random ResNet32x4 in eval mode emits logits with std ~25.  A DKD loss
    on those (~450) drives some students to inf/NaN on the first step; the
    ShuffleNetV1 pair does this in the reference's PyTorch formulation on
    the CPU too.  Scaling the last Linear to logit std TEACHER_LOGIT_STD is
    still a random teacher of the same architecture.  It keeps every
    configuration's loss finite and leaves the timed work unchanged.
    """
    import torch.nn as nn
    teacher = getattr(distiller, "teacher", None)
    if teacher is None:
        return
    fc = [m for m in teacher.modules() if isinstance(m, nn.Linear)]
    if not fc:
        return
    from .data.synthetic import SyntheticLoader
    b = next(iter(SyntheticLoader(ds, 32, dev, steps_per_epoch=1, pool=1, seed=99,
                                  channels_last=(dev.type == "cuda"))))
    was = teacher.training
    teacher.eval()
    with torch.no_grad():
        out = teacher(b["image"])
        logits = out[0] if isinstance(out, (tuple, list)) else out
        std = float(logits.float().std())
        if std > 0:
            fc[-1].weight.mul_(TEACHER_LOGIT_STD / std)
            if fc[-1].bias is not None:
                fc[-1].bias.mul_(TEACHER_LOGIT_STD / std)
    teacher.train(was)


def run(cfg_file: str, per_gpu_batch: int, steps: int, warmup: int, opts=(), use_graph=True,
        backend="auto", dtype="bf16", teacher_stream=True, dataset=None, crd_k=None,
        check_replicas=False):
    from .ops.backend import set_backend
    from .parallel import dist as D
    from .config import get_cfg
    from .engine.build import build_distiller
    from .engine.step import TrainStep
    from .engine.trainer import BATCH_KEYS
    from .data.synthetic import SyntheticLoader, dataset_shape
    from .runtime import streams

    set_backend(backend)
    streams.set_enabled(teacher_stream)
    # release the graphs of an earlier run in this process first: a live graph
    # keeps its internal parallel streams (and their hardware queues), which
    # changes how the next step's concurrent streams share queues
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    info = D.init_distributed() if not D.is_dist() else D.info()
    dev = info.device
    if dev.type == "cuda":
        torch.backends.cudnn.benchmark = True
    cfg = get_cfg()
    cfg.merge_from_file(cfg_file)
    if opts:
        cfg.merge_from_list(list(opts))
    cfg.DISTILLER.RANDOM_TEACHER = True
    cfg.freeze()
    ds = dataset or cfg.DATASET.TYPE
    _, ncls, ntrain, _ = dataset_shape(ds)
    # same seed on every rank is NOT relied upon: TrainStep broadcasts rank 0's
    # full state (C2) -- rank-dependent seeding here proves it
    torch.manual_seed(1234 + info.rank)
    distiller = build_distiller(cfg, num_classes=ncls, device=dev, num_data=ntrain)
    _calibrate_random_teacher(distiller, ds, dev)
    dt = torch.bfloat16 if (dtype == "bf16" and dev.type == "cuda") else torch.float32
    trainer = cfg.SOLVER.TRAINER
    step = TrainStep(distiller, cfg, dev, trainer=trainer, use_graph=use_graph, dtype=dt,
                     batch_keys=BATCH_KEYS[trainer],
                     warmup_eager=int(os.environ.get("MDA_WARMUP_EAGER", "3")))
    distiller.train()
    # past any warm-up ramp (DKD / ReviewKD): full loss
    step.set_epoch(float(max(cfg.DKD.WARMUP, cfg.REVIEWKD.WARMUP_EPOCHS) + 1))
    step.set_lr(cfg.SOLVER.LR)
    k = (crd_k if crd_k is not None else cfg.CRD.NCE.K) if cfg.DISTILLER.TYPE == "CRD" else 0
    loader = SyntheticLoader(ds, per_gpu_batch, dev, steps_per_epoch=10 ** 9, pool=4,
                             seed=info.rank, crd_k=k, num_data=ntrain,
                             channels_last=(dev.type == "cuda"))
    it = iter(loader)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    # each step is handed the batch of the step after it (what a prefetching data
    # loader has ready), so the captured step can run that batch's teacher forward
    # beside this step's student work (TrainStep teacher look-ahead)
    cur = next(it)

    def advance(b):
        nb = next(it)
        step.step(b, next_batch=nb)
        return nb

    # the set-up objects (models, graphs, earlier configs in this process) move to
    # the permanent generation: the timed loop's generation-2 collections no longer
    # walk them.  Launch-bound steps (DOT's five graph replays) otherwise slow down
    # with the process history (1.33 -> 1.60 ms/step after two other configs).
    # The collection runs BEFORE the last warm-up step, not between it and the
    # timed loop: a ~50 ms gc.collect() there left the host caches cold and the
    # GPU idle, and the first timed steps paid for it -- +30 us/step on a 20-step
    # window, 0.875 vs 0.845 ms (profiles/r6_ab.md)
    gc_frozen = os.environ.get("MDA_GC_FREEZE", "1") != "0"
    for i in range(warmup):
        if gc_frozen and i == warmup - 1:
            gc.collect()
            gc.freeze()
        cur = advance(cur)
    if gc_frozen and warmup == 0:
        gc.collect()
        gc.freeze()
    sync()
    D.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        cur = advance(cur)
    host = time.perf_counter() - t0  # host time to enqueue the K steps (launch-bound if ~el)
    sync()
    D.barrier()
    sync()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if D.is_dist():
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    el = float(t.item())
    # host cost of enqueueing one step with an idle GPU (no queue back-pressure):
    # the launch-bound floor of the step
    hs = []
    for _ in range(10):
        sync()
        h0 = time.perf_counter()
        cur = advance(cur)
        hs.append(time.perf_counter() - h0)
    sync()
    if gc_frozen:
        gc.unfreeze()
    m = step.meters.summary(reduce=True)
    n = info.world_size
    same = None
    if check_replicas and D.is_dist():
        # after the timed steps: every rank's parameters (student, distiller modules,
        # teacher) must equal rank 0's
        from .parallel import state_checksum
        c = state_checksum(distiller, step.flat, buffers=False)
        allc = [torch.empty_like(c) for _ in range(n)]
        torch.distributed.all_gather(allc, c)
        same = all(torch.equal(allc[0], a) for a in allc)
    return {
        "seconds": el,
        "ms_per_step": 1000.0 * el / steps,
        "host_ms_per_step": 1000.0 * host / steps,
        "host_idle_ms_per_step": 1000.0 * sorted(hs)[len(hs) // 2],
        "images_per_s": n * per_gpu_batch * steps / el,
        "n_gpus": n,
        "global_batch": n * per_gpu_batch,
        "final_loss": m["loss"],
        "graph": step.use_graph,
        "graph_comm": step.graph_comm,
        "comm_backend": info.backend,
        "replicas_identical": same,
        "dtype": "bf16" if dt == torch.bfloat16 else "fp32",
        "rank": info.rank,
    }
