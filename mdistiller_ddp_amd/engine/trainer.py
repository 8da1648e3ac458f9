"""Trainers (reference `mdistiller/engine/trainer.py:42-555`).

``trainer_dict`` keys are the ``SOLVER.TRAINER`` strings of the YAMLs:
``base``, ``crd``, ``dot``, ``crd_dot``.  All four share one epoch loop;
they differ only in the batch layout they feed the distiller (CRD adds the
dataset index and contrastive indices) and in the optimiser (DOT's dual
momentum with two gradient sets), both handled by :class:`TrainStep`.

What the epoch loop keeps from the reference (file formats are identical):

* output dir ``LOG.PREFIX/<experiment_name>`` with ``code/_cfg.yaml``,
  ``code/distiller.py``, ``worklog.txt``, ``worklog.yaml``, optional
  tensorboard events / wandb;
* checkpoints ``latest``, ``epoch_N`` (every ``SAVE_CHECKPOINT_FREQ``),
  ``best`` = ``{"epoch", "model" (``module.``-prefixed distiller state),
  "optimizer" (torch.optim layout), "best_acc"}`` and ``student_latest`` /
  ``student_N`` / ``student_best`` = ``{"model": student state}``;
* ``--resume`` restores model, optimizer, best_acc and epoch from
  ``latest``.

What changes (MI355X-first): the per-iteration body is a captured hipGraph
with no host synchronisation; metrics are read once every
``LOG.METRIC_FREQ`` iterations; BN running statistics are broadcast from
rank 0 before every evaluation/checkpoint (bit-identical to DDP's per-forward
buffer broadcast, without paying it every step); the data sampler is
re-seeded every epoch; a replica checksum can be asserted every
``RUNTIME.CHECK_REPLICAS`` steps; ``RUNTIME.FAULT_INJECT`` kills a rank at a
chosen step (resume tests).
"""
from __future__ import annotations

import inspect
import os
import shutil
import time
from collections import OrderedDict

import torch
import torch.distributed as dist

from ..config import dump_cfg
from ..parallel import dist_fn
from ..parallel.dist import is_master, get_rank, get_world_size, is_dist
from ..utils.logging import log_msg
from .step import TrainStep
from .utils import adjust_learning_rate, save_checkpoint, load_checkpoint, validate

BATCH_KEYS = {
    "base": ("image", "target"),
    "dot": ("image", "target"),
    "crd": ("image", "target", "index", "contrastive_index"),
    "crd_dot": ("image", "target", "index", "contrastive_index"),
}

_DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def _as_batch(data, keys):
    if isinstance(data, dict):
        return data
    return {k: v for k, v in zip(("image", "target", "index", "contrastive_index"), data)}


def strip_module(sd: dict) -> dict:
    return {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}


class BaseTrainer:
    kind = "base"

    def __init__(self, experiment_name, distiller, train_loader, val_loader, cfg, device=None):
        self.cfg = cfg
        self.distiller = distiller
        self.train_loader = train_loader
        self.val_loader = val_loader
        self.device = device or next(distiller.parameters()).device
        self.best_acc = -1.0
        self.log_path = os.path.join(cfg.LOG.PREFIX, experiment_name)
        dtype = _DTYPES[cfg.RUNTIME.DTYPE] if self.device.type == "cuda" else torch.float32
        if cfg.EXPERIMENT.AMP and self.device.type == "cuda":
            dtype = torch.bfloat16  # reference AMP = fp16 autocast + GradScaler; bf16 needs no scaler
        self.dtype = dtype
        from ..runtime import streams
        from ..ops.hip_layers import set_fold_bn
        streams.set_enabled(bool(cfg.RUNTIME.TEACHER_STREAM))
        set_fold_bn(bool(cfg.RUNTIME.FOLD_TEACHER_BN))
        self.step = TrainStep(distiller, cfg, self.device, trainer=self.kind,
                              use_graph=bool(cfg.RUNTIME.HIP_GRAPH), dtype=dtype,
                              batch_keys=BATCH_KEYS[self.kind])
        self.optimizer = self.step.opt
        self.tf_writer = None
        if is_master():
            os.makedirs(self.log_path, exist_ok=True)
            self._init_writer()
            self._dump_code()
        self._fault = self._parse_fault(cfg.RUNTIME.FAULT_INJECT)
        self.global_step = 0

    # ------------------------------------------------------------------ setup
    def _init_writer(self):
        try:
            from tensorboardX import SummaryWriter
        except ImportError:
            try:
                from torch.utils.tensorboard import SummaryWriter
            except Exception:
                SummaryWriter = None
        if SummaryWriter is not None:
            self.tf_writer = SummaryWriter(os.path.join(self.log_path, "train.events"))

    def _dump_code(self):
        code_path = os.path.join(self.log_path, "code")
        os.makedirs(code_path, exist_ok=True)
        with open(os.path.join(code_path, "_cfg.yaml"), "w") as f:
            print(dump_cfg(self.cfg, show=False).dump(), end="", file=f)
        try:  # works for every distiller incl. vanilla (reference D9)
            src = inspect.getsourcefile(type(self.distiller))
            shutil.copyfile(src, os.path.join(code_path, "distiller.py"))
        except (TypeError, OSError):
            pass

    @staticmethod
    def _parse_fault(spec):
        if not spec:
            return None
        r, s = spec.split(":")
        return int(r), int(s)

    # ------------------------------------------------------------------ logging
    def log(self, lr, epoch, log_dict):
        if self.tf_writer is not None:
            for k, v in log_dict.items():
                if isinstance(v, dict):
                    for name, value in v.items():
                        self.tf_writer.add_scalar(f"{k}/{name}", value, epoch)
                else:
                    self.tf_writer.add_scalar(k, v, epoch)
            self.tf_writer.flush()
        if self.cfg.LOG.WANDB:
            try:
                import wandb
                wandb.log({"current lr": lr})
                wandb.log(log_dict)
            except Exception:
                pass
        if log_dict["test_acc"] > self.best_acc and self.cfg.LOG.WANDB:
            try:
                import wandb
                wandb.run.summary["best_acc"] = log_dict["test_acc"]
            except Exception:
                pass
        with open(os.path.join(self.log_path, "worklog.txt"), "a") as w:
            lines = ["-" * 35 + os.linesep, f"epoch: {epoch}" + os.linesep,
                     "lr: {:.4f}".format(float(lr)) + os.linesep]
            for k, v in log_dict.items():
                if isinstance(v, dict):
                    lines.append(f"{k}:" + os.linesep)
                    for name, value in v.items():
                        lines.append("    {}: {:.4f}".format(name, value) + os.linesep)
                elif isinstance(v, int):
                    lines.append("{}: {:d}".format(k, v) + os.linesep)
                else:
                    lines.append("{}: {:.4f}".format(k, float(v)) + os.linesep)
            lines.append("-" * 35 + os.linesep)
            w.writelines(lines)
        with open(os.path.join(self.log_path, "worklog.yaml"), "a") as w:
            lines = [f"- epoch: {epoch}{os.linesep}", f"  lr: {float(lr):.4f}{os.linesep}"]
            for k, v in log_dict.items():
                if isinstance(v, dict):
                    lines.append(f"  {k}:{os.linesep}")
                    for name, value in v.items():
                        lines.append(f"    {name}: {value:.4f}{os.linesep}")
                elif isinstance(v, int):
                    lines.append(f"  {k}: {v:d}{os.linesep}")
                else:
                    lines.append(f"  {k}: {float(v):.4f}{os.linesep}")
            lines.append("\n")
            w.writelines(lines)

    # ------------------------------------------------------------------ state
    def sync_buffers(self):
        """Broadcast every module buffer of the student / distiller modules
        from rank 0 (DDP ``broadcast_buffers`` semantics, paid once per
        evaluation instead of every forward).  CRD banks are excluded: they
        are kept consistent by the update exchange."""
        if not is_dist():
            return
        for name, b in self.distiller.named_buffers():
            if name.startswith("teacher.") or "memory_v" in name:
                continue
            if b.is_floating_point() or b.dtype in (torch.int64, torch.int32, torch.long):
                dist.broadcast(b.data, 0)
        from ..ops.hip_layers import bump_weight_generation
        bump_weight_generation()

    def model_state(self):
        return OrderedDict(("module." + k, v) for k, v in self.distiller.state_dict().items())

    def load_model_state(self, sd):
        from ..ops.hip_layers import bump_weight_generation
        self.distiller.load_state_dict(strip_module(sd))
        bump_weight_generation()

    def save(self, epoch, is_best):
        state = {"epoch": epoch, "model": self.model_state(),
                 "optimizer": self.optimizer.state_dict(), "best_acc": float(self.best_acc)}
        student_state = {"model": self.distiller.student.state_dict()}
        save_checkpoint(state, os.path.join(self.log_path, "latest"))
        save_checkpoint(student_state, os.path.join(self.log_path, "student_latest"))
        if epoch % self.cfg.LOG.SAVE_CHECKPOINT_FREQ == 0:
            save_checkpoint(state, os.path.join(self.log_path, f"epoch_{epoch}"))
            save_checkpoint(student_state, os.path.join(self.log_path, f"student_{epoch}"))
        if is_best:
            save_checkpoint(state, os.path.join(self.log_path, "best"))
            save_checkpoint(student_state, os.path.join(self.log_path, "student_best"))

    def check_replicas(self):
        """Assert bit-identical learnable parameters on every rank."""
        if not is_dist():
            return True
        flat = self.step.flat.data
        s = torch.stack([flat.double().sum(), (flat.double() * torch.arange(
            flat.numel(), device=flat.device, dtype=torch.float64).remainder(97)).sum()])
        allv = [torch.empty_like(s) for _ in range(get_world_size())]
        dist.all_gather(allv, s)
        ok = all(torch.equal(allv[0], a) for a in allv)
        if not ok:
            raise RuntimeError(f"replica divergence detected at step {self.global_step}: "
                               f"{[a.tolist() for a in allv]}")
        return ok

    # ------------------------------------------------------------------ loops
    def train(self, resume=False):
        epoch = 1
        if resume:
            path = os.path.join(self.log_path, "latest")
            state = load_checkpoint(path)
            epoch = state["epoch"] + 1
            self.load_model_state(state["model"])
            self.optimizer.load_state_dict(state["optimizer"])
            self.best_acc = float(state["best_acc"])
            self.step.invalidate_graph()
            if is_master():
                print(log_msg(f"resumed from {path} at epoch {epoch}", "INFO"), flush=True)
        while epoch < self.cfg.SOLVER.EPOCHS + 1:
            self.train_epoch(epoch)
            epoch += 1
        if is_master():
            print(log_msg("Best accuracy:{}".format(self.best_acc), "EVAL"), flush=True)
            with open(os.path.join(self.log_path, "worklog.txt"), "a") as w:
                w.write("best_acc\t" + "{:.2f}".format(float(self.best_acc)))

    def train_epoch(self, epoch):
        cfg = self.cfg
        if hasattr(self.train_loader, "set_epoch"):
            self.train_loader.set_epoch(epoch)
        elif hasattr(getattr(self.train_loader, "sampler", None), "set_epoch"):
            self.train_loader.sampler.set_epoch(epoch)
        n_iter = len(self.train_loader)
        max_iter = int(cfg.RUNTIME.MAX_ITERS_PER_EPOCH) or n_iter
        self.distiller.train()
        self.step.set_epoch(float(epoch))
        if self.step.meters is not None:
            self.step.meters.reset()
        pbar = None
        if is_master():
            try:
                from tqdm import tqdm
                pbar = tqdm(total=min(n_iter, max_iter), dynamic_ncols=True)
            except Exception:  # pragma: no cover
                pbar = None
        freq = max(1, int(cfg.LOG.METRIC_FREQ))
        t0 = time.perf_counter()
        lr = cfg.SOLVER.LR
        prof = StepProfiler(cfg, self.log_path, self.device) if epoch == 1 else None
        keys = BATCH_KEYS[self.kind]
        loader_it = iter(self.train_loader)
        nxt = next(loader_it, None)
        for idx in range(n_iter):
            if nxt is None or idx >= max_iter:
                break
            batch = _as_batch(nxt, keys)
            # one batch of look-ahead (the teacher of batch idx+1 runs during step idx)
            nxt = next(loader_it, None) if idx + 1 < max_iter else None
            lr = adjust_learning_rate(epoch, idx, cfg, n_iter)
            self.step.set_lr(lr)
            if prof is not None:
                prof.before(idx)
            self.step.step(batch, next_batch=None if nxt is None else _as_batch(nxt, keys))
            if prof is not None:
                prof.after(idx)
            self.global_step += 1
            if self._fault is not None and self._fault == (get_rank(), self.global_step):
                raise RuntimeError(f"injected fault on rank {get_rank()} at step {self.global_step}")
            if cfg.RUNTIME.CHECK_REPLICAS and self.global_step % int(cfg.RUNTIME.CHECK_REPLICAS) == 0:
                self.check_replicas()
            if pbar is not None:
                pbar.update()
            if (idx + 1) % freq == 0 and pbar is not None:
                m = self.step.meters.summary(reduce=False)
                dt = (time.perf_counter() - t0) / (idx + 1)
                pbar.set_description(log_msg(
                    "Epoch:{}| Time(step):{:.4f}| Loss:{:.4f}| Top-1:{:.3f}| Top-5:{:.3f}".format(
                        epoch, dt, m["loss"], m["top1"], m["top5"]), "TRAIN"))
        if pbar is not None:
            pbar.close()
        if prof is not None:
            prof.close()
        train_m = self.step.meters.summary(reduce=True)
        self.sync_buffers()
        test_acc, test_acc_top5, test_loss = validate(self.val_loader, self.distiller, self.device,
                                                      self.dtype)
        if is_master():
            keys = [k for k in self.step.meters.loss_keys]
            log_dict = OrderedDict({
                "train_acc": train_m["top1"],
                "train_loss": {k.replace("loss_", ""): train_m[k] for k in keys},
                "test_acc": test_acc,
                "test_acc_top5": test_acc_top5,
                "test_loss": test_loss,
            })
            self.log(lr, epoch, log_dict)
            is_best = test_acc >= self.best_acc
            self.best_acc = max(self.best_acc, test_acc)
            self.save(epoch, is_best)
        if is_dist():
            t = torch.tensor([self.best_acc], dtype=torch.float64, device=self.device)
            dist.broadcast(t, 0)
            self.best_acc = float(t.item())


class StepProfiler:
    """``RUNTIME.PROFILE``: in-framework profiling of a window of
    training steps of the first epoch.

    * hipEvent-bracketed device time of every step in the window (the wall
      between events recorded on the step's stream before and after it) ->
      ``<log>/step_times_rank<r>.txt``, read once at the end (no per-step sync);
    * a ``torch.profiler`` trace of the same window (CPU + ROCm kernel activity)
      -> ``<log>/profile_rank<r>.json`` (chrome trace) plus the kernel table
      ``<log>/profile_rank<r>.txt``.

    Window: ``RUNTIME.PROFILE_START`` .. ``+ RUNTIME.PROFILE_STEPS``.  Kernel
    names are stable (``mda_*`` exports, named HIP kernels), so the table lines
    up with ``rocprofv3 --kernel-trace --stats`` summaries.
    """

    def __init__(self, cfg, log_path, device):
        self.on = bool(cfg.RUNTIME.PROFILE)
        self.start = int(cfg.RUNTIME.PROFILE_START)
        self.stop = self.start + int(cfg.RUNTIME.PROFILE_STEPS)
        self.log_path = log_path
        self.cuda = device.type == "cuda"
        self.events = []
        self.prof = None
        self.rank = get_rank()

    def before(self, idx):
        if not self.on or not (self.start <= idx < self.stop):
            return
        if idx == self.start:
            from torch.profiler import profile, ProfilerActivity
            acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if self.cuda else [])
            self.prof = profile(activities=acts, record_shapes=False)
            self.prof.__enter__()
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events.append([e, None])
        else:
            self.events.append([time.perf_counter(), None])

    def after(self, idx):
        if not self.on or not (self.start <= idx < self.stop):
            return
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events[-1][1] = e
        else:
            self.events[-1][1] = time.perf_counter()
        if idx == self.stop - 1:
            self.close()

    def close(self):
        if not self.on or (self.prof is None and not self.events):
            return
        if self.cuda:
            torch.cuda.synchronize()
            ms = [a.elapsed_time(b) for a, b in self.events if b is not None]
        else:
            ms = [1000.0 * (b - a) for a, b in self.events if b is not None]
        os.makedirs(self.log_path, exist_ok=True)
        with open(os.path.join(self.log_path, f"step_times_rank{self.rank}.txt"), "w") as f:
            for i, v in enumerate(ms):
                f.write(f"{self.start + i}\t{v:.4f}\n")
            if ms:
                f.write(f"# mean_ms\t{sum(ms) / len(ms):.4f}\n")
        if self.prof is not None:
            self.prof.__exit__(None, None, None)
            base = os.path.join(self.log_path, f"profile_rank{self.rank}")
            self.prof.export_chrome_trace(base + ".json")
            key = "self_cuda_time_total" if self.cuda else "self_cpu_time_total"
            with open(base + ".txt", "w") as f:
                f.write(self.prof.key_averages().table(sort_by=key, row_limit=60))
        self.prof = None
        self.events = []
        self.on = False


class CRDTrainer(BaseTrainer):
    kind = "crd"


class DOT(BaseTrainer):
    kind = "dot"


class CRDDOT(BaseTrainer):
    kind = "crd_dot"


trainer_dict = {"base": BaseTrainer, "crd": CRDTrainer, "dot": DOT, "crd_dot": CRDDOT}
