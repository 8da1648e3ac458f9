"""OFD (train-mode teacher BN) with the teacher look-ahead forced on and a
caller that passes no next batch: which step goes non-finite, and in which
teacher output?  Per step: loss values, and the max |.| of every teacher
output buffer the step graph reads."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from mdistiller_ddp_amd.config import get_cfg
from mdistiller_ddp_amd.engine.build import build_distiller
from mdistiller_ddp_amd.engine.step import TrainStep
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader

mode = sys.argv[1] if len(sys.argv) > 1 else "nonext"
cfg = get_cfg()
cfg.DISTILLER.TYPE = "OFD"
cfg.DISTILLER.TEACHER = "resnet32x4"
cfg.DISTILLER.STUDENT = "resnet8x4"
cfg.DISTILLER.RANDOM_TEACHER = True
cfg.RUNTIME.TEACHER_LOOKAHEAD = os.environ.get("LA", "on")
if len(sys.argv) > 2:
    cfg.merge_from_list(sys.argv[2:])
torch.manual_seed(0)
d = build_distiller(cfg, 100, "cuda")
d.train()
st = TrainStep(d, cfg, "cuda", use_graph=True, dtype=torch.bfloat16)
st.set_epoch(1.0)
bs = list(SyntheticLoader("cifar100", 32, "cuda", steps_per_epoch=int(os.environ.get("STEPS", "10")), channels_last=True))
for i, b in enumerate(bs):
    nxt = bs[i + 1] if (mode == "next" and i + 1 < len(bs)) else None
    preds, losses = st.step(b, nxt)
    torch.cuda.synchronize()
    if i >= int(os.environ.get("SHOW", "6")):
        if i % 10 == 9 or i == len(bs) - 1:
            print(i, {k: round(float(v), 4) for k, v in losses.items()},
                  "bad", [n for n, t in d.named_buffers() if t.is_floating_point() and not torch.isfinite(t).all()][:3], flush=True)
        continue
    lv = {k: round(float(v), 4) for k, v in losses.items()}
    feed = getattr(d, "_teacher_feed", None)
    tinfo = ""
    if feed is not None:
        for name in ("_x", "x_bufs", "bufs", "_bufs"):
            if hasattr(feed, name):
                tinfo = name
    def _flat(o, acc):
        if torch.is_tensor(o):
            acc.append(o)
        elif isinstance(o, dict):
            for v in o.values():
                _flat(v, acc)
        elif isinstance(o, (list, tuple)):
            for v in o:
                _flat(v, acc)
        return acc
    bad_p = [n for n, t in list(d.teacher.named_parameters()) + list(d.teacher.named_buffers())
             if t.is_floating_point() and not torch.isfinite(t).all()]
    bad_s = [n for n, t in list(d.named_parameters()) + list(d.named_buffers())
             if not n.startswith("teacher.") and t.is_floating_point() and not torch.isfinite(t).all()]
    xs = _flat(feed.X, []) if feed is not None and feed.X is not None else []
    bad_x = [(j, tuple(t.shape)) for j, t in enumerate(xs) if not torch.isfinite(t.float()).all()]
    if i >= int(os.environ.get("SHOW", "6")):
        continue
    bad_bn = [n for n, m in d.named_modules() if isinstance(m, torch.nn.BatchNorm2d)
              and not n.startswith("teacher.") and not (torch.isfinite(m.running_mean).all()
                                                       and torch.isfinite(m.running_var).all())]
    big_bn = [(n, round(float(m.running_var.max()), 2)) for n, m in d.named_modules()
              if isinstance(m, torch.nn.BatchNorm2d) and n.startswith("connectors")]
    print("   bad bn", bad_bn[:8], "conn", big_bn, flush=True)
    print("   bad teacher", bad_p[:6], "bad other", bad_s[:6], "bad X", bad_x, "nX", len(xs), flush=True)
    print(i, "graph" if st._graphs is not None else "eager", "tsplit" if st._tsplit is not None else "-",
          "la" if st._pipe is not None else "-", lv, "pmax", float(preds.float().abs().max()),
          "rm", [round(float(m.running_var.float().abs().max()), 3) for m in d.teacher.modules()
                 if isinstance(m, torch.nn.BatchNorm2d)][:3], flush=True)
