"""Per-step losses of a config on the GPU (eager vs graph, bf16 vs fp32):
debugging aid for divergence/NaN reports from benchmarks/throughput.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mdistiller_ddp_amd.config import get_cfg
from mdistiller_ddp_amd.engine.build import build_distiller
from mdistiller_ddp_amd.engine.step import TrainStep
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader


def run(yaml, steps, graph, dtype, backend="auto"):
    from mdistiller_ddp_amd.ops.backend import set_backend
    set_backend(backend)
    cfg = get_cfg()
    cfg.merge_from_file(yaml)
    cfg.DISTILLER.RANDOM_TEACHER = True
    torch.manual_seed(0)
    d = build_distiller(cfg, 100, "cuda")
    d.train()
    st = TrainStep(d, cfg, "cuda", use_graph=graph, dtype=dtype)
    st.set_epoch(5.0)
    st.set_lr(cfg.SOLVER.LR)
    out = []
    for b in SyntheticLoader("cifar100", 64, "cuda", steps_per_epoch=steps, pool=4, channels_last=True):
        p, l = st.step(b)
        out.append((float(l["loss_ce"]), float(l["loss_kd"]), float(p.float().abs().max())))
    return out


if __name__ == "__main__":
    yaml, steps = sys.argv[1], int(sys.argv[2])
    for graph, dt, be in ((False, torch.float32, "torch"), (False, torch.bfloat16, "auto"),
                          (True, torch.bfloat16, "auto")):
        r = run(yaml, steps, graph, dt, be)
        print(f"graph={graph} dtype={dt} backend={be}")
        for i, (a, b, c) in enumerate(r):
            print(f"  {i:3d} ce {a:10.4f} kd {b:12.4f} |logit|max {c:10.3f}")
