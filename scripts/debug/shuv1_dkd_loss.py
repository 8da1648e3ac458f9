"""Is ShuffleV1's large DKD loss inherent?  40 DKD steps of res32x4 -> ShuffleV1
(random teacher), native bf16 hipGraph vs PyTorch fp32 eager (NCHW)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mdistiller_ddp_amd.config import get_cfg  # noqa: E402
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader  # noqa: E402
from mdistiller_ddp_amd.engine.build import build_distiller  # noqa: E402
from mdistiller_ddp_amd.engine.step import TrainStep  # noqa: E402
from mdistiller_ddp_amd.ops.backend import use_backend  # noqa: E402

cfg = get_cfg()
cfg.merge_from_file("configs/cifar100/dkd/res32x4_shuv1.yaml")
cfg.DISTILLER.RANDOM_TEACHER = True
torch.manual_seed(0)
d1 = build_distiller(cfg, 100, "cuda")
d2 = copy.deepcopy(d1)
for d, g, dt, be in ((d1, True, torch.bfloat16, "auto"), (d2, False, torch.float32, "torch")):
    with use_backend(be):
        d.train()
        cl = be != "torch"
        st = TrainStep(d, cfg, "cuda", use_graph=g, dtype=dt, channels_last=cl)
        st.set_epoch(1.0)
        ld = SyntheticLoader("cifar100", 64, "cuda", steps_per_epoch=40, channels_last=cl)
        for i, b in enumerate(ld):
            preds, losses = st.step(b)
            if i % 10 == 9:
                torch.cuda.synchronize()
                print(f"{be}: step {i + 1} " + " ".join(f"{k} {float(v):.4g}" for k, v in losses.items()), flush=True)
