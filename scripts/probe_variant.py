import sys, torch
sys.path.insert(0, '.')
from mdistiller_ddp_amd.config import get_cfg
from mdistiller_ddp_amd.engine.build import build_distiller
from mdistiller_ddp_amd.engine.step import TrainStep
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
v = sys.argv[1]
dev = torch.device("cuda", 0) if "dev0" in v else "cuda"
cfg = get_cfg()
if "yaml" in v:
    cfg.merge_from_file("configs/cifar100/kd.yaml")
cfg.DISTILLER.TYPE = "KD"; cfg.DISTILLER.TEACHER = "resnet32x4"; cfg.DISTILLER.STUDENT = "resnet8x4"
cfg.DISTILLER.RANDOM_TEACHER = True
torch.manual_seed(0)
d = build_distiller(cfg, 100, dev, num_data=2000)
if "trainfirst" in v: d.train()
st = TrainStep(d, cfg, dev, trainer="base", use_graph=True, dtype=torch.bfloat16)
d.train()
st.set_epoch(1.0)
ld = SyntheticLoader("cifar100", 32 if "b32" in v else 64, dev, steps_per_epoch=8, channels_last=True,
                     crd_k=1024 if "crd" in v else 0, num_data=2000)
for b in ld:
    if "hold" in v:
        preds, losses = st.step(b)
    else:
        st.step(b)
torch.cuda.synchronize()
print("variant", v, "ok", st.meters.summary(reduce=False)["loss"], flush=True)
