"""Default configuration tree.

Schema parity with the reference's yacs tree (`mdistiller/engine/cfg.py:26-194`):
every key the reference declares exists here with the same default, so all 45
shipped YAMLs merge unchanged and CLI ``KEY VALUE`` overrides behave the same.

MI355X-native additions live in two extra nodes that the reference does not
have (`RUNTIME`, `DIST`) plus a few leaf keys (marked ``# ext``); they default
to the fast path and never change the meaning of a reference key.
"""
from __future__ import annotations

from .cfgnode import CfgNode as CN

CFG = CN()

# Experiment ---------------------------------------------------------------
CFG.EXPERIMENT = CN()
CFG.EXPERIMENT.PROJECT = "distill"
CFG.EXPERIMENT.NAME = ""
CFG.EXPERIMENT.TAG = "default"
CFG.EXPERIMENT.DDP = False
CFG.EXPERIMENT.AMP = False
CFG.EXPERIMENT.SEED = -1             # ext: <0 = nondeterministic seeding
CFG.EXPERIMENT.DETERMINISTIC = False  # ext: deterministic reductions / algos

# Dataset ------------------------------------------------------------------
CFG.DATASET = CN()
CFG.DATASET.TYPE = "cifar100"
CFG.DATASET.NUM_WORKERS = 2
CFG.DATASET.TEST = CN()
CFG.DATASET.TEST.BATCH_SIZE = 64
CFG.DATASET.SYNTHETIC = False        # ext: device-resident synthetic data of the dataset's shape
CFG.DATASET.SYNTHETIC_SIZE = 0       # ext: #train samples for synthetic data (0 = real dataset size)
CFG.DATASET.GPU_AUG = True           # ext: crop/flip/normalise on device (HIP kernel)
CFG.DATASET.ROOT = ""                # ext: data root ('' = <repo>/data)

# Distiller ----------------------------------------------------------------
CFG.DISTILLER = CN()
CFG.DISTILLER.TYPE = "NONE"  # Vanilla as default
CFG.DISTILLER.TEACHER = "ResNet50"
CFG.DISTILLER.STUDENT = "resnet32"
CFG.DISTILLER.TEACHER_CKPT = ""      # ext: override teacher checkpoint path
CFG.DISTILLER.RANDOM_TEACHER = False  # ext: allow random-init teacher (benchmarks only)

# Solver -------------------------------------------------------------------
CFG.SOLVER = CN()
CFG.SOLVER.TRAINER = "base"
CFG.SOLVER.BATCH_SIZE = 64
CFG.SOLVER.EPOCHS = 240
CFG.SOLVER.LR = 0.05
CFG.SOLVER.WEIGHT_DECAY = 0.0001
CFG.SOLVER.TYPE = "SGD"
CFG.SOLVER.GRAD_CLIP = 0.0
CFG.SOLVER.SGD = CN()
CFG.SOLVER.SGD.MOMENTUM = 0.9
CFG.SOLVER.ADAM = CN()
CFG.SOLVER.ADAM.BETAS = [0.9, 0.999]
CFG.SOLVER.ADAM.EPSILON = 1.0e-8
CFG.SOLVER.SCHEDULE = CN()
CFG.SOLVER.SCHEDULE.TYPE = "MULTISTEP"
CFG.SOLVER.SCHEDULE.MULTISTEP = CN()
CFG.SOLVER.SCHEDULE.MULTISTEP.STAGES = [150, 180, 210]
CFG.SOLVER.SCHEDULE.MULTISTEP.RATE = 0.1
CFG.SOLVER.SCHEDULE.COSINE = CN()
CFG.SOLVER.SCHEDULE.COSINE.WARMUP = 5
CFG.SOLVER.SCHEDULE.COSINE.RATE = 1.0e-4
CFG.SOLVER.DOT = CN()
CFG.SOLVER.DOT.DELTA = 0.075

# Log ----------------------------------------------------------------------
CFG.LOG = CN()
CFG.LOG.TENSORBOARD_FREQ = 500
CFG.LOG.SAVE_CHECKPOINT_FREQ = 40
CFG.LOG.PREFIX = "./output"
CFG.LOG.WANDB = False
CFG.LOG.METRIC_FREQ = 50             # ext: iterations between on-device metric syncs

# Runtime (ext) ------------------------------------------------------------
CFG.RUNTIME = CN()
CFG.RUNTIME.BACKEND = "auto"         # auto | hip | torch   (kernel backend)
CFG.RUNTIME.DTYPE = "bf16"           # bf16 | fp32           (compute dtype on GPU)
CFG.RUNTIME.HIP_GRAPH = True         # capture fwd+bwd+step into a hipGraph
CFG.RUNTIME.TEACHER_STREAM = True    # teacher forward on its own HIP stream
CFG.RUNTIME.DOT_DUAL_STREAM = True   # DOT: replay the task / KD backwards as concurrent graphs
# DOT: both backwards as ONE pass over two stacked cotangents (auto = CIFAR
# ResNet students on the HIP kernels; otherwise the two-pass path above)
CFG.RUNTIME.DOT_SINGLE_PASS = "auto"
CFG.RUNTIME.TEACHER_LOOKAHEAD = "auto"  # auto | on | off: captured steps run the teacher of batch t+1
                                        # beside the student step t (auto: off for >= 128 px feature KD)
CFG.RUNTIME.TEACHER_GRAPH = "split"  # split | fork: the look-ahead teacher as its OWN single-chain graph
                                     # replayed on the teacher stream (split), or forked inside the step graph
CFG.RUNTIME.TEACHER_FIRST = True     # split: enqueue the teacher graph before the student's
CFG.RUNTIME.WGRAD_DEFER = True       # captured backward: all layers' wgrad split reductions in one launch
CFG.RUNTIME.FOLD_TEACHER_BN = True   # fold frozen teacher BN into conv weights
CFG.RUNTIME.PROFILE = False          # torch.profiler trace + hipEvent step times of a window
CFG.RUNTIME.PROFILE_START = 20       #   first profiled iteration of epoch 1
CFG.RUNTIME.PROFILE_STEPS = 10       #   window length
CFG.RUNTIME.MAX_ITERS_PER_EPOCH = 0  # >0: truncate epochs (smoke / CI)
CFG.RUNTIME.FAULT_INJECT = ""        # "rank:step" -> raise on that rank at that step (tests)
CFG.RUNTIME.CHECK_REPLICAS = 0       # >0: every N steps assert param checksums equal across ranks

# Distributed (ext) --------------------------------------------------------
CFG.DIST = CN()
CFG.DIST.BACKEND = "auto"            # auto -> nccl(RCCL) on GPU, gloo on CPU
CFG.DIST.BUCKET_MB = 0.0             # gradient bucket size (MB of fp32); 0 = auto:
                                     # total / 4 clamped to [0.5, 8] MB (parallel/grad_reducer.py)
CFG.DIST.TIMEOUT_S = 600
CFG.DIST.GRAD_DTYPE = "fp32"         # fp32 | bf16 wire format for gradient all-reduce
CFG.DIST.GRAPH_COMM = "auto"         # events | split | auto (= events):
                                     # per-bucket all-reduce behind events of the captured backward
                                     # (events), or eager between the fwd+bwd and update graphs (split)
CFG.DIST.BROADCAST_INIT = True       # rank-0 broadcast of all params/buffers at step construction (C2)

# Distillation methods -----------------------------------------------------
CFG.KD = CN()
CFG.KD.TEMPERATURE = 4
CFG.KD.LOSS = CN()
CFG.KD.LOSS.CE_WEIGHT = 0.1
CFG.KD.LOSS.KD_WEIGHT = 0.9

CFG.AT = CN()
CFG.AT.P = 2
CFG.AT.LOSS = CN()
CFG.AT.LOSS.CE_WEIGHT = 1.0
CFG.AT.LOSS.FEAT_WEIGHT = 1000.0

CFG.RKD = CN()
CFG.RKD.DISTANCE_WEIGHT = 25
CFG.RKD.ANGLE_WEIGHT = 50
CFG.RKD.LOSS = CN()
CFG.RKD.LOSS.CE_WEIGHT = 1.0
CFG.RKD.LOSS.FEAT_WEIGHT = 1.0
CFG.RKD.PDIST = CN()
CFG.RKD.PDIST.EPSILON = 1e-12
CFG.RKD.PDIST.SQUARED = False

CFG.FITNET = CN()
CFG.FITNET.HINT_LAYER = 2  # (0, 1, 2, 3, 4)
CFG.FITNET.INPUT_SIZE = [32, 32]
CFG.FITNET.LOSS = CN()
CFG.FITNET.LOSS.CE_WEIGHT = 1.0
CFG.FITNET.LOSS.FEAT_WEIGHT = 100.0

CFG.KDSVD = CN()
CFG.KDSVD.K = 1
CFG.KDSVD.LOSS = CN()
CFG.KDSVD.LOSS.CE_WEIGHT = 1.0
CFG.KDSVD.LOSS.FEAT_WEIGHT = 1.0

CFG.OFD = CN()
CFG.OFD.LOSS = CN()
CFG.OFD.LOSS.CE_WEIGHT = 1.0
CFG.OFD.LOSS.FEAT_WEIGHT = 0.001
CFG.OFD.CONNECTOR = CN()
CFG.OFD.CONNECTOR.KERNEL_SIZE = 1
CFG.OFD.TEACHER_TRAIN_BN = True      # ext: reference OFD leaves teacher BN in train mode

CFG.NST = CN()
CFG.NST.LOSS = CN()
CFG.NST.LOSS.CE_WEIGHT = 1.0
CFG.NST.LOSS.FEAT_WEIGHT = 50.0

CFG.PKT = CN()
CFG.PKT.LOSS = CN()
CFG.PKT.LOSS.CE_WEIGHT = 1.0
CFG.PKT.LOSS.FEAT_WEIGHT = 30000.0

CFG.SP = CN()
CFG.SP.LOSS = CN()
CFG.SP.LOSS.CE_WEIGHT = 1.0
CFG.SP.LOSS.FEAT_WEIGHT = 3000.0

CFG.VID = CN()
CFG.VID.LOSS = CN()
CFG.VID.LOSS.CE_WEIGHT = 1.0
CFG.VID.LOSS.FEAT_WEIGHT = 1.0
CFG.VID.EPS = 1e-5
CFG.VID.INIT_PRED_VAR = 5.0
CFG.VID.INPUT_SIZE = [32, 32]

CFG.CRD = CN()
CFG.CRD.MODE = "exact"  # ("exact", "relax")
CFG.CRD.FEAT = CN()
CFG.CRD.FEAT.DIM = 128
CFG.CRD.FEAT.STUDENT_DIM = 256
CFG.CRD.FEAT.TEACHER_DIM = 256
CFG.CRD.LOSS = CN()
CFG.CRD.LOSS.CE_WEIGHT = 1.0
CFG.CRD.LOSS.FEAT_WEIGHT = 0.8
CFG.CRD.NCE = CN()
CFG.CRD.NCE.K = 16384
CFG.CRD.NCE.MOMENTUM = 0.5
CFG.CRD.NCE.TEMPERATURE = 0.07

CFG.REVIEWKD = CN()
CFG.REVIEWKD.CE_WEIGHT = 1.0
CFG.REVIEWKD.REVIEWKD_WEIGHT = 1.0
CFG.REVIEWKD.WARMUP_EPOCHS = 20
CFG.REVIEWKD.SHAPES = [1, 8, 16, 32]
CFG.REVIEWKD.OUT_SHAPES = [1, 8, 16, 32]
CFG.REVIEWKD.IN_CHANNELS = [64, 128, 256, 256]
CFG.REVIEWKD.OUT_CHANNELS = [64, 128, 256, 256]
CFG.REVIEWKD.MAX_MID_CHANNEL = 512
CFG.REVIEWKD.STU_PREACT = False

CFG.DKD = CN()
CFG.DKD.CE_WEIGHT = 1.0
CFG.DKD.ALPHA = 1.0
CFG.DKD.BETA = 8.0
CFG.DKD.T = 4.0
CFG.DKD.WARMUP = 20

METHOD_NODES = ("KD", "AT", "RKD", "FITNET", "KDSVD", "OFD", "NST", "PKT", "SP",
                "VID", "CRD", "REVIEWKD", "DKD")


def get_cfg() -> CN:
    """A fresh, mutable copy of the default tree."""
    return CFG.clone()


def dump_cfg(cfg: CN, show: bool = False) -> CN:
    """The experiment-facing subset of ``cfg`` (reference `cfg.py:5-23`):
    the five common nodes, the runtime/dist extensions and the active
    method's node only."""
    from ..utils.logging import log_msg

    dump = CN()
    for key in ("EXPERIMENT", "DATASET", "DISTILLER", "SOLVER", "LOG", "RUNTIME", "DIST"):
        if key in cfg:
            dump[key] = cfg[key].clone()
    distiller_type = cfg.DISTILLER.TYPE
    if distiller_type.startswith("SRMD."):
        distiller_type = distiller_type[5:]
    if distiller_type in cfg:
        dump[distiller_type] = cfg[distiller_type].clone()
    if show:
        print(log_msg("CONFIG:\n{}".format(dump.dump()), "INFO"))
    return dump
