"""mdistiller_ddp_amd -- an MI355X-native knowledge-distillation framework.

Capabilities of youngyoonii/mdistiller-ddp (13 KD methods + vanilla, DOT,
CIFAR-100 / Tiny-ImageNet / ImageNet model zoos, torchrun DDP CLI, yacs-style
YAML configs, checkpoint format) re-designed for AMD Instinct MI355X (gfx950):
hand-written CDNA4 HIP kernels for the hot ops, RCCL over xGMI for data
parallelism, hipGraph-captured training steps.
"""
__version__ = "0.1.0"
