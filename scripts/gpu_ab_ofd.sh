# OFD (teacher BN in train mode) eager vs hipGraph mean loss, bf16 native and fp32 torch.
set -x
Y=configs/cifar100/ofd.yaml
MODES=auto:bf16:1 timeout -k 10 120 python -u scripts/bench_loss_ab.py $Y 100 > gpurun_out/ab1.log 2>&1 && grep final_loss gpurun_out/ab1.log &&
MODES=torch:fp32:0,auto:bf16:0,auto:bf16:1 timeout -k 10 200 python -u scripts/bench_loss_ab.py $Y 300 > gpurun_out/ab4.log 2>&1 && grep final_loss gpurun_out/ab4.log &&
MODES=auto:bf16:1 timeout -k 10 120 python -u scripts/bench_loss_ab.py configs/cifar100/dkd/res32x4_shuv1.yaml 100 DKD.BETA 1.0 > gpurun_out/ab5.log 2>&1 && grep final_loss gpurun_out/ab5.log
