"""ResNet-50 mixed-precision DDP (reference: resnet_ddp_apex.py, "Apex").

fp16 compute + native dynamic loss scaling (pytorch_distributed_amd.amp.LossScaler,
GradScaler-compatible defaults 2**16 / x2 per 2000 / x0.5); MX_DTYPE=bf16 selects bf16.
"""
from restnet_ddp import launch

if __name__ == "__main__":
    launch("ddp_amp")
