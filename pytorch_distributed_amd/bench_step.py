"""One full training step per engine, shared by ``bench.py`` and the GPU tests.

``make_trainer(...).step(i)`` = generate batch ``i`` on device -> forward -> loss
-> backward (bucketed all-reduce when distributed) -> SGD(momentum, wd) update.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from .data.synthetic import SyntheticImageNet

__all__ = ["make_trainer", "tensor_checksum"]


def tensor_checksum(tensors) -> torch.Tensor:
    """Bit-exact, order-independent checksum of float tensors: int64[2] = (sum of the raw bit
    patterns, sum of bit pattern x (index mod 65521 + 1)), with wrapping int64 arithmetic. Equal
    on two ranks iff (with overwhelming probability) every element is bitwise equal."""
    tensors = [t for t in tensors if t is not None and t.numel()]
    dev = tensors[0].device
    c = torch.zeros(2, dtype=torch.int64, device=dev)
    ints = {4: torch.int32, 2: torch.int16, 8: torch.int64}
    for t in tensors:
        x = t.detach().contiguous().view(-1)
        b = x.view(ints[x.element_size()]).to(torch.int64)
        w = torch.arange(b.numel(), dtype=torch.int64, device=dev) % 65521 + 1
        c[0] += b.sum()
        c[1] += (b * w).sum()
    return c


class _TorchTrainer:
    """PyTorch-ROCm reference engine (MIOpen/hipBLASLt) -- oracle and fallback only."""

    engine = "torch"

    def __init__(self, arch, batch, dtype, device, world, rank, bucket_mb, image_size):
        from .models.resnet import build_model
        torch.manual_seed(0)
        self.model = build_model(arch).to(device).to(memory_format=torch.channels_last)
        self.dtype = dtype
        self.device = device
        self.batch = batch
        self.world, self.rank = world, rank
        self.ds = SyntheticImageNet("train", seed=0, image_size=image_size)
        if world > 1:
            from .parallel.ddp import DistributedDataParallel
            self.net = DistributedDataParallel(self.model, bucket_cap_mb=bucket_mb)
        else:
            self.net = self.model
        self.opt = torch.optim.SGD(self.model.parameters(), lr=0.1, momentum=0.9,
                                   weight_decay=1e-4, foreach=True)
        self.crit = nn.CrossEntropyLoss()
        self._loss = None

    def step(self, i: int) -> None:
        ids = torch.arange(self.batch, device=self.device) + (i * self.world + self.rank) * self.batch
        x, y = self.ds.batch(ids, device=self.device)
        x = x.contiguous(memory_format=torch.channels_last)
        with torch.autocast(self.device.type, dtype=self.dtype, enabled=self.dtype != torch.float32):
            out = self.net(x)
        loss = self.crit(out.float(), y)
        self.opt.zero_grad(set_to_none=False)
        loss.backward()
        self.opt.step()
        self._loss = loss.detach()

    def last_loss(self) -> Optional[float]:
        return None if self._loss is None else float(self._loss.item())

    def state_checksum(self) -> torch.Tensor:
        ps = list(self.model.parameters())
        moms = [self.opt.state.get(p, {}).get("momentum_buffer") for p in ps]
        return tensor_checksum(ps + moms)


class _DPTrainer:
    """Single-process multi-GPU DataParallel step (the reference's ``resnet_dp.py`` configuration):
    one native replica per GPU, each replica's forward+loss+backward replayed from a HIP graph,
    one grouped in-process RCCL all-reduce, replicated fused SGD. Each GPU generates its own chunk
    of the global batch (no scatter from GPU 0)."""

    engine = "native-dp"

    def __init__(self, arch, batch, dtype, devices, image_size):
        from .models.native import NativeResNet
        from .models.resnet import build_model
        from .parallel.dp import DataParallel
        torch.manual_seed(0)
        dev0 = torch.device("cuda", devices[0])
        self.dp = DataParallel(NativeResNet(build_model(arch), device=dev0, dtype=dtype,
                                            image_size=image_size), device_ids=list(devices))
        self.opt = self.dp.make_optimizer(lr=0.1, momentum=0.9, weight_decay=1e-4)
        ds = SyntheticImageNet("train", seed=0, image_size=image_size)
        self.gens = [m.input_generator(ds) for m in self.dp.all_modules]
        self.batch, self.n = batch, len(devices)
        self.graphed = True
        self._loss = None

    def step(self, i: int) -> None:
        base = i * self.batch * self.n
        xs, ys = [], []
        for r, g in enumerate(self.gens):
            x, y = g(torch.arange(self.batch, dtype=torch.int64) + base + r * self.batch)
            xs.append(x)
            ys.append(y)
        self._loss = self.dp.train_step_chunks(xs, ys, self.opt)

    def last_loss(self) -> Optional[float]:
        return None if self._loss is None else float(self._loss.item())

    def state_checksum(self) -> torch.Tensor:
        """Replica 0's checksum; raises if any replica's weights differ from it (the replicated
        SGD must keep every GPU's copy bit-identical)."""
        sums = [tensor_checksum([m.flat_params]).cpu() for m in self.dp.all_modules]
        if any(not torch.equal(sums[0], c) for c in sums[1:]):
            raise RuntimeError(f"DataParallel replicas diverged: {[c.tolist() for c in sums]}")
        return sums[0]


class _DPTrainerCPU(_TorchTrainer):
    """``bench.py --dp --device cpu``: the rehearsal of the DataParallel pass's launch and record
    contract without a GPU -- the framework's DataParallel around the torch-engine model on the CPU
    (no replicas), one autograd step per call."""

    engine = "torch-dp-cpu"

    def __init__(self, arch, batch, dtype, image_size):
        super().__init__(arch, batch, dtype, torch.device("cpu"), 1, 0, 32.0, image_size)
        from .parallel.dp import DataParallel
        self.dp = DataParallel(self.model)
        self.net = self.dp
        self.graphed = False


def make_dp_trainer(arch: str, batch: int, dtype: torch.dtype, ngpus: int, image_size: int = 224,
                    device: str = "cuda"):
    if device == "cpu":
        return _DPTrainerCPU(arch, batch, dtype, image_size)
    return _DPTrainer(arch, batch, dtype, list(range(ngpus)), image_size)


def make_trainer(arch: str, batch: int, dtype: torch.dtype, device: torch.device,
                 engine: str = "auto", world: int = 1, rank: int = 0, bucket_mb: float = 32.0,
                 image_size: int = 224, graph: bool = False):
    if engine in ("auto", "native"):
        from .models import native
        if native.supports(arch, dtype):
            return native.NativeTrainer(arch, batch, dtype, device, world, rank, bucket_mb,
                                        image_size, graph=graph)
        if engine == "native":
            raise RuntimeError(f"native engine unavailable for {arch}/{dtype}")
    return _TorchTrainer(arch, batch, dtype, device, world, rank, bucket_mb, image_size)
