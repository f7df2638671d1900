import os, sys, socket
sys.path.insert(0, os.getcwd())
import torch, torch.distributed as dist, torch.multiprocessing as mp

def worker(rank, world, port):
    os.environ["PDA_COMM"] = "torch"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", world_size=world, rank=rank)
    torch.cuda.set_device(0); dev = torch.device("cuda", 0)
    from pytorch_distributed_amd.data import SyntheticImageNet
    from pytorch_distributed_amd.models import build_model
    from pytorch_distributed_amd.models.native import NativeResNet
    from pytorch_distributed_amd.ops import native_ops as K
    from pytorch_distributed_amd.parallel import DistributedDataParallel, convert_sync_batchnorm
    torch.manual_seed(0)
    sd = {k: v.clone() for k, v in build_model("resnet18").state_dict().items()}
    nets = []
    for _ in range(2):
        m = NativeResNet(build_model("resnet18"), device=dev, dtype=torch.float32, image_size=64)
        m.load_state_dict(sd); nets.append(m)
    model, full = convert_sync_batchnorm(nets[0]), nets[1]
    ddp = DistributedDataParallel(model, bucket_cap_mb=4.0)
    calls = []
    orig = K._sync_sums
    def wrap(part, G, QC, ws):
        r = orig(part, G, QC, ws); calls.append((G, QC, r[2])); return r
    K._sync_sums = wrap
    gen = model.input_generator(SyntheticImageNet("train", image_size=64))
    x, y = gen(torch.arange(8) + 8 * rank)
    xf, yf = gen(torch.arange(16))
    xx, yy = gen(torch.arange(8) + 8 * rank)
    print(rank, "gen consistent:", torch.equal(xf[8*rank:8*rank+8], x), torch.equal(yf[8*rank:8*rank+8], y), flush=True)
    model.zero_grad_flat()
    out = ddp(x)
    nf = len(calls)
    loss = model.make_criterion()(out, y); loss.backward(); torch.cuda.synchronize()
    print(rank, "sync calls fwd", nf, "bwd", len(calls) - nf, calls[:3], calls[nf:nf+3], flush=True)
    K._sync_sums = orig
    full.zero_grad_flat()
    of = full(xf)
    lf = full.make_criterion()(of, yf); lf.backward(); torch.cuda.synchronize()
    lt = torch.tensor([loss.item()]); dist.all_reduce(lt)
    print(rank, "loss mean", lt.item() / 2, "full", lf.item(), "logits err", ((out - of[8*rank:8*rank+8]).norm() / of.norm()).item(), flush=True)
    sdg = model.state_dict(); fdg = full.state_dict()
    # gradients by name
    g1 = dict((n, p.grad) for n, p in model.named_parameters() if p.grad is not None)
    g2 = dict((n, p.grad) for n, p in full.named_parameters() if p.grad is not None)
    if rank == 0:   # torch fp32 oracle on the same 16 images
        ds = SyntheticImageNet("train", image_size=64)
        xt, yt = ds.batch(torch.arange(16), device=dev)
        tm = build_model("resnet18").to(dev)
        tm.load_state_dict(sd)
        torch.nn.functional.cross_entropy(tm(xt.float()), yt).backward()
        g3 = dict((n, p.grad) for n, p in tm.named_parameters())
        for n in list(g1):
            if n in g3:
                e1 = ((g1[n] - g3[n]).norm() / (g3[n].norm() + 1e-30)).item()
                e2 = ((g2[n] - g3[n]).norm() / (g3[n].norm() + 1e-30)).item()
                if max(e1, e2) > 1e-4:
                    print("vs torch", n, "sync", e1, "full", e2, flush=True)
        for n in list(g1):
            if n in g2:
                e = ((g1[n] - g2[n]).norm() / (g2[n].norm() + 1e-30)).item()
                if e > 1e-4:
                    print(rank, n, e, flush=True)
    dist.destroy_process_group()

if __name__ == "__main__":
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(worker, args=(2, port), nprocs=2)
