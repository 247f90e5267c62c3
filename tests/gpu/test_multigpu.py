"""Multi-GPU data parallel over real RCCL/xGMI — runs itself whenever the box has >= 2 devices
(skipped on the single-GPU box; the ranks-on-one-GPU rehearsals are ``test_ddp_graph.py``).

Two ranks, one per GPU, default transport (native RCCL communicator + side-stream reducer,
``capture_mode == "overlap"``), ResNet-18 with BatchNorm:

1. reducer correctness: one captured forward/backward per rank on its half of a batch (BatchNorm
   in eval mode so the loss is a per-sample mean), replayed; the all-reduced gradients must equal
   the world-1 gradients of the concatenated batch, computed on every rank from the same weights;
2. a captured training run through the capsule stack (``Launcher → Looper → Module``, overlapped
   all-reduce inside the step graph, rank-0 BatchNorm buffer broadcast): the replicas must end
   bit-identical (cross-rank weight checksums) and the reported loss is the cross-rank mean.

Reference anchors: ``/root/reference/rocket/core/module.py:103-106`` (DDP prepare),
``/root/reference/rocket/core/loss.py:95,119`` (gathered loss, reducer-driven backward).
"""

import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _checksum(net):
    s0 = s1 = 0.0
    off = 0
    for p in net.parameters():
        v = p.detach().reshape(-1).double()
        w = (torch.arange(v.numel(), device=v.device, dtype=torch.float64) + off).remainder_(97.0)
        s0 += float(v.sum())
        s1 += float((v * w).sum())
        off += v.numel()
    return [s0, s1]


def _worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROCKET_P2P="0",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    import rocket_amd as rocket
    from rocket_amd.core.capsule import Capsule
    from rocket_amd.models import CrossEntropy, resnet18
    from rocket_amd.ops.optim import FusedSGD
    from rocket_amd.parallel.ddp import DataParallel
    from rocket_amd.parallel.rccl import RcclComm
    from rocket_amd.runtime import comm

    ctx = comm.init()
    dev = ctx.device
    assert dev.index == rank
    res = {"rank": rank, "device": str(dev), "backend": ctx.backend}

    # ---- 1. reducer correctness vs the world-1 full batch -------------------------------------
    torch.manual_seed(0)
    net = resnet18(10).to(dev).to(memory_format=torch.channels_last).eval()
    g = torch.Generator(device=dev).manual_seed(7)
    bs = 32
    x = torch.rand(world * bs, 3, 32, 32, generator=g, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (world * bs,), generator=g, device=dev)
    ref_net = resnet18(10).to(dev).to(memory_format=torch.channels_last).eval()
    ref_net.load_state_dict(net.state_dict())
    with torch.autocast("cuda", dtype=torch.bfloat16):
        torch.nn.functional.cross_entropy(ref_net(x).float(), y).backward()
    ref = [p.grad.detach().float().clone() for p in ref_net.parameters()]

    rc = RcclComm(dev)
    dp = DataParallel(net, comm=rc)
    res["mode"] = dp.capture_mode
    xs, ys = x[rank * bs:(rank + 1) * bs].clone(), y[rank * bs:(rank + 1) * bs].clone()

    def step():
        dp.zero_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            torch.nn.functional.cross_entropy(dp(xs).float(), ys).backward()

    step()  # eager: grad views, workspaces
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        step()
    graph.replay()
    torch.cuda.synchronize()
    errs = []
    for p, r in zip(net.parameters(), ref):
        errs.append(float((p.grad.float() - r).norm() / r.norm().clamp_min(1e-12)))
    res["grad_rel_err_max"] = max(errs)
    rc.close()

    # ---- 2. captured training run through the capsule stack -----------------------------------
    class Rec(Capsule):
        def __init__(self):
            super().__init__(priority=10)
            self.losses = []

        def launch(self, attrs=None):
            if attrs.looper.state.loss is not None:
                self.losses.append(attrs.looper.state.loss)

    torch.manual_seed(0)
    net2 = resnet18(10).to(memory_format=torch.channels_last)
    opt = FusedSGD(net2.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-5)
    g2 = torch.Generator(device=dev).manual_seed(11 + rank)
    x2 = torch.rand(bs * 10, 3, 32, 32, generator=g2, device=dev)
    y2 = torch.randint(0, 10, (bs * 10,), generator=g2, device=dev)
    rec = Rec()
    mod = rocket.Module(net2, [rocket.Loss(CrossEntropy(fused=True)), rocket.Optimizer(opt)], capture=True,
                        warmup=1)
    rocket.Launcher(
        [rocket.Looper([rocket.Dataset(rocket.DeviceTensorDataset(x2, y2, pre_sharded=True), batch_size=bs), mod,
                        rec], repeats=10, progress=False)],
        mixed_precision="bf16",
        num_procs=world,
        destroy_process_group_after_launch=False,
    ).launch()
    torch.cuda.synchronize()
    res.update(mode2=mod._module.capture_mode, transport=("native" if mod._module._native is not None else "other"),
               replays=mod._graphs.replays, parts=mod._graphs.parts, losses=[float(v) for v in rec.losses],
               checksum=_checksum(net2))
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as fh:
        json.dump(res, fh)
    comm.barrier()
    comm.shutdown()


@pytest.mark.skipif(torch.cuda.device_count() < WORLD, reason="needs >= 2 GPUs (runs on a multi-GPU box)")
def test_two_gpu_native_rccl(tmp_path):
    mp.start_processes(_worker, args=(WORLD, _free_port(), str(tmp_path)), nprocs=WORLD, start_method="spawn",
                       join=True)
    r = [json.load(open(tmp_path / f"r{i}.json")) for i in range(WORLD)]
    for i, x in enumerate(r):
        assert x["device"] == f"cuda:{i}" and x["backend"] == "nccl", x
        assert x["mode"] == "overlap" and x["mode2"] == "overlap" and x["transport"] == "native", x
        # bf16 autocast: the two-half all-reduced gradients and the full batch round differently
        assert x["grad_rel_err_max"] < 2e-2, x["grad_rel_err_max"]
        assert x["replays"] > 0 and x["parts"] == 1, x
    assert r[0]["checksum"] == r[1]["checksum"], (r[0]["checksum"], r[1]["checksum"])
    assert r[0]["losses"] == r[1]["losses"]
