"""Headline benchmark: whole-node samples/s of the MNIST ConvNet training step (BASELINE.json).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` — for N>1
launched under ``torch.distributed.run`` (one rank per GPU, RCCL).  W untimed
steps, then exactly K steps bracketed by barrier + device sync on both sides;
the elapsed time is the MAX over ranks; rank 0 prints ONE JSON line.

What runs: the reference ``examples/mnist.py`` topology built from this
framework's capsules — ``Launcher → Looper → {Dataset, Module(LeNet) →
{Loss(CrossEntropy), Optimizer(AdamW), Scheduler(StepLR(100))}, StepTimer}`` —
bf16 mixed precision, per-GPU batch 1024 (weak scaling: global batch 1024·N),
synthetic MNIST-shaped data (random 1×28×28 images / labels, each rank generating
and holding only its own shard in HBM, reshuffled every epoch on-device),
random-init weights.  Every timed step
does the full work: batch gather, forward, loss, backward, gradient all-reduce
(N>1), AdamW update, LR schedule, loss accounting.

Extra flags (for A/B runs): ``--impl torch`` uses stock PyTorch ops instead of
the fused HIP kernels; ``--no-graph`` disables HIP-graph capture of the step.

``--model`` selects the other BASELINE configs with the same harness:
``resnet18`` (CIFAR-10 shape 3×32×32, 10 classes, per-GPU batch 256), ``resnet50``
(ImageNet shape 3×224×224, 1000 classes, batch 256) and ``vit_b16`` (3×224×224,
1000 classes, batch 128) — all bf16 autocast, DDP over RCCL for N>1, SGD(momentum)
for the ResNets and AdamW for ViT, synthetic HBM-resident data (stored bf16).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

# MIOpen: benchmark-based solution search at first use (done in the untimed warm-up).  The
# heuristic-only FAST mode picks ~50x slower NHWC bf16 kernels (bench/conv_probe.py).
os.environ.setdefault("MIOPEN_FIND_MODE", "NORMAL")

BASELINE_METRIC = "samples/sec (whole node) MNIST ConvNet at 1/2/4/8 MI355X; step-time p50"
REFERENCE_CPU_SAMPLES_PER_S = 27460.0  # reference pipeline on this container's 8 CPUs

MODELS = {
    # name: (per-GPU batch, input shape, classes, description)
    "lenet": (1024, (1, 28, 28), 10, "LeNet-5 MNIST 2-conv CNN (reference examples/mnist.py)"),
    "resnet18": (256, (3, 32, 32), 10, "ResNet-18 CIFAR-10 shape"),
    "resnet50": (256, (3, 224, 224), 1000, "ResNet-50 ImageNet shape"),
    "vit_b16": (128, (3, 224, 224), 1000, "ViT-Base/16 ImageNet shape"),
}


def _baseline_value(n_gpus: int):
    """Reference number to divide by: 1-GPU MI355X reference × N (ideal weak scaling)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench", "reference_mi355x.json")
    try:
        with open(path) as fh:
            b = json.load(fh)
        per_gpu = b.get("reference_mi355x_1gpu_bf16_samples_per_s")
        if per_gpu:
            return float(per_gpu) * n_gpus
    except Exception:
        pass
    return None


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(n: int) -> int:
    """``python bench.py --gpus N`` without a launcher: start N ranks (one per GPU) under
    ``torch.distributed.run`` as a CHILD process and exit with its status.  Runs before anything
    touches the GPU (this process never initialises HIP, and never execs)."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def _weight_checksum(net) -> list:
    """Two float64 sums over every parameter (plain and position-weighted): equal on every rank iff
    the replicas ended identical (DP applies the same averaged update everywhere)."""
    s0 = torch.zeros((), dtype=torch.float64, device=next(net.parameters()).device)
    s1 = torch.zeros_like(s0)
    off = 0
    for p in net.parameters():
        v = p.detach().reshape(-1).to(torch.float64)
        w = (torch.arange(v.numel(), device=v.device, dtype=torch.float64) + off).remainder_(97.0)
        s0 += v.sum()
        s1 += (v * w).sum()
        off += v.numel()
    return [s0.item(), s1.item()]


def _dp_record(mod, net, ctx, comm) -> dict:
    """What ran: the data-parallel transport and capture mode, bucket sizes, how many ranks the
    communicator spans, the capture counters, and whether the replicas ended bit-identical
    (cross-rank weight checksums, compared on every rank)."""
    from rocket_amd.parallel.ddp import DataParallel

    rep = getattr(mod, "_module", None)
    rec = {"world": ctx.world_size, "backend": ctx.backend}
    if isinstance(rep, DataParallel):
        c = rep.comm
        if rep._p2p is not None:
            transport = "p2p-xgmi"
        elif rep._native is not None:
            transport = "native-rccl"
        else:
            transport = "torch-" + str(ctx.backend)
        rec.update(transport=transport, capture_mode=rep.capture_mode,
                   bucket_mb=[round(b.flat.numel() * b.flat.element_size() / 2**20, 4) for b in rep.buckets],
                   comm_ranks=int(getattr(c, "world", ctx.world_size)))
    else:
        rec.update(transport="none", capture_mode=None, bucket_mb=[], comm_ranks=1)
    g = getattr(mod, "_graphs", None)
    if g is not None:
        rec["graph"] = {"captures": g.captures, "replays": g.replays, "parts": g.parts,
                        "launch_lists": g.launch_lists}
    sums = _weight_checksum(net)
    parts = comm.all_gather_object(sums) if ctx.world_size > 1 else [sums]
    rec["weight_checksum"] = sums
    rec["replicas_identical"] = all(p == parts[0] for p in parts)
    return rec


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: LeNet 1000 timed steps (~60 ms: one host/runtime hiccup must not dominate the
    # mean of a 58 us step) after 50 warmup; the large models 200 / 20
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--model", choices=sorted(MODELS), default="lenet")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default per model)")
    ap.add_argument("--impl", choices=["fused", "torch"], default="fused")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--graph", action="store_true", help="force HIP-graph capture for the non-LeNet models")
    ap.add_argument("--mp", default="bf16")
    ap.add_argument("--cpu", action="store_true")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _spawn(args.gpus)
    if args.steps is None:
        args.steps = 1000 if args.model == "lenet" else 200
    if args.warmup is None:
        args.warmup = 50 if args.model == "lenet" else 20

    import rocket_amd as rocket
    from rocket_amd.models import CrossEntropy, LeNet
    from rocket_amd.runtime import comm
    from rocket_amd.runtime.data import DeviceTensorDataset
    from rocket_amd.runtime.profiling import StepTimer

    ctx = comm.init(cpu=args.cpu)
    world = ctx.world_size
    if world != args.gpus and ctx.rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev = ctx.device
    on_gpu = dev.type == "cuda"
    fused = on_gpu and args.impl == "fused"
    from rocket_amd import ops

    ops.set_fused(fused)
    if fused:
        ops.require_native()

    bs_default, in_shape, classes, desc = MODELS[args.model]
    args.batch = args.batch or bs_default
    total_iters = args.warmup + args.steps
    # each rank generates only its own shard (weak scaling: per-rank data is fixed as N grows);
    # one epoch covers the whole run
    n = (total_iters + 1) * args.batch
    g = torch.Generator(device=dev).manual_seed(1234 + ctx.rank)
    img_dtype = torch.float32 if args.model == "lenet" else torch.bfloat16
    x = torch.rand((n,) + in_shape, generator=g, device=dev, dtype=img_dtype)
    y = torch.randint(0, classes, (n,), generator=g, device=dev)
    data = DeviceTensorDataset(x, y, pre_sharded=True)

    torch.manual_seed(0)
    if args.model == "lenet":
        net = LeNet(fused=fused)
    else:
        from rocket_amd import models

        net = {"resnet18": lambda: models.resnet18(classes), "resnet50": lambda: models.resnet50(classes),
               "vit_b16": lambda: models.vit_b16(classes)}[args.model]()
        if on_gpu and args.model.startswith("resnet"):  # NHWC convs; ViT's patch embedding is a GEMM
            net = net.to(memory_format=torch.channels_last)
    if fused:
        from rocket_amd.ops.optim import FusedAdamW, FusedSGD

        if args.model.startswith("resnet"):
            opt = FusedSGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
        else:
            opt = FusedAdamW(net.parameters())
    elif args.model.startswith("resnet"):
        opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=True)
    else:
        opt = torch.optim.AdamW(net.parameters(), foreach=True)
    sched = torch.optim.lr_scheduler.StepLR(opt, 100)
    # step-time p50 from timing events every `stride` steps (an event per ~80 us LeNet step would
    # itself cost ~5 us of queue time); the headline number is the barrier/sync-bracketed wall time
    stride = max(10, args.steps // 50) if args.model == "lenet" else 1
    timer = StepTimer(warmup=args.warmup, steps=args.steps, stride=stride)
    launcher = rocket.Launcher(
        [
            rocket.Looper(
                [
                    rocket.Dataset(data, batch_size=args.batch, shuffle=True, drop_last=True),
                    mod := rocket.Module(
                        net,
                        [rocket.Loss(CrossEntropy(fused=fused)), rocket.Optimizer(opt), rocket.Scheduler(sched)],
                        # every model's step is captured and replayed (ResNet-18: host 3.9 -> 0.56 ms/step,
                        # ResNet-50 10.1 -> 1.4, ViT-B/16 11.4 -> 1.6; profiles/r2_graph_models.jsonl)
                        capture=fused and not args.no_graph,
                        warmup=1,  # one eager step primes optimizer state; every capture then lands in it
                    ),
                    timer,
                ],
                repeats=total_iters,
                progress=False,
            )
        ],
        mixed_precision=args.mp if on_gpu else None,
        num_procs=world,
        num_epochs=1,
        destroy_process_group_after_launch=False,
        cpu=args.cpu,
    )
    step_trace = None
    if os.environ.get("ROCKET_LENET_TRACE") and args.model == "lenet" and on_gpu and fused:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench"))
        from lenet_timeline import StepTrace

        step_trace = StepTrace(args.batch)  # installed before capture: every replay stamps
    prof_path = os.environ.get("ROCKET_BENCH_PROFILE")  # host-side cProfile of the run (diagnostics)
    prof = None
    if prof_path:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    launcher.launch()
    wall = time.perf_counter() - t0
    if prof is not None:
        prof.disable()
        prof.dump_stats(f"{prof_path}.{ctx.rank}")
    if step_trace is not None:
        with open(os.environ["ROCKET_LENET_TRACE"], "w") as fh:
            json.dump(step_trace.report(), fh)

    elapsed = timer.elapsed
    summ = timer.summary()
    dp = _dp_record(mod, net, ctx, comm)
    stats = torch.tensor([elapsed, summ.get("step_ms_p50", 0.0)], dtype=torch.float64)
    if world > 1:
        parts = comm.all_gather_object(stats.tolist())
        elapsed = max(p[0] for p in parts)
        p50 = max(p[1] for p in parts)
    else:
        p50 = summ.get("step_ms_p50", 0.0)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * args.batch * args.steps / elapsed
    base = None
    if args.model == "lenet":
        # CPU: BASELINE config #1 (reference on CPU, W=1: 27,460 samples/s p50)
        base = _baseline_value(world) if on_gpu else REFERENCE_CPU_SAMPLES_PER_S * world
    if ctx.rank == 0:
        rec = {
            "metric": BASELINE_METRIC if args.model == "lenet" else f"samples/sec (whole node) {desc}; step-time p50",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "step_ms_p50": round(p50, 4),
            # host enqueue interval (GPU-paced once the device queue is full) and the unpaced host
            # cost of issuing one step from an empty queue (runtime/profiling.py StepTimer)
            "host_ms_p50": round(summ.get("host_ms_p50", 0.0), 4),
            "host_issue_ms": round(summ.get("host_issue_ms", 0.0), 4),
            "step_ms_max": round(summ.get("step_ms_max", 0.0), 4),  # rank 0, worst timing group
            "step_ms_max_at": summ.get("step_ms_max_at"),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base, 3) if base else None,
            "dtype": args.mp if (args.mp in ("bf16", "fp16") and on_gpu) else "fp32",
            "data": f"synthetic (random {'x'.join(map(str, in_shape))} images / {classes}-class labels resident in "
            f"{'HBM' if on_gpu else 'host memory'}, "
            "random-init weights)",
            "config": {
                "model": desc,
                "global_batch": args.batch * world,
                "per_gpu_batch": args.batch,
                "seq_len": None,
                "input_shape": list(in_shape),
                "optimizer": ("SGD(momentum)" if args.model.startswith("resnet") else "AdamW") + " + StepLR(100)",
                "parallelism": f"dp{world}",
                "impl": ("fused-hip" + ("" if args.no_graph else "+hipgraph"))
                if fused else "torch-eager",
                **({"gemm_route": __import__("rocket_amd.ops.mlinear", fromlist=["MODE"]).MODE}
                   if args.model == "vit_b16" and fused else {}),
            },
            "wall_s": round(wall, 2),
            "dp": dp,
        }
        print(json.dumps(rec), flush=True)
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
