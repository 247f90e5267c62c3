"""Data-parallel captured steps vs eager, 2 ranks on one GPU.

The ranks share ``cuda:0`` and their host group is gloo (``ROCKET_DIST_BACKEND=gloo``): this
rehearses the multi-GPU code paths on the single-GPU box, one per ``DataParallel.capture_mode`` —

* ``split`` (``ROCKET_P2P=0``, torch.distributed transport): graph A -> host-issued bucket
  all-reduce -> graph B;
* ``inline`` (``ROCKET_P2P=force``, LeNet): the one-shot IPC all-reduce kernel captured INSIDE one
  graph per step;
* ``overlap`` (``ROCKET_DP_COMM=p2p``): every bucket's all-reduce forked onto a side stream from
  the gradient hooks during capture and joined before the optimizer — ONE graph whose reduction
  branches run alongside the rest of backward (the structure the native RCCL reducer captures on
  real multi-GPU nodes), with the rank-0 BatchNorm buffer broadcast captured in the forward —

plus side-channel loss averaging in all of them, for LeNet and a BatchNorm ResNet-18; and the
overlap capture failing on ONE rank (``overlap_fail``: rank 1's first overlapped capture raises after
it has claimed the pending batch and set the fused optimizer's step flags): both ranks must drop to
split mode together, with the side effects of the discarded capture undone (runtime/graphs.py
``_capture``), and train exactly like the eager run.
"""

import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_ENV = {"split": dict(ROCKET_P2P="0"), "inline": dict(ROCKET_P2P="force"),
        "overlap": dict(ROCKET_P2P="0", ROCKET_DP_COMM="p2p"),
        "overlap_fail": dict(ROCKET_P2P="0", ROCKET_DP_COMM="p2p")}


def _inject_capture_failure(rank, injected):
    """Rank 1's first overlapped capture runs to the end (every side effect of a capture happens) and
    then raises, as a rank-local capture error would."""
    from rocket_amd.runtime import graphs as G

    orig = G.StepGraphs._capture_inner

    def capture_inner(self, attrs, tens, pend):
        v = orig(self, attrs, tens, pend)
        rep = self._replica()
        if rank == 1 and not injected and rep is not None and rep.capture_mode == "overlap" and v.sync:
            injected.append(1)
            raise RuntimeError("injected overlapped-capture failure")
        return v

    G.StepGraphs._capture_inner = capture_inner


def _worker(rank, world, port, out_dir, mode, model):
    if os.environ.get("ROCKET_TEST_HANG_DUMP"):  # debugging: dump the worker's stacks and exit on a hang
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["ROCKET_TEST_HANG_DUMP"]), exit=True)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROCKET_DIST_BACKEND="gloo", **_ENV[mode])
    import rocket_amd as rocket
    from rocket_amd.core.capsule import Capsule
    from rocket_amd.models import CrossEntropy, LeNet, resnet18
    from rocket_amd.ops.optim import FusedAdamW, FusedSGD

    class Rec(Capsule):
        def __init__(self):
            super().__init__(priority=10)
            self.losses = []

        def launch(self, attrs=None):
            if attrs.looper.state.loss is not None:
                self.losses.append(attrs.looper.state.loss)

    injected = []
    if mode == "overlap_fail":
        _inject_capture_failure(rank, injected)
    res = {}
    from rocket_amd.core import objectives as _obj

    variants = [(False, True), (True, True)]
    if mode == "inline":
        variants.append((True, False))  # captured, the all-reduce NOT fused with the AdamW update
    for capture, fuse in variants:
        _obj._OPT_EPILOGUE = fuse
        dev = torch.device("cuda", 0)
        g = torch.Generator(device=dev).manual_seed(3)
        bs = 128 if model == "lenet" else 32
        shape = (1, 28, 28) if model == "lenet" else (3, 32, 32)
        x = torch.rand((bs * 2 * 12,) + shape, generator=g, device=dev)
        y = torch.randint(0, 10, (bs * 2 * 12,), generator=g, device=dev)
        torch.manual_seed(0)
        if model == "lenet":
            net = LeNet(fused=True)
            opt = FusedAdamW(net.parameters(), lr=1e-2)
        else:
            net = resnet18(10).to(memory_format=torch.channels_last)
            opt = FusedSGD(net.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-5)
        rec = Rec()
        mod = rocket.Module(net, [rocket.Loss(CrossEntropy(fused=True)), rocket.Optimizer(opt)], capture=capture,
                            warmup=2)
        rocket.Launcher(
            [rocket.Looper([rocket.Dataset(rocket.DeviceTensorDataset(x, y), batch_size=bs), mod, rec],
                           repeats=12, progress=False)],
            logging_dir=os.path.join(out_dir, f"logs{int(capture)}"),
            mixed_precision="bf16",
            gradient_accumulation_steps=2,
            num_procs=world,
            destroy_process_group_after_launch=False,
        ).launch()
        torch.cuda.synchronize()
        rep = mod._module
        res[str(capture) if fuse else "unfused"] = dict(
            fused=getattr(rep, "fused_updates", 0),
            loss_folds=getattr(rep, "loss_folds", 0),
            losses=[float(v) for v in rec.losses],
            w=float(sum(p.detach().double().sum() for p in net.parameters())),
            bufs=float(sum(b.detach().double().sum() for b in net.buffers())),
            replays=(mod._graphs.replays if mod._graphs is not None else 0),
            sync_captures=(mod._graphs.sync_captures if mod._graphs is not None else 0),
            parts=(mod._graphs.parts if mod._graphs is not None else 0),
            mode=getattr(mod._module, "capture_mode", None),
            reason=(mod._graphs.disabled_reason if mod._graphs is not None else None),
            injected=len(injected),
        )
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as fh:
        json.dump(res, fh)
    import torch.distributed as dist

    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,model", [("split", "lenet"), ("inline", "lenet"), ("overlap", "lenet"),
                                        ("split", "resnet18"), ("overlap", "resnet18"),
                                        ("overlap_fail", "lenet")])
def test_ddp_graph_two_ranks(tmp_path, mode, model):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path), mode, model), nprocs=2, start_method="spawn",
                       join=True)
    r = [json.load(open(tmp_path / f"r{i}.json")) for i in range(2)]
    # BatchNorm-trained ResNet steps amplify bf16 rounding differences between eager and captured
    # kernels more than LeNet's: looser bounds there
    tol_l, tol_w = (2e-3, 5e-3) if model == "lenet" else (2e-2, 2e-2)
    for rank in range(2):
        e, g = r[rank]["False"], r[rank]["True"]
        assert g["replays"] > 0 and g["reason"] == "released", g
        if mode == "overlap_fail":
            # both ranks dropped to split mode together; only rank 1 failed its capture
            assert g["mode"] == "split" and g["parts"] == 2, g
            assert g["injected"] == (1 if rank == 1 else 0), g
        else:
            assert g["mode"] == mode and g["parts"] == (2 if mode == "split" else 1), g
        assert len(e["losses"]) == len(g["losses"]) > 0
        for a, b in zip(e["losses"], g["losses"]):
            assert abs(a - b) <= tol_l * max(1.0, abs(a)), (e["losses"], g["losses"])
        # weight sums: eager (separate CE launch, fp32 d(logits)) and captured (CE fused into the
        # backward launch) round differently; Adam at lr 1e-2 turns near-zero gradients' rounding
        # differences into +-lr steps, so this checksum gets a looser bound than the losses
        assert abs(e["w"] - g["w"]) <= tol_w * max(1.0, abs(e["w"])), (e["w"], g["w"])
    # replicas stay identical across ranks (weights AND rank-0-broadcast buffers), and the
    # reported loss is the cross-rank mean
    assert abs(r[0]["True"]["w"] - r[1]["True"]["w"]) < 1e-6 * max(1.0, abs(r[0]["True"]["w"]))
    assert r[0]["True"]["losses"] == pytest.approx(r[1]["True"]["losses"], rel=1e-6)
    if mode == "inline":
        # the P2P reduce applied the AdamW update in its write-back on every captured sync step,
        # and that equals all-reduce -> optimizer launch bit for bit (same sums, same update math)
        for rank in range(2):
            g, u = r[rank]["True"], r[rank]["unfused"]
            # every captured sync step (each loader-ring slot is its own capture) takes the fused path
            assert g["fused"] > 0 and g["fused"] == g["sync_captures"] and u["fused"] == 0, (g, u)
            # ... and its all-reduce also did the loss-ring bookkeeping (no separate launch), fused or not
            assert g["loss_folds"] == g["sync_captures"] and u["loss_folds"] == u["sync_captures"] > 0, (g, u)
            assert g["w"] == u["w"] and g["losses"] == u["losses"], (g, u)
    if model != "lenet":
        # BatchNorm statistics are rank 0's at the start of every synchronised forward (torch DDP's
        # broadcast_buffers semantics), then each rank folds in its own batch: after the last step
        # they differ only by that one local momentum update (momentum 0.1)
        b0, b1 = r[0]["True"]["bufs"], r[1]["True"]["bufs"]
        assert abs(b0 - b1) < 2e-3 * max(1.0, abs(b0)), (b0, b1)
