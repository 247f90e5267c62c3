"""MNIST LeNet training with the rocket_amd capsule tree (the reference ``examples/mnist.py`` topology).

    python examples/mnist.py                      # 1 GPU (or CPU), synthetic MNIST-shaped data
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 examples/mnist.py
    python examples/mnist.py --data /path/to/mnist   # raw idx files (train-images-idx3-ubyte, ...)

Tree (reference ``examples/mnist.py:89-106``, with the evaluation looper the
reference's ``Meter``/``Metric`` classes exist for):

    Launcher ─ Looper(train) ─ Dataset, Module(LeNet) ─ {Loss, Optimizer, Scheduler}, Tracker, Checkpointer
             └ Looper(eval, grad off, every epoch) ─ Dataset, Module(LeNet), Meter ─ Accuracy

There is no network here, so real MNIST is only used when ``--data`` points at
the four raw idx files; otherwise the data are random images/labels of the same
shape (accuracy then stays at chance — the example exercises the machinery).
"""

from __future__ import annotations

import argparse
import gzip
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import rocket_amd as rocket  # noqa: E402
from rocket_amd.models import CrossEntropy, LeNet, synthetic_mnist  # noqa: E402


class Accuracy(rocket.Metric):
    """Running top-1 accuracy over the (cross-rank gathered) eval batches."""

    def __init__(self, priority: int = 1000) -> None:
        super().__init__(priority=priority)
        self.positive = 0
        self.total = 0

    def launch(self, attrs=None):
        gt, logits = attrs.batch[1], attrs.batch[2]
        self.total += gt.numel()
        self.positive += int((logits.argmax(1) == gt).sum())
        attrs.looper.state.accuracy = self.positive / max(self.total, 1)
        if attrs.tracker is not None:
            attrs.tracker.scalars.append(rocket.Attributes(step=self._step, data={"eval.accuracy": attrs.looper.state.accuracy}))

    def reset(self, attrs=None):
        self.positive = 0
        self.total = 0


def _idx(path: str) -> np.ndarray:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as fh:
        data = fh.read()
    ndim = data[3]
    dims = [int.from_bytes(data[4 + 4 * i : 8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def load_mnist(root: str, train: bool):
    stem = "train" if train else "t10k"
    for suffix in ("", ".gz"):
        xi = os.path.join(root, f"{stem}-images-idx3-ubyte{suffix}")
        yi = os.path.join(root, f"{stem}-labels-idx1-ubyte{suffix}")
        if os.path.exists(xi) and os.path.exists(yi):
            x = torch.from_numpy(_idx(xi).copy()).float().div_(255.0).unsqueeze(1)
            y = torch.from_numpy(_idx(yi).astype(np.int64))
            return x, y
    raise FileNotFoundError(f"no MNIST idx files under {root}")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=None, help="directory with the raw MNIST idx files")
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--ga", type=int, default=1, help="gradient accumulation steps")
    ap.add_argument("--tag", default="mnist")
    ap.add_argument("--logs", default="./logs")
    ap.add_argument("--resume", default=None)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--train-size", type=int, default=60000, help="synthetic training samples")
    ap.add_argument("--test-size", type=int, default=10000, help="synthetic evaluation samples")
    ap.add_argument("--save-every", type=int, default=50, help="Checkpointer cadence (iterations)")
    ap.add_argument("--capture", type=int, default=None, help="HIP-graph capture of the train step (default: on GPUs)")
    args = ap.parse_args()

    from rocket_amd.runtime import comm

    ctx = comm.init(cpu=args.cpu)
    dev = ctx.device
    if args.data:
        xtr, ytr = load_mnist(args.data, True)
        xte, yte = load_mnist(args.data, False)
    else:
        xtr, ytr = synthetic_mnist(args.train_size, seed=0)
        xte, yte = synthetic_mnist(args.test_size, seed=1)
    # the whole dataset fits in HBM many times over: keep it resident, gather batches on-device
    train = rocket.DeviceTensorDataset(xtr.to(dev), ytr.to(dev))
    test = rocket.DeviceTensorDataset(xte.to(dev), yte.to(dev))

    net = LeNet()
    if dev.type == "cuda":
        from rocket_amd.ops.optim import FusedAdamW

        opt = FusedAdamW(net.parameters())
    else:
        opt = torch.optim.AdamW(net.parameters())
    sched = torch.optim.lr_scheduler.StepLR(opt, 100)

    launcher = rocket.Launcher(
        [
            rocket.Looper(
                [
                    rocket.Dataset(train, batch_size=args.batch, shuffle=True),
                    rocket.Module(net, [rocket.Loss(CrossEntropy()), rocket.Optimizer(opt), rocket.Scheduler(sched)],
                                  capture=dev.type == "cuda" if args.capture is None else bool(args.capture)),
                    rocket.Tracker(backend="jsonl"),
                    rocket.Checkpointer(save_every=args.save_every),
                ],
                tag="train",
            ),
            rocket.Looper(
                [
                    rocket.Dataset(test, batch_size=args.batch),
                    rocket.Module(net),
                    rocket.Meter([Accuracy()], keys=[1, 2]),
                    rocket.Tracker(backend="jsonl"),
                ],
                tag="eval",
                grad_enabled=False,
            ),
        ],
        tag=args.tag,
        logging_dir=args.logs,
        mixed_precision="bf16" if dev.type == "cuda" else None,
        gradient_accumulation_steps=args.ga,
        num_epochs=args.epochs,
        statefull=True,
        cpu=args.cpu,
    )
    if args.resume:
        launcher.resume(args.resume)
    launcher.launch()
    return 0


if __name__ == "__main__":
    sys.exit(main())
