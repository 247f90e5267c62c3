"""Step-0 baseline: run the *reference* rocket pipeline on this machine (SURVEY §6 protocol).

The reference tree is copied (git-ignored) into ``_refbase/rocket`` together with
two tiny shims for its uninstallable deps (``adict``, ``termcolor``).  The
pipeline is the ``examples/mnist.py`` topology — LeNet, AdamW, StepLR(100),
CrossEntropy — on synthetic MNIST-shaped data (1×28×28 floats, 10 classes)
served by a map-style ``TensorDataset`` through the reference ``Dataset``
capsule (its ``DataLoader`` + accelerate ``prepare`` path), exactly as a user of
the reference would run it.  Timing: a lowest-priority capsule records
``perf_counter`` deltas between consecutive iterations (the reference syncs the
host every step via ``loss.item()``, so the deltas are true step times).

``--device-data``: the synthetic tensors live on the GPU and the
map-style dataset implements ``__getitems__`` (one ``index_select`` per batch, identity
``collate_fn`` passed through the reference capsule's DataLoader kwargs), so the reference
is not charged for host-side collation of 1024 samples per step.

Usage: ``python bench/reference_baseline.py --steps 60 --warmup 10 [--mp bf16] [--device-data]``
(single process; for N>1 launch under torchrun).  Prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "_refbase"), os.path.join(ROOT, "_refbase", "shims")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch import nn  # noqa: E402


class LeNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 6, 5, padding=2)
        self.conv2 = nn.Conv2d(6, 16, 5)
        self.fc1 = nn.Linear(400, 120)
        self.fc2 = nn.Linear(120, 84)
        self.fc3 = nn.Linear(84, 10)

    def forward(self, x):
        inp = x
        x = F.max_pool2d(F.relu(self.conv1(x[0])), 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = x.flatten(1)
        x = F.relu(self.fc1(x))
        x = F.relu(self.fc2(x))
        return (inp[0], inp[1], self.fc3(x))


class CE(nn.Module):
    def forward(self, b):
        return F.cross_entropy(b[2], b[1])


class _DeviceBatches(torch.utils.data.Dataset):
    """Map-style dataset over GPU tensors with batched fetching (``__getitems__``)."""

    def __init__(self, x, y):
        self.x, self.y = x, y

    def __len__(self):
        return self.x.shape[0]

    def __getitem__(self, i):
        return self.x[i], self.y[i]

    def __getitems__(self, idx):
        i = torch.as_tensor(idx, device=self.x.device)
        return [self.x.index_select(0, i), self.y.index_select(0, i)]


def _identity(batch):
    return batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--mp", default="no")
    ap.add_argument("--device-data", action="store_true")
    args = ap.parse_args()

    import rocket  # the reference package from _refbase

    world = int(os.environ.get("WORLD_SIZE", "1"))
    total = args.steps + args.warmup + 2
    n = total * args.batch * world
    g = torch.Generator().manual_seed(0)
    X = torch.rand(n, 1, 28, 28, generator=g)
    Y = torch.randint(0, 10, (n,), generator=g)
    ds = torch.utils.data.TensorDataset(X, Y)
    loader_kw = {}
    if args.device_data:
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        ds = _DeviceBatches(X.to(dev), Y.to(dev))
        loader_kw["collate_fn"] = _identity

    deltas = []

    class Timer(rocket.Capsule):
        def __init__(self):
            super().__init__(priority=1)
            self.last = None

        def launch(self, attrs=None):
            now = time.perf_counter()
            if self.last is not None:
                deltas.append(now - self.last)
            self.last = now

    net = LeNet()
    opt = torch.optim.AdamW(net.parameters())
    sched = torch.optim.lr_scheduler.StepLR(opt, 100)
    launcher = rocket.Launcher(
        [
            rocket.Looper(
                [
                    rocket.Dataset(ds, batch_size=args.batch, **loader_kw),
                    rocket.Module(net, capsules=[rocket.Loss(objective=CE()), rocket.Optimizer(opt), rocket.Scheduler(sched)]),
                    Timer(),
                ],
                repeats=total,
            )
        ],
        mixed_precision=args.mp,
        num_epochs=1,
        num_procs=world,
    )
    t0 = time.perf_counter()
    launcher.launch()
    wall = time.perf_counter() - t0
    steady = deltas[args.warmup :][: args.steps]
    p50 = statistics.median(steady)
    mean = sum(steady) / len(steady)
    rec = {
        "impl": "reference dsenushkin/rocket (accelerate + torch eager)",
        "data": "GPU-resident, one index_select per batch" if args.device_data else "host TensorDataset + collate",
        "device": torch.cuda.get_device_name(0) if torch.cuda.is_available() else "cpu",
        "mixed_precision": args.mp,
        "world": world,
        "batch_per_rank": args.batch,
        "steps": len(steady),
        "step_ms_p50": p50 * 1e3,
        "step_ms_mean": mean * 1e3,
        "samples_per_s_p50": world * args.batch / p50,
        "samples_per_s_mean": world * args.batch / mean,
        "wall_s": wall,
    }
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
