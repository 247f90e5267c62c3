"""Multi-process (gloo, W=2) checks of the data-parallel path on CPU.

* the bucketed reducer yields the full-batch mean gradient on every rank;
* a W=2 Launcher run equals a W=1 run over the same global batches;
* ``gather_for_metrics`` drops the wrap-around padding of the last batch.
"""

import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))


def _run(fn, world, *args):
    port = _port()
    mp.start_processes(fn, args=(world, port) + args, nprocs=world, start_method="spawn", join=True)


# ---------------------------------------------------------------- reducer
def _reducer_worker(rank, world, port, out):
    _env(rank, world, port)
    from rocket_amd.runtime import comm
    from rocket_amd.parallel.ddp import DataParallel

    comm.init(cpu=True)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    if rank == 1:  # different init on rank 1: construction must broadcast rank 0's weights
        with torch.no_grad():
            for p in net.parameters():
                p.add_(1.0)
    dp = DataParallel(net, first_bucket_mb=1e-4, bucket_cap_mb=1e-3)  # several buckets
    x = torch.randn(2 * world, 8, generator=torch.Generator().manual_seed(1))
    mine = x[rank * 2 : rank * 2 + 2]
    for _ in range(2):  # second pass checks re-arming and no_sync accumulation
        dp.zero_grad()
        with dp.no_sync():
            dp(mine).pow(2).mean().backward()
        dp(mine).pow(2).mean().backward()
    grads = [p.grad.tolist() for p in net.parameters()]
    with open(os.path.join(out, f"g{rank}.json"), "w") as fh:
        json.dump(dict(grads=grads, nb=len(dp.buckets)), fh)
    comm.shutdown()


def test_reducer_matches_full_batch(tmp_path):
    _run(_reducer_worker, 2, str(tmp_path))
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    x = torch.randn(4, 8, generator=torch.Generator().manual_seed(1))
    # per-rank loss is a mean over 2 rows, gradients averaged over ranks, 2 accumulated backward passes
    loss = 2 * sum(net(x[r * 2 : r * 2 + 2]).pow(2).mean() for r in range(2)) / 2
    loss.backward()
    ref = [p.grad for p in net.parameters()]
    for r in range(2):
        got = json.load(open(tmp_path / f"g{r}.json"))
        assert got["nb"] > 1
        for g, e in zip(got["grads"], ref):
            torch.testing.assert_close(torch.tensor(g), e, rtol=1e-5, atol=1e-6)


# --------------------------------------------------------- launcher W=2 == W=1
def _train(world, out_file, bs):
    import rocket_amd as rocket

    torch.manual_seed(0)
    n = 24
    x = torch.randn(n, 6, generator=torch.Generator().manual_seed(5))
    y = torch.randint(0, 3, (n,), generator=torch.Generator().manual_seed(6))
    data = [(x[i], y[i]) for i in range(n)]
    net = torch.nn.Linear(6, 3)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = net

        def forward(self, b):
            return (self.lin(b[0]), b[1])

    class Obj(torch.nn.Module):
        def forward(self, b):
            return torch.nn.functional.cross_entropy(b[0], b[1])

    losses = []

    class Rec(rocket.Capsule):
        def __init__(self):
            super().__init__(priority=10)

        def launch(self, attrs=None):
            losses.append(float(attrs.looper.state.loss))

    opt = torch.optim.SGD(net.parameters(), lr=0.5)
    rocket.Launcher(
        [rocket.Looper([rocket.Dataset(data, batch_size=bs), rocket.Module(Net(), [rocket.Loss(Obj()), rocket.Optimizer(opt)]),
                        Rec()], progress=False)],
        num_procs=world, cpu=True, destroy_process_group_after_launch=(world > 1),
    ).launch()
    if out_file:
        with open(out_file, "w") as fh:
            json.dump(dict(w=[p.tolist() for p in net.parameters()], losses=losses), fh)
    return net, losses


def _launcher_worker(rank, world, port, out, bs):
    _env(rank, world, port)
    _train(world, os.path.join(out, f"r{rank}.json"), bs=bs)


@pytest.mark.parametrize("world", [2, 4])
def test_launcher_ranks_equal_global_batch(tmp_path, world):
    _run(_launcher_worker, world, str(tmp_path), 8 // world)
    net, losses = _train(1, None, bs=8)  # same global batches: rank r gets batches r, r+W, ...
    for r in range(world):
        got = json.load(open(tmp_path / f"r{r}.json"))
        for g, p in zip(got["w"], net.parameters()):
            torch.testing.assert_close(torch.tensor(g), p.detach(), rtol=1e-5, atol=1e-6)
        # reported loss = mean over ranks of per-rank mean == global-batch mean
        assert got["losses"] == pytest.approx(losses, rel=1e-5)


# ------------------------------------------------------- gather_for_metrics
def _meter_worker(rank, world, port, out):
    _env(rank, world, port)
    import rocket_amd as rocket

    seen = []

    class Collect(rocket.Metric):
        def launch(self, attrs=None):
            seen.extend(attrs.batch["idx"].tolist())

        def reset(self, attrs=None):
            pass

    data = [{"idx": torch.tensor(i)} for i in range(10)]  # 10 samples, bs 3, W 2 -> padded to 12
    rocket.Launcher(
        [rocket.Looper([rocket.Dataset(data, batch_size=3), rocket.Meter([Collect()], keys=["idx"])],
                       grad_enabled=False, progress=False)],
        num_procs=world, cpu=True,
    ).launch()
    with open(os.path.join(out, f"m{rank}.json"), "w") as fh:
        json.dump(seen, fh)


def test_gather_for_metrics_truncates_padding(tmp_path):
    _run(_meter_worker, 2, str(tmp_path))
    for r in range(2):
        seen = json.load(open(tmp_path / f"m{r}.json"))
        assert sorted(seen) == list(range(10))


def test_bench_multi_rank_cpu(tmp_path):
    """bench.py under torch.distributed.run with 4 gloo ranks (the driver's N-GPU launch shape, CPU
    edition): one JSON line from rank 0 with whole-job numbers."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(root, "bench.py"), "--gpus", "4", "--cpu",
           "--steps", "3", "--warmup", "1", "--batch", "64"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 4 and rec["steps"] == 3 and rec["config"]["global_batch"] == 256
    assert rec["config"]["parallelism"] == "dp4" and rec["value"] > 0


# ------------------------------------ GA with a branch unused in the sync micro-step
class _Branchy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(4, 4)
        self.b = torch.nn.Linear(4, 4)

    def forward(self, x, use_b):
        y = self.a(x)
        return y + self.b(x) if use_b else y


def _unused_worker(rank, world, port, out):
    _env(rank, world, port)
    from rocket_amd.parallel.ddp import DataParallel
    from rocket_amd.runtime import comm

    comm.init(cpu=True)
    torch.manual_seed(0)
    net = _Branchy()
    dp = DataParallel(net, first_bucket_mb=1e-5, bucket_cap_mb=1e-5)
    x = torch.randn(2 * world, 4, generator=torch.Generator().manual_seed(3))
    mine = x[rank * 2 : rank * 2 + 2]
    dp.zero_grad()
    with dp.no_sync():
        dp(mine, True).pow(2).sum().backward()   # micro-step 1: both branches
    dp(mine, False).pow(2).sum().backward()      # micro-step 2 (sync): branch b unused
    with open(os.path.join(out, f"u{rank}.json"), "w") as fh:
        json.dump([p.grad.tolist() for p in net.parameters()], fh)
    comm.shutdown()


def test_ga_unused_in_sync_step_keeps_accumulated_grad(tmp_path):
    """a param that got gradients in a no_sync micro-step but none in the sync one must
    contribute its accumulated local gradient to the all-reduce (torch DDP semantics)."""
    _run(_unused_worker, 2, str(tmp_path))
    torch.manual_seed(0)
    net = _Branchy()
    x = torch.randn(4, 4, generator=torch.Generator().manual_seed(3))
    for r in range(2):
        m = x[r * 2 : r * 2 + 2]
        (net(m, True).pow(2).sum() / 2).backward()
        (net(m, False).pow(2).sum() / 2).backward()
    ref = [p.grad for p in net.parameters()]
    assert float(ref[2].abs().sum()) > 0  # branch b really has an accumulated gradient
    for r in range(2):
        got = json.load(open(tmp_path / f"u{r}.json"))
        for g, e in zip(got, ref):
            torch.testing.assert_close(torch.tensor(g), e, rtol=1e-5, atol=1e-6)


# ------------------------------------------------------- scheduler steps x W
def _sched_worker(rank, world, port, out):
    _env(rank, world, port)
    import rocket_amd as rocket

    net = torch.nn.Linear(3, 2)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = net

        def forward(self, b):
            return (self.lin(b[0]), b[1])

    class Obj(torch.nn.Module):
        def forward(self, b):
            return torch.nn.functional.mse_loss(b[0], b[1])

    opt = torch.optim.SGD(net.parameters(), lr=1.0)
    sched = torch.optim.lr_scheduler.StepLR(opt, 4)
    data = [(torch.randn(3), torch.randn(2)) for _ in range(8)]
    rocket.Launcher(
        [rocket.Looper([rocket.Dataset(data, batch_size=1),
                        rocket.Module(Net(), [rocket.Loss(Obj()), rocket.Optimizer(opt), rocket.Scheduler(sched)])],
                       progress=False)],
        num_procs=world, cpu=True, destroy_process_group_after_launch=True,
    ).launch()
    with open(os.path.join(out, f"s{rank}.json"), "w") as fh:
        json.dump(dict(count=sched._step_count, lr=opt.param_groups[0]["lr"]), fh)


def test_scheduler_steps_times_world(tmp_path):
    """accelerate's AcceleratedScheduler steps the wrapped scheduler W times per optimizer step
    (reference ``rocket/core/scheduler.py:112-113``): 8 samples, batch 1, W=2 ->
    4 steps per rank -> 1 (construction) + 4*2 = 9 scheduler steps; StepLR(4) has decayed twice."""
    _run(_sched_worker, 2, str(tmp_path))
    for r in range(2):
        got = json.load(open(tmp_path / f"s{r}.json"))
        assert got["count"] == 9
        assert got["lr"] == pytest.approx(0.01)


def test_bench_self_spawns_ranks(tmp_path):
    """``python bench.py --gpus 4 --cpu`` with no launcher starts the 4 ranks itself (child
    process, no exec) and prints ONE whole-job line with n_gpus 4."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "4", "--cpu", "--steps", "3", "--warmup", "1",
           "--batch", "32"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 4 and rec["config"]["parallelism"] == "dp4"


# ------------------------------------------- BatchNorm buffers: one flat broadcast
def _bn_worker(rank, world, port, out):
    _env(rank, world, port)
    from rocket_amd.parallel.ddp import DataParallel
    from rocket_amd.runtime import comm

    comm.init(cpu=True)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3), torch.nn.BatchNorm2d(4), torch.nn.ReLU(),
                              torch.nn.Conv2d(4, 2, 1), torch.nn.BatchNorm2d(2))
    dp = DataParallel(net)
    assert dp._flat_buffers is not None and len(dp._bufs) == 6
    x = torch.randn(2, 3, 6, 6, generator=torch.Generator().manual_seed(10 + rank))  # different data per rank
    for _ in range(3):
        dp(x).sum().backward()
    net.eval()
    dp(x)  # broadcasts rank 0's statistics (after 3 local updates); eval: no further update
    with open(os.path.join(out, f"b{rank}.json"), "w") as fh:
        json.dump([b.tolist() for b in net.buffers()], fh)
    comm.shutdown()


def test_bn_buffers_single_flat_broadcast(tmp_path):
    _run(_bn_worker, 2, str(tmp_path))
    b0 = json.load(open(tmp_path / "b0.json"))
    b1 = json.load(open(tmp_path / "b1.json"))
    assert b0 == b1
    # rank 0's statistics moved away from the init values (updates go through the views) and the
    # counters count every training forward on rank 0 (3) -- broadcast and in-place updates compose
    assert b0[2] == 3 and b0[0] != [0.0] * 4


def _debug_worker(rank, world, port, out):
    os.environ["ROCKET_DEBUG_SYNC"] = "1"
    _reducer_worker(rank, world, port, out)


def test_reducer_debug_assertions(tmp_path):
    """ROCKET_DEBUG_SYNC=1: the reducer's bucket / stream-ordering assertions hold on a correct
    multi-bucket run (W=2 gloo) and the result is unchanged."""
    _run(_debug_worker, 2, str(tmp_path))
    got = [json.load(open(tmp_path / f"g{r}.json")) for r in range(2)]
    assert got[0]["nb"] > 1 and got[0]["grads"] == got[1]["grads"]


def test_reducer_debug_detects_double_launch():
    from rocket_amd.parallel.ddp import DataParallel

    class _Comm:
        rank, world = 0, 1

        def all_reduce_avg(self, flat):
            class _W:
                def wait(self):
                    pass

            return _W()

        def broadcast(self, t, src=0):
            return None

    os.environ["ROCKET_DEBUG_SYNC"] = "1"
    try:
        dp = DataParallel(torch.nn.Linear(4, 4), comm=_Comm())
    finally:
        os.environ.pop("ROCKET_DEBUG_SYNC")
    dp(torch.randn(2, 4)).sum().backward()
    b = dp.buckets[0]
    dp._launched = [b.index]
    with pytest.raises(RuntimeError, match="reduced twice"):
        dp._launch(b)
