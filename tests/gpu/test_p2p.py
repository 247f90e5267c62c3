"""One-shot IPC/xGMI all-reduce kernel (``native/kernels/p2p.hip``), 2 ranks sharing ``cuda:0``.

Rank r contributes a deterministic tensor x_r; every rank must end with (x_0 + x_1) / 2 exactly
(the kernel sums in rank order in fp32, like the reference expression below), for sizes that are
and are not multiples of the per-block chunk, under uneven load (one rank busy before each
launch), and when the launch is captured in a HIP graph and replayed.
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


def _x(n, it, r, dev):
    g = torch.Generator(device=dev).manual_seed(1000 * it + r)
    return torch.randn(n, generator=g, device=dev)


def _worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from rocket_amd.parallel.p2p import P2PAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cap = 1 << 16
    ar = P2PAllReduce.create(cap, group=dist.group.WORLD, device=dev)
    res = dict(created=ar is not None, bad=[])
    if ar is not None:
        busy = torch.randn(2048, 2048, device=dev)
        it = 0
        for n in (61722, 2048, 5, cap, 4096 + 3):
            for rep in range(6):
                it += 1
                x = _x(n, it, rank, dev)
                want = sum(_x(n, it, r, dev) for r in range(world)) * (1.0 / world)
                if (rank + rep) % 2 == 0:  # uneven arrival: this rank is late
                    for _ in range(4):
                        busy = busy @ busy * 1e-3
                ar.all_reduce_(x, 1.0 / world)
                torch.cuda.synchronize()
                if not torch.equal(x, want):
                    res["bad"].append([n, rep, float((x - want).abs().max())])
        # captured: static buffer refreshed before each replay
        n = 61722
        static = torch.zeros(n, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        graph = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        dist.barrier()
        with torch.cuda.graph(graph, stream=s):
            ar.all_reduce_(static, 1.0 / world)
        for rep in range(20):
            it += 1
            static.copy_(_x(n, it, rank, dev))
            want = sum(_x(n, it, r, dev) for r in range(world)) * (1.0 / world)
            if rep % 3 == rank:
                for _ in range(4):
                    busy = busy @ busy * 1e-3
            graph.replay()
            torch.cuda.synchronize()
            if not torch.equal(static, want):
                res["bad"].append(["graph", rep, float((static - want).abs().max())])
        ar.check()
        res["launches"] = ar.launches
        dist.barrier()
        ar.close()
    with open(os.path.join(out_dir, f"p{rank}.json"), "w") as fh:
        json.dump(res, fh)
    dist.barrier()
    dist.destroy_process_group()


def test_p2p_allreduce_two_ranks(tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, start_method="spawn", join=True)
    for r in range(2):
        res = json.load(open(tmp_path / f"p{r}.json"))
        assert res["created"], res
        assert res["bad"] == [], res["bad"][:5]
