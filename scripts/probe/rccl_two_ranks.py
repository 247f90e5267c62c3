"""Probe: can two ranks share one GPU in one RCCL communicator on this box? (W=2 rehearsal)"""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def worker(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROCKET_DIST_BACKEND="gloo")
    from rocket_amd.runtime import comm
    from rocket_amd.parallel.rccl import RcclComm

    comm.init()
    c = RcclComm(torch.device("cuda", 0))
    t = torch.full((1024,), float(rank + 1), device="cuda")
    c.all_reduce_avg(t)
    torch.cuda.synchronize()
    print(f"rank {rank}: avg = {t[0].item()}", flush=True)
    c.close()


if __name__ == "__main__":
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(worker, args=(2, port), nprocs=2, start_method="spawn", join=True)
