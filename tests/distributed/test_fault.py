"""Fault injection: a rank dying mid-training must surface as an error on the survivors (no hang)."""

import os
import socket
import time

import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROCKET_PG_TIMEOUT="30")
    import rocket_amd as rocket

    class Crash(rocket.Capsule):
        def __init__(self):
            super().__init__(priority=10)
            self.n = 0

        def launch(self, attrs=None):
            self.n += 1
            if rank == 1 and self.n == 3:
                os._exit(17)  # simulated node loss: no cleanup, no goodbye

    data = [(torch.randn(4), torch.tensor(0)) for _ in range(64)]
    net = torch.nn.Linear(4, 2)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = net

        def forward(self, b):
            return (self.lin(b[0]), b[1])

    class Obj(torch.nn.Module):
        def forward(self, b):
            return torch.nn.functional.cross_entropy(b[0], b[1])

    rocket.Launcher([rocket.Looper([rocket.Dataset(data, batch_size=2),
                                    rocket.Module(Net(), [rocket.Loss(Obj()), rocket.Optimizer(torch.optim.SGD(net.parameters(), lr=0.1))]),
                                    Crash()], progress=False)], num_procs=world, cpu=True).launch()


def test_dead_rank_surfaces_as_error():
    ctx = mp.start_processes(_worker, args=(2, _port()), nprocs=2, start_method="spawn", join=False)
    t0 = time.time()
    while not all(not p.is_alive() for p in ctx.processes) and time.time() - t0 < 120:
        time.sleep(0.5)
    alive = [p for p in ctx.processes if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "a surviving rank hung after its peer died"
    codes = [p.exitcode for p in ctx.processes]
    assert codes[1] == 17
    assert codes[0] != 0  # the survivor failed loudly instead of finishing or hanging
