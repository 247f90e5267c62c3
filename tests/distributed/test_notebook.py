"""Notebook launch path: inside a (simulated) Jupyter kernel, Launcher.launch spawns num_procs
workers that each run the whole tree as one rank of a gloo group."""

import os

import torch

import rocket_amd as rocket
import rocket_amd.core.launcher as launcher_mod


class MarkRank(rocket.Capsule):
    def __init__(self, out_dir):
        super().__init__(priority=10)
        self.out_dir = out_dir

    def launch(self, attrs=None):
        e = self._accelerator
        with open(os.path.join(self.out_dir, f"rank{e.process_index}_of{e.num_processes}"), "a") as fh:
            fh.write("x")


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(4, 2)

    def forward(self, b):
        return (self.lin(b[0]), b[1])


class Obj(torch.nn.Module):
    def forward(self, b):
        return torch.nn.functional.cross_entropy(b[0], b[1])


def test_notebook_launch_spawns_ranks(tmp_path, monkeypatch):
    monkeypatch.setattr(launcher_mod, "in_notebook", lambda: True)
    data = [(torch.randn(4), torch.tensor(i % 2)) for i in range(16)]
    net = Net()
    tree = rocket.Launcher(
        [rocket.Looper([rocket.Dataset(data, batch_size=2),
                        rocket.Module(net, [rocket.Loss(Obj()), rocket.Optimizer(torch.optim.SGD(net.parameters(), lr=0.1))]),
                        MarkRank(str(tmp_path))], progress=False)],
        num_procs=2, cpu=True,
    )
    tree.launch()
    files = sorted(os.listdir(tmp_path))
    assert files == ["rank0_of2", "rank1_of2"]
    assert all(len(open(tmp_path / f).read()) == 4 for f in files)  # 16 samples / (bs 2 x 2 ranks)
