"""A script written against the reference's import paths (``import rocket``, ``rocket.core.*``,
``rocket.utils.*``) runs unchanged on this framework (CPU, W=1)."""

import torch
from torch import nn

import rocket
from rocket.core.capsule import Attributes, Capsule, Events
from rocket.core.loop import Looper
from rocket.core.meter import rebuild_batch
from rocket.utils.collections import apply_to_collection
from rocket.utils.torch import torch_collate, torch_move


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(4, 3)

    def forward(self, batch):
        x, y = batch
        return x, y, self.fc(x)


class _Acc(rocket.Metric):
    def __init__(self, out):
        super().__init__()
        self.out = out

    def launch(self, attrs: Attributes = None):
        self.out.append(int((attrs.batch[2].argmax(1) == attrs.batch[1]).sum()))

    def reset(self, attrs: Attributes = None):
        pass


def test_reference_import_paths_resolve():
    assert rocket.Launcher is rocket.core.launcher.Launcher
    assert Looper is rocket.Looper
    assert Events.LAUNCH.value == "launch" and issubclass(rocket.Dispatcher, Capsule)
    assert [c.__name__ for c in rocket.core.__sphinx_classes__][:3] == ["Capsule", "Dispatcher", "Dataset"]
    batch = torch_collate([(torch.ones(2), 1, "a"), (torch.zeros(2), 2, "b")])
    assert batch[0].shape == (2, 2) and batch[2] == ["a", "b"]
    assert torch_move({"k": torch.ones(1)}, "cpu")["k"].device.type == "cpu"
    assert apply_to_collection([1, 2], lambda v, key=None: v * 2) == [2, 4]
    assert callable(rebuild_batch({}))


def test_reference_style_pipeline_runs(tmp_path):
    g = torch.Generator().manual_seed(0)
    data = [(torch.randn(4, generator=g), torch.tensor(i % 3)) for i in range(24)]
    net = _Net()
    opt = torch.optim.AdamW(net.parameters())
    seen = []
    launcher = rocket.Launcher(
        [
            rocket.Looper([
                rocket.Dataset(data, batch_size=8),
                rocket.Module(net, capsules=[
                    rocket.Loss(lambda b: nn.functional.cross_entropy(b[2], b[1])),
                    rocket.Optimizer(opt),
                    rocket.Scheduler(torch.optim.lr_scheduler.StepLR(opt, 100)),
                ]),
                rocket.Checkpointer(save_every=3),
            ], tag="train"),
            rocket.Looper([rocket.Dataset(data, batch_size=8), rocket.Module(net), rocket.Meter([_Acc(seen)], keys=[1, 2])],
                          tag="eval", grad_enabled=False),
        ],
        tag="compat", logging_dir=str(tmp_path), num_epochs=2,
    )
    launcher.launch()
    assert len(seen) == 6  # 3 eval batches x 2 epochs
    ck = tmp_path / "compat" / "v0" / "weights"  # experiment_versioning=True by default
    assert sorted(p.name for p in ck.iterdir()) == ["002", "005"]  # global iterations 2 and 5
    assert (ck / "002" / "model.safetensors").exists()
