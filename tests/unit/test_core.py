"""Capsule-tree semantics on CPU: attributes, ordering, LIFO registration, event-order oracle."""

import os

import pytest
import torch

import rocket_amd as rocket
from rocket_amd.core.attributes import Attributes
from rocket_amd.core.capsule import Capsule, Events
from rocket_amd.core.dispatcher import Dispatcher


class _FakeEngine:
    def __init__(self):
        self._custom_objects = []

    def register_for_checkpointing(self, *objs):
        self._custom_objects.extend(objs)


class _State(Capsule):
    def __init__(self, **kw):
        super().__init__(statefull=True, **kw)

    def state_dict(self):
        return {}

    def load_state_dict(self, s):
        pass


def test_attributes_semantics():
    a = Attributes(x=1)
    assert a.x == 1 and a.y is None
    a.z = 2
    assert a["z"] == 2
    del a.z
    assert "z" not in a
    with pytest.raises(AttributeError):
        a.__missing_dunder__
    b = Attributes(a)
    b.x = 5
    assert a.x == 1  # copy, not alias


def test_dispatcher_priority_is_stable_descending():
    caps = [Capsule(priority=p) for p in (1, 5, 5, 3)]
    d = Dispatcher(caps)
    assert d._capsules == [caps[1], caps[2], caps[3], caps[0]]


def test_dispatcher_rejects_non_capsules():
    with pytest.raises(ValueError):
        Dispatcher([object()])


def test_looper_rejects_nested_looper():
    with pytest.raises(RuntimeError):
        rocket.Looper([rocket.Looper([], repeats=1)], repeats=1)


def test_check_accelerator():
    with pytest.raises(RuntimeError):
        Capsule().setup()


def test_lifo_registration_enforced():
    eng = _FakeEngine()
    a, b = _State(), _State()
    for c in (a, b):
        c.accelerate(eng)
        c.setup()
    with pytest.raises(RuntimeError, match="Illegal destroy"):
        a.destroy()
    assert eng._custom_objects == [a, b]  # the wrong pop was undone
    b.destroy()
    a.destroy()
    assert eng._custom_objects == []


def test_unregistered_stateful_destroy_is_noop():
    eng = _FakeEngine()
    other = _State()
    other.accelerate(eng)
    other.setup()
    c = _State()
    c.accelerate(eng)
    c.destroy()  # never set up -> must not pop `other` (reference Q1)
    assert eng._custom_objects == [other]


def _tree(tmp_path, n=10, bs=2, ckpt_every=2, repeats=None, statefull=True, tag="exp", **launcher_kw):
    torch.manual_seed(0)
    x = torch.randn(n, 4)
    y = torch.randint(0, 3, (n,))
    data = [(x[i], y[i]) for i in range(n)]
    net = torch.nn.Linear(4, 3)
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    sched = torch.optim.lr_scheduler.StepLR(opt, 2)

    class Objective(torch.nn.Module):
        def forward(self, batch):
            return torch.nn.functional.cross_entropy(batch[2], batch[1])

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = net

        def forward(self, batch):
            return (batch[0], batch[1], self.lin(batch[0]))

    caps = [
        rocket.Dataset(data, batch_size=bs),
        rocket.Module(Net(), [rocket.Loss(Objective()), rocket.Optimizer(opt), rocket.Scheduler(sched)]),
    ]
    if ckpt_every:
        caps.append(rocket.Checkpointer(save_every=ckpt_every))
    looper = rocket.Looper(caps, repeats=repeats, progress=False)
    launcher = rocket.Launcher([looper], tag=tag, logging_dir=str(tmp_path), statefull=statefull, cpu=True,
                               destroy_process_group_after_launch=False, **launcher_kw)
    return launcher, net, opt, sched


def test_event_order_oracle(tmp_path, monkeypatch):
    trace = []
    orig = Capsule.dispatch

    def spy(self, event, attrs=None):
        trace.append((type(self).__name__, event.value))
        return orig(self, event, attrs)

    monkeypatch.setattr(Capsule, "dispatch", spy)
    launcher, *_ = _tree(tmp_path, n=4, bs=2)
    launcher.launch()
    setup = [n for n, e in trace if e == "setup"]
    assert setup == ["Looper", "Dataset", "Module", "Loss", "Optimizer", "Scheduler", "Checkpointer"]
    destroy = [n for n, e in trace if e == "destroy"]
    assert destroy == ["Looper", "Checkpointer", "Module", "Scheduler", "Optimizer", "Loss", "Dataset"]
    launches = [n for n, e in trace if e == "launch"]
    it = ["Dataset", "Module", "Loss", "Optimizer", "Scheduler", "Checkpointer"]
    # the Launcher calls Looper.launch directly; 2 batches -> 2 full iterations
    assert launches == it * 2
    assert [n for n, e in trace if e == "set"] == ["Dataset", "Module", "Loss", "Optimizer", "Scheduler", "Checkpointer"]


def test_checkpoint_layout_and_versioning(tmp_path):
    launcher, *_ = _tree(tmp_path, n=10, bs=2, ckpt_every=2)
    launcher.launch()
    root = tmp_path / "exp" / "v0" / "weights"
    assert sorted(os.listdir(root)) == ["001", "003"]
    files = sorted(os.listdir(root / "003"))
    assert files == sorted([
        "model.safetensors", "optimizer.bin", "scheduler.bin", "random_states_0.pkl",
        "custom_checkpoint_0.pkl", "custom_checkpoint_1.pkl", "custom_checkpoint_2.pkl",
        "custom_checkpoint_3.pkl",
    ])
    # Launcher, Looper, Dataset, Loss in registration order
    c = [torch.load(root / "003" / f"custom_checkpoint_{i}.pkl", weights_only=True) for i in range(4)]
    assert set(c[0]) == {"epoch_idx", "num_procs", "num_nodes"}
    assert c[2] == {"batch_idx": 4}
    assert set(c[3]) == {"value", "step"} and c[3]["step"] == 4
    launcher2, *_ = _tree(tmp_path, n=10, bs=2, ckpt_every=2)
    launcher2.launch()
    assert sorted(os.listdir(tmp_path / "exp")) == ["v0", "v1"]


def test_no_versioning_refuses_existing_dir(tmp_path):
    l1, *_ = _tree(tmp_path, ckpt_every=0, experiment_versioning=False)
    l1.launch()
    l2, *_ = _tree(tmp_path, ckpt_every=0, experiment_versioning=False)
    with pytest.raises(ValueError):
        l2.launch()


def test_checkpointer_requires_project_dir(tmp_path):
    launcher, *_ = _tree(tmp_path, ckpt_every=2, tag=None)
    with pytest.raises(ValueError, match="project directory"):
        launcher.launch()


def test_resume_mid_epoch_matches_uninterrupted(tmp_path):
    # uninterrupted: 2 epochs of 5 batches
    ref, net_ref, *_ = _tree(tmp_path / "a", n=10, bs=2, ckpt_every=0, num_epochs=2)
    ref.launch()
    # interrupted: stop after 3 batches of epoch 0 with a checkpoint, then resume
    part, *_ = _tree(tmp_path / "b", n=10, bs=2, ckpt_every=3, repeats=3, num_epochs=1)
    part.launch()
    ck = tmp_path / "b" / "exp" / "v0" / "weights" / "002"
    res, net_res, *_ = _tree(tmp_path / "c", n=10, bs=2, ckpt_every=0, num_epochs=2)
    res.resume(str(ck))
    res.launch()
    for a, b in zip(net_ref.parameters(), net_res.parameters()):
        torch.testing.assert_close(a, b)


def test_looper_needs_repeats():
    eng_launcher = rocket.Launcher([rocket.Looper([Capsule()], progress=False)], cpu=True,
                                   destroy_process_group_after_launch=False)
    with pytest.raises(RuntimeError, match="infinite loops"):
        eng_launcher.launch()


def test_looper_run_every(tmp_path):
    seen = []

    class Probe(Capsule):
        def launch(self, attrs=None):
            seen.append(attrs.launcher.epoch_idx)

    rocket.Launcher([rocket.Looper([Probe()], repeats=1, run_every=2, progress=False)], num_epochs=5, cpu=True,
                    destroy_process_group_after_launch=False).launch()
    assert seen == [0, 2, 4]


def test_events_enum_values():
    assert [e.value for e in Events] == ["setup", "destroy", "set", "reset", "launch"]


def test_resume_latest(tmp_path):
    part, *_ = _tree(tmp_path, n=10, bs=2, ckpt_every=2, repeats=4, num_epochs=1)
    part.launch()
    from rocket_amd.core.launcher import latest_checkpoint

    latest = latest_checkpoint(str(tmp_path / "exp"))
    assert latest is not None and latest.endswith("003")
    res, *_ = _tree(tmp_path, n=10, bs=2, ckpt_every=0, num_epochs=1)
    res.resume("latest")
    assert res._resume_from == latest
    res.launch()
    fresh, *_ = _tree(tmp_path / "none", n=10, bs=2, ckpt_every=0)
    assert fresh.resume("latest")._resume_from is None
