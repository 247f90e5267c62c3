"""End-to-end capsule trees on the GPU: checkpoint/resume with the fused optimizer's device state,
fp16 autocast + GradScaler through the fused kernels, and the eval looper (Meter) on fused LeNet."""

import os

import pytest
import torch

import rocket_amd as rocket
from rocket_amd.models import CrossEntropy, LeNet

pytestmark = pytest.mark.gpu


def _data(n=2048, seed=0):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(seed)
    return torch.rand(n, 1, 28, 28, generator=g, device=dev), torch.randint(0, 10, (n,), generator=g, device=dev)


def _tree(tmp, data, net, opt, repeats=None, ckpt=0, epochs=1, mp="bf16", capture=True, extra=()):
    caps = [rocket.Dataset(rocket.DeviceTensorDataset(*data), batch_size=256, shuffle=True),
            rocket.Module(net, [rocket.Loss(CrossEntropy()), rocket.Optimizer(opt)], capture=capture, warmup=2)]
    if ckpt:
        caps.append(rocket.Checkpointer(save_every=ckpt))
    return rocket.Launcher([rocket.Looper(caps + list(extra), repeats=repeats, progress=False)], tag="gpu",
                           logging_dir=str(tmp), num_epochs=epochs, mixed_precision=mp, statefull=True,
                           destroy_process_group_after_launch=False)


def test_resume_with_fused_optimizer_state(tmp_path):
    from rocket_amd.ops.optim import FusedAdamW

    data = _data()
    torch.manual_seed(0)
    ref = LeNet()
    _tree(tmp_path / "a", data, ref, FusedAdamW(ref.parameters(), lr=1e-3), epochs=2).launch()
    torch.manual_seed(0)
    part = LeNet()
    _tree(tmp_path / "b", data, part, FusedAdamW(part.parameters(), lr=1e-3), repeats=5, ckpt=5).launch()
    ck = tmp_path / "b" / "gpu" / "v0" / "weights" / "004"
    assert (ck / "optimizer.bin").exists()
    sd = torch.load(ck / "optimizer.bin", weights_only=True)
    assert all(float(st["step"]) == 5.0 for st in sd["state"].values())  # device step synced into state
    torch.manual_seed(1)  # different init: everything must come from the checkpoint
    res = LeNet()
    _tree(tmp_path / "c", data, res, FusedAdamW(res.parameters(), lr=1e-3), epochs=2).resume(str(ck)).launch()
    # The resumed run's first steps are eager (plain loss kernel -> d(logits) -> backward) where
    # the uninterrupted run replays the captured fused-cross-entropy step: the same math with a
    # different bf16 rounding of d(logits), and Adam turns such differences on near-zero gradients
    # into up to ~lr-sized weight deltas per step.  Resume is exact if the bulk agrees tightly and no
    # element drifts further than a few Adam steps (a wrong restore is off by O(0.1) everywhere).
    for a, b in zip(ref.parameters(), res.parameters()):
        d = (a - b).abs()
        assert d.max().item() <= 8e-3, d.max().item()
        assert (d > 2e-4).float().mean().item() < 0.01


def test_fp16_gradscaler_with_fused_kernels(tmp_path):
    from rocket_amd.ops.optim import FusedAdamW

    data = _data(1024)
    torch.manual_seed(0)
    net = LeNet()
    w0 = net.fc3.weight.detach().clone()
    losses = []

    class Rec(rocket.Capsule):
        def __init__(self):
            super().__init__(priority=10)

        def launch(self, attrs=None):
            losses.append(float(attrs.looper.state.loss))

    _tree(tmp_path, data, net, FusedAdamW(net.parameters(), lr=1e-3), mp="fp16", extra=[Rec()]).launch()
    assert len(losses) == 4 and all(torch.isfinite(torch.tensor(losses)))
    assert not torch.equal(w0.cpu(), net.fc3.weight.detach().cpu())


def test_eval_looper_meter_on_fused_lenet(tmp_path):
    from rocket_amd.ops.optim import FusedAdamW

    data = _data(1024)
    net = LeNet()
    seen = []

    class Acc(rocket.Metric):
        def launch(self, attrs=None):
            seen.append(attrs.batch[2].shape[0])
            attrs.looper.state.acc = float((attrs.batch[2].argmax(1) == attrs.batch[1]).float().mean())

        def reset(self, attrs=None):
            pass

    ev = _data(1000, seed=3)
    rocket.Launcher(
        [rocket.Looper([rocket.Dataset(rocket.DeviceTensorDataset(*data), batch_size=256),
                        rocket.Module(net, [rocket.Loss(CrossEntropy()), rocket.Optimizer(FusedAdamW(net.parameters()))],
                                      capture=True)], progress=False),
         rocket.Looper([rocket.Dataset(rocket.DeviceTensorDataset(*ev), batch_size=256), rocket.Module(net),
                        rocket.Meter([Acc()], keys=[1, 2])], grad_enabled=False, progress=False)],
        logging_dir=str(tmp_path), mixed_precision="bf16", num_epochs=2, destroy_process_group_after_launch=False,
    ).launch()
    assert sum(seen) == 2000  # 1000 eval samples per epoch (last batch 232)


def test_fp16_step_is_captured_and_matches_eager(tmp_path):
    """fp16 steps with the device-resident scaler replay as graphs (flag check + scaled update
    in-graph, the skip flag copied after each replay for the LR scheduler) and give the eager
    run's weights, loss scale and learning rate."""
    from rocket_amd.ops.optim import FusedSGD

    class Mlp(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.net = torch.nn.Sequential(torch.nn.Flatten(), torch.nn.Linear(784, 128), torch.nn.ReLU(),
                                           torch.nn.Linear(128, 10))

        def forward(self, batch):
            return (batch[0], batch[1], self.net(batch[0]))

    class Grab(rocket.Capsule):  # keeps the engine's scaler for after the launch
        def __init__(self):
            super().__init__(statefull=False)

        def setup(self, attrs=None):
            super().setup(attrs)
            held["scaler"] = self._accelerator.scaler

    held = {}
    data = _data(2048)
    runs = {}
    for capture in (False, True):
        torch.manual_seed(0)
        net = Mlp().cuda()
        opt = FusedSGD(net.parameters(), lr=0.05, momentum=0.9)
        sched = torch.optim.lr_scheduler.StepLR(opt, 3, gamma=0.5)
        mod = rocket.Module(net, [rocket.Loss(CrossEntropy()), rocket.Optimizer(opt), rocket.Scheduler(sched)],
                            capture=capture, warmup=2)
        launcher = rocket.Launcher(
            [rocket.Looper([rocket.Dataset(rocket.DeviceTensorDataset(*data), batch_size=256), mod, Grab()],
                           progress=False)],
            logging_dir=str(tmp_path / str(capture)), num_epochs=1, mixed_precision="fp16",
            destroy_process_group_after_launch=False)
        launcher.launch()
        scale = held["scaler"].get_scale()
        runs[capture] = ([p.detach().clone() for p in net.parameters()], sched.get_last_lr()[0], scale,
                         mod._graphs)
    g = runs[True][3]
    assert g is not None and g.captures >= 1 and g.replays >= 3, (g.disabled_reason, g.captures, g.replays)
    assert runs[True][1] == runs[False][1] < 0.05  # same skipped steps -> same scheduler steps
    assert runs[True][2] == runs[False][2]
    for a, b in zip(runs[False][0], runs[True][0]):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5)


def test_fp16_fused_lenet_captured_steps(tmp_path):
    """fp16 fused LeNet under the engine: captured steps run the speculative whole-step launch with
    the device loss scale and take the non-finite check from the weight-gradient launch (no check
    launch once captured), and end within Adam-rounding distance of the same run with capture off
    (plain loss kernel, separate check launch every step)."""
    from rocket_amd.ops.optim import FusedAdamW

    data = _data(2048)
    runs = {}
    for capture in (False, True):
        torch.manual_seed(0)
        net = LeNet()
        opt = FusedAdamW(net.parameters(), lr=1e-3)
        checks = []
        orig = opt.amp_check
        opt.amp_check = lambda amp, _o=orig: (checks.append(1), _o(amp))
        _tree(tmp_path / str(capture), data, net, opt, mp="fp16", capture=capture, epochs=2).launch()
        runs[capture] = ([p.detach().clone() for p in net.parameters()], len(checks))
    assert runs[False][1] == 2 * 2048 // 256  # eager: one check launch per optimizer step
    assert runs[True][1] <= 2  # captured: only the eager warm-up steps launch it
    for a, b in zip(runs[False][0], runs[True][0]):
        d = (a - b).abs()
        assert d.max().item() <= 2e-2, d.max().item()
        assert (d > 1e-3).float().mean().item() < 0.05, (d > 1e-3).float().mean().item()
