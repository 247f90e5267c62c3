"""HIP-graph capture of the training step must reproduce eager training.

Same seeds, same data order, same fused kernels: the captured run replays the
eager micro-step, so per-step losses and final weights agree to fp32 rounding
(atomics in split-K weight gradients make it not bit-exact).
"""

import pytest
import torch

import rocket_amd as rocket
from rocket_amd.core.capsule import Capsule

pytestmark = pytest.mark.gpu


class _Record(Capsule):
    def __init__(self):
        super().__init__(priority=10)
        self.losses = []

    def launch(self, attrs=None):
        if attrs is not None and attrs.looper is not None and attrs.looper.state.loss is not None:
            self.losses.append(attrs.looper.state.loss)


def _train(tmp_path, capture, steps=14, ga=1, batch=256):
    from rocket_amd.models import CrossEntropy, LeNet
    from rocket_amd.ops.optim import FusedAdamW

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    n = batch * (steps + 1)
    x = torch.rand(n, 1, 28, 28, generator=g, device=dev)
    y = torch.randint(0, 10, (n,), generator=g, device=dev)
    data = rocket.DeviceTensorDataset(x, y)
    torch.manual_seed(0)
    net = LeNet(fused=True)
    opt = FusedAdamW(net.parameters(), lr=2e-3)
    sched = torch.optim.lr_scheduler.StepLR(opt, 4, gamma=0.5)
    rec = _Record()
    mod = rocket.Module(
        net, [rocket.Loss(CrossEntropy(fused=True)), rocket.Optimizer(opt), rocket.Scheduler(sched)],
        capture=capture, warmup=2,
    )
    rocket.Launcher(
        [rocket.Looper([rocket.Dataset(data, batch_size=batch, shuffle=False), mod, rec], repeats=steps, progress=False)],
        logging_dir=str(tmp_path),
        mixed_precision="bf16",
        gradient_accumulation_steps=ga,
        destroy_process_group_after_launch=False,
    ).launch()
    torch.cuda.synchronize()
    losses = [float(v) for v in rec.losses]
    weights = {k: v.detach().float().cpu() for k, v in net.state_dict().items()}
    return losses, weights, mod


@pytest.mark.parametrize("ga", [1, 2])
def test_graph_matches_eager(tmp_path, ga):
    le, we, _ = _train(tmp_path / "e", capture=False, ga=ga)
    lg, wg, mod = _train(tmp_path / "g", capture=True, ga=ga)
    assert mod._graphs is not None and mod._graphs.disabled_reason == "released", mod._graphs.disabled_reason
    assert mod._graphs.replays > 0
    assert len(le) == len(lg) and len(le) > 0
    for a, b in zip(le, lg):
        assert abs(a - b) <= 2e-3 * max(1.0, abs(a)), (le, lg)
    for k in we:
        d = (we[k] - wg[k]).norm() / we[k].norm().clamp_min(1e-6)
        assert d < 5e-3, (k, float(d))
