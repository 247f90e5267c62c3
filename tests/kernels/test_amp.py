"""fp16 dynamic loss scaling on the device (runtime/amp.py + optim.hip AmpSlot) vs torch.amp.GradScaler."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 8)).cuda()


@pytest.mark.parametrize("kind", ["adamw", "sgd"])
def test_fused_scaler_matches_torch_gradscaler(kind):
    from rocket_amd.ops.optim import FusedAdamW, FusedSGD
    from rocket_amd.runtime.amp import FusedGradScaler

    ref, mine = _model(), _model()
    if kind == "adamw":
        o_ref = torch.optim.AdamW(ref.parameters(), lr=1e-2)
        o_mine = FusedAdamW(mine.parameters(), lr=1e-2)
    else:
        o_ref = torch.optim.SGD(ref.parameters(), lr=1e-2, momentum=0.9)
        o_mine = FusedSGD(mine.parameters(), lr=1e-2, momentum=0.9)
    # small growth interval so growth AND backoff both happen within 10 steps
    s_ref = torch.amp.GradScaler("cuda", init_scale=1024.0, growth_interval=3)
    s_mine = FusedGradScaler("cuda", init_scale=1024.0, growth_interval=3)
    g = torch.Generator(device="cuda").manual_seed(1)
    skipped = []
    for step in range(10):
        x = torch.randn(16, 32, device="cuda", generator=g)
        for net, opt, sc in ((ref, o_ref, s_ref), (mine, o_mine, s_mine)):
            with torch.autocast("cuda", dtype=torch.float16):
                loss = net(x).float().pow(2).mean()
            sc.scale(loss).backward()
            if step == 4:  # injected overflow: this step must be skipped, scale halved
                next(net.parameters()).grad[0, 0] = float("inf")
            sc.step(opt)
            sc.update()
            opt.zero_grad()
        skipped.append(s_mine.last_step_skipped())
        assert s_mine.get_scale() == s_ref.get_scale(), step
    assert skipped[4] and not any(skipped[:4] + skipped[5:])
    # fp32 op-order differences only (torch divides by sqrt(bc2), the kernel multiplies by its
    # rsqrt); Adam amplifies them on near-zero second moments: same bound as test_ce_optim at 10x lr
    for a, b in zip(ref.parameters(), mine.parameters()):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5)
    # checkpoint format interchangeable with torch's GradScaler
    sd = s_mine.state_dict()
    assert sd.keys() == s_ref.state_dict().keys() and sd["scale"] == s_ref.state_dict()["scale"]
    assert sd["_growth_tracker"] == s_ref.state_dict()["_growth_tracker"]


def test_engine_fp16_uses_device_scaler():
    """Through the engine's optimizer wrapper: no per-step host read unless the scheduler asks."""
    from rocket_amd.ops.optim import FusedAdamW
    from rocket_amd.runtime.amp import FusedGradScaler
    from rocket_amd.runtime.engine import Engine

    eng = Engine(mixed_precision="fp16")
    assert isinstance(eng.scaler, FusedGradScaler)
    net = eng.prepare_model(_model())
    opt = eng.prepare_optimizer(FusedAdamW(net.parameters(), lr=1e-3))
    x = torch.randn(16, 32, device="cuda")
    for _ in range(3):
        with eng.autocast():
            loss = net(x).float().pow(2).mean()
        eng.backward(loss)
        opt.step_and_zero_grad()
    assert opt.step_was_skipped is False
    assert eng.scaler.get_scale() == 65536.0


def test_torch_gradscaler_protocol_with_fused_optimizer():
    """A user-supplied torch.amp.GradScaler drives the fused optimizer through
    ``_step_supports_amp_scaling`` (grad_scale = the scale, found_inf) with torch's results."""
    from rocket_amd.ops.optim import FusedAdamW

    ref, mine = _model(), _model()
    o_ref = torch.optim.AdamW(ref.parameters(), lr=1e-2)
    o_mine = FusedAdamW(mine.parameters(), lr=1e-2)
    s_ref = torch.amp.GradScaler("cuda", init_scale=256.0)
    s_mine = torch.amp.GradScaler("cuda", init_scale=256.0)
    x = torch.randn(16, 32, device="cuda")
    for step in range(4):
        for net, opt, sc in ((ref, o_ref, s_ref), (mine, o_mine, s_mine)):
            loss = net(x).pow(2).mean()
            sc.scale(loss).backward()
            if step == 2:
                next(net.parameters()).grad[1, 1] = float("nan")
            sc.step(opt)
            sc.update()
            opt.zero_grad()
    # fp32 op-order differences only (torch divides by sqrt(bc2), the kernel multiplies by its
    # rsqrt); Adam amplifies them on near-zero second moments: same bound as test_ce_optim at 10x lr
    for a, b in zip(ref.parameters(), mine.parameters()):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5)


def test_skip_flags_published_to_host_ring():
    """Each fused update's last block publishes its own skip flag into the host-mapped ring: once
    the updates ran, every handle is readable with a plain host load (no copy, no event), and
    handles of earlier steps still resolve to THEIR step's flag after later steps ran."""
    from rocket_amd.ops.optim import FusedAdamW
    from rocket_amd.runtime.amp import SEQ, FusedGradScaler

    net = _model()
    opt = FusedAdamW(net.parameters(), lr=1e-3)
    sc = FusedGradScaler("cuda", init_scale=1024.0)
    x = torch.randn(16, 32, device="cuda")
    handles = []
    for step in range(6):
        with torch.autocast("cuda", dtype=torch.float16):
            loss = net(x).float().pow(2).mean()
        sc.scale(loss).backward()
        if step in (1, 4):
            next(net.parameters()).grad[0, 0] = float("inf")
        sc.step(opt)
        sc.update()
        opt.zero_grad()
        handles.append(sc.last_handle())
    torch.cuda.synchronize()
    assert all(FusedGradScaler.handle_ready(h) for h in handles)
    assert [FusedGradScaler.handle_skipped(h) for h in handles] == [False, True, False, False, True, False]
    assert int(sc.state.view(torch.int32)[SEQ]) == 6
