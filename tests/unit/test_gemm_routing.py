"""Routing predicates of the ViT GEMM modes (ops/mlinear.py): which products the default route
(`mixed`) sends to the native kernels.  Host-only (no kernel runs)."""
import torch

from rocket_amd.ops import mlinear


def test_mixed_routes_wide_bf16_products_to_xgemm5(monkeypatch):
    monkeypatch.setattr(mlinear, "MODE", "mixed")
    assert mlinear._x5_fwd(2304, 768, torch.bfloat16)      # qkv forward
    assert mlinear._x5_fwd(3072, 768, torch.bfloat16)      # fc1 forward / fc2 input gradient
    assert not mlinear._x5_fwd(768, 768, torch.bfloat16)   # 768-wide: the library
    assert not mlinear._x5_fwd(768, 3072, torch.bfloat16)
    assert not mlinear._x5_fwd(3072, 768, torch.float16)   # xgemm5 takes bf16 operands only
    assert not mlinear._x5_fwd(1000, 768, torch.bfloat16)  # N % 128


def test_mixed_small_products_are_bf16_heads_only(monkeypatch):
    monkeypatch.setattr(mlinear, "MODE", "mixed")
    assert mlinear._small(128, 1000, 768, torch.bfloat16)      # ViT head
    assert mlinear._small(256, 1000, 2048, torch.bfloat16)     # ResNet-50 head
    assert not mlinear._small(128, 1000, 768, torch.float16)   # mgemm is bf16-only: fp16 stays on the library
    assert not mlinear._small(25216, 768, 768, torch.bfloat16)  # a transformer projection


def test_other_modes_take_no_small_route(monkeypatch):
    for mode in ("lib", "x5", "native"):
        monkeypatch.setattr(mlinear, "MODE", mode)
        assert not mlinear._small(128, 1000, 768, torch.bfloat16)
    monkeypatch.setattr(mlinear, "MODE", "x5")
    assert mlinear._x5_fwd(768, 768, torch.bfloat16)  # x5: every x5-able product
