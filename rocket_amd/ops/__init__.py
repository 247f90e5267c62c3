"""Hot-path operators implemented as hand-written CDNA4 HIP kernels.

=====================  ================================================  ==========================
op                      kernel(s)                                          replaces
=====================  ================================================  ==========================
cross_entropy           one-pass fused softmax-CE fwd; recompute-bwd      K6, K7
FusedAdamW / FusedSGD   multi-tensor update, device step/hyper-params     K12, N6, N7
linear                  MFMA bf16 GEMM + bias/ReLU/GELU epilogue,         K5, K8
                        dgrad/wgrad with fused bias-grad
conv_bias_relu_pool     direct conv + bias + ReLU + 2x2 maxpool (fwd),    K1-K4, K9-K11
                        unpool+ReLU-bwd fused into dgrad/wgrad
lenet_features/mlp_head MFMA LeNet conv stack / classifier, fwd+bwd        K1-K11 (flagship)
BatchNormAct2d          stats+apply(+residual+ReLU) fwd, reduce+apply bwd  ResNet configs
FusedLayerNorm          one wave per row, fused dgamma/dbeta reduction      ViT config
gelu / softmax          erf-GELU, scaled row softmax (attention)           ViT config
gather_rows/loss_accum  batch assembly, on-device loss bookkeeping         data path / Loss capsule
=====================  ================================================  ==========================

``set_fused(False)`` (or ``ROCKET_FUSED=0``) switches the model-level modules
(BatchNormAct2d, FusedLayerNorm, gelu, softmax) to their stock PyTorch
implementations for A/B runs; the default on a HIP device is the kernels.
"""

from __future__ import annotations

import os

import torch

from rocket_amd.ops import _lib


_FUSED = os.environ.get("ROCKET_FUSED", "1") != "0"


def set_fused(enabled: bool) -> None:
    global _FUSED
    _FUSED = bool(enabled)


def fused_enabled() -> bool:
    return _FUSED


def native_available() -> bool:
    return _lib.available()


def require_native() -> None:
    """Fail loudly when running on a GPU without the native kernels."""
    _lib.kernels()


def on_hip(*tensors: torch.Tensor) -> bool:
    return all(t is not None and t.device.type == "cuda" for t in tensors if t is not None)
