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
layer_norm / batch_norm fused fwd/bwd                                      BASELINE configs
=====================  ================================================  ==========================
"""

from __future__ import annotations

import torch

from rocket_amd.ops import _lib


def native_available() -> bool:
    return _lib.available()


def require_native() -> None:
    """Fail loudly when running on a GPU without the native kernels."""
    _lib.kernels()


def on_hip(*tensors: torch.Tensor) -> bool:
    return all(t is not None and t.device.type == "cuda" for t in tensors if t is not None)
