"""LeNet-5 as in the reference example (``examples/mnist.py:42-74``).

Topology: conv1 1→6 5×5 pad 2 → ReLU → maxpool 2 → conv2 6→16 5×5 → ReLU →
maxpool 2 → flatten(400) → fc1 120 → ReLU → fc2 84 → ReLU → fc3 10.  The forward
takes the batch tuple ``(img, label)`` and returns ``(img, label, logits)`` —
the reference's batch-in/batch-out contract.

``fused=True`` (default on a GPU) routes the layers through the hand-written
CDNA4 kernels of :mod:`rocket_amd.ops.lenet`:

* the whole feature extractor (both conv+bias+ReLU+maxpool stages) is one MFMA
  implicit-GEMM launch forward and one backward that routes the pooled
  gradient through saved 1-byte argmax/ReLU codes;
* the classifier (fc1-ReLU-fc2-ReLU-fc3) is one MFMA launch forward, one for
  the input-gradient chain and three split-K weight-gradient GEMMs with fused
  bias gradients (K5, K8).

``fused=False`` is the plain PyTorch module (CPU reference and numerics oracle);
both share parameter names, so checkpoints are interchangeable.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn


class LeNet(nn.Module):
    def __init__(self, num_classes: int = 10, fused: bool | None = None):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 6, 5, padding=2)
        self.conv2 = nn.Conv2d(6, 16, 5)
        self.fc1 = nn.Linear(16 * 5 * 5, 120)
        self.fc2 = nn.Linear(120, 84)
        self.fc3 = nn.Linear(84, num_classes)
        self._fused = fused

    def use_fused(self, x: torch.Tensor) -> bool:
        if self._fused is False:
            return False
        if x.device.type != "cuda":
            if self._fused:
                raise RuntimeError("fused LeNet kernels need a HIP device")
            return False
        return True

    def logits(self, x: torch.Tensor, target: torch.Tensor | None = None) -> torch.Tensor:
        """``target`` (optional, the batch's labels): lets the fused path run the training step's
        cross-entropy backward speculatively inside the forward launch (ops/lenet.py)."""
        if self.use_fused(x):
            from rocket_amd.ops.lenet import lenet_features, lenet_forward, mlp_head

            if x.shape[0] % 8 == 0 and self.fc3.out_features == 10:
                return lenet_forward(x, self.conv1, self.conv2, self.fc1, self.fc2, self.fc3,
                                     target if self.training else None)
            h = lenet_features(x, self.conv1.weight, self.conv1.bias, self.conv2.weight, self.conv2.bias)
            return mlp_head(h, [self.fc1, self.fc2, self.fc3])
        x = F.max_pool2d(F.relu(self.conv1(x)), 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = torch.flatten(x, 1)
        x = F.relu(self.fc1(x))
        x = F.relu(self.fc2(x))
        return self.fc3(x)

    #: the fused training step gathers a deferred device-loader batch itself (runtime/data.py
    #: PendingRows; the Looper defers the gather of batches this model consumes)
    consumes_pending_rows = True

    def _whole_fused(self, x: torch.Tensor) -> bool:
        return self.use_fused(x) and x.shape[0] % 8 == 0 and self.fc3.out_features == 10

    def forward(self, batch):
        from rocket_amd.runtime.data import materialize_batch

        if isinstance(batch, torch.Tensor):
            materialize_batch(batch)
            return self.logits(batch)
        img, label = batch[0], batch[1]
        if not self._whole_fused(img):  # only the whole-step fused path gathers a deferred batch
            materialize_batch(batch)
        return (img, label, self.logits(img, label))


class CrossEntropy(nn.Module):
    """``CrossEntropyLoss(batch[2], batch[1])`` (reference ``examples/mnist.py:81-84``).

    On a HIP device it uses the fused softmax-cross-entropy kernel (loss and
    d(logits) in one pass).
    """

    def __init__(self, fused: bool | None = None):
        super().__init__()
        self._fused = fused

    def forward(self, batch):
        logits, target = batch[2], batch[1]
        if self._fused is not False and logits.device.type == "cuda":
            from rocket_amd.ops.cross_entropy import cross_entropy

            return cross_entropy(logits, target)
        return F.cross_entropy(logits.float(), target)


    def loss_and_grad(self, batch, grad_scale: float, accum=None, dev_scale=None):
        """Training-step fast path (used by the Loss capsule under graph capture): loss and
        d(logits) in one launch.  Returns ``(loss, outputs, output_grads)`` or None.  ``dev_scale``:
        the fp16 loss scale (1-element device tensor) d(logits) is multiplied by; only the fused
        LeNet backward takes one (None is returned for other logits)."""
        logits, target = batch[2], batch[1]
        if self._fused is False or logits.device.type != "cuda":
            return None
        from rocket_amd.ops.cross_entropy import ce_train
        from rocket_amd.ops.lenet import fuse_cross_entropy

        # CE inside the LeNet backward launch
        fused = fuse_cross_entropy(logits, target, grad_scale, accum, dev_scale=dev_scale)
        if fused is not None:
            return fused[0], [logits], [fused[1]]
        if dev_scale is not None:
            return None
        res = ce_train(logits, target, grad_scale, accum)
        if res is None:
            return None
        loss, dlogits = res
        return loss, [logits], [dlogits]


def synthetic_mnist(n: int = 60000, device="cpu", seed: int = 0, dtype=torch.float32):
    """Random 1×28×28 images in [0,1) and labels in [0,10) (no network: no real MNIST)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.rand(n, 1, 28, 28, generator=g, dtype=torch.float32).to(dtype)
    y = torch.randint(0, 10, (n,), generator=g)
    return x.to(device), y.to(device)
