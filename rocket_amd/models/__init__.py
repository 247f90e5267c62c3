"""Model zoo for the BASELINE configs (LeNet/MNIST, ResNet-18/50, ViT-B/16)."""

from rocket_amd.models.lenet import CrossEntropy, LeNet, synthetic_mnist  # noqa: F401
