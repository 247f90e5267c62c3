"""Model zoo for the BASELINE configs (LeNet/MNIST, ResNet-18/50, ViT-B/16)."""

from rocket_amd.models.lenet import CrossEntropy, LeNet, synthetic_mnist  # noqa: F401
from rocket_amd.models.resnet import ResNet, resnet18, resnet50  # noqa: F401
from rocket_amd.models.vit import VisionTransformer, vit_b16  # noqa: F401
