"""ResNet feature extractor feeding the MCDO kernel (PyTorch-ROCm; not part of the kernel).

torchvision is not available in this image, so the backbone the reference builds with
`torchvision.models.resnet18/34/50` (reference model.py:166-179) is defined here with the same
module tree, so reference checkpoints (state_dict keys `feature_extractor.conv1.weight`,
`feature_extractor.layer1.0.bn1.weight`, ...) load strictly. The reference replaces `fc` with an
Identity (model.py:179) and, in infer.py, forces every BatchNorm to batch statistics
(infer.py:105-109 deactivate_batchnorm); both are mirrored here.

ImageNet weights cannot be downloaded offline: `pretrained=True` builds the same architecture
with random initialisation and warns (load a checkpoint to get trained weights).

The stem `maxpool(relu(bn1(conv1(x))))` goes through `features.run_stem` (one fused MFMA
convolution + statistics + BN/ReLU/pool call on the GPU) and every
`relu?(bn(conv(x)) [+ identity])` of the blocks goes through `features.conv_bn_act`: on the GPU
with channels-last bf16 activations that is the MFMA implicit-GEMM convolution (which also emits
the BN batch statistics of its output) and one fused HIP BatchNorm(+add)(+ReLU)
(include/mcgmil_features.h). A block's first `relu(bn1(.))` is not materialised where the next
convolution is a 3x3 / stride 1 halo kernel: that convolution applies it to its input patch
(features.DeferredBN, mcgmil_conv_args.in_ab). Elsewhere (CPU, autograd, fp32) they are the
torch layers.
"""
import warnings

import torch
import torch.nn as nn

from .features import conv_bn_act, run_stem


class Identity(nn.Module):
    """reference model.py:16-21."""

    def forward(self, x):
        return x


def deactivate_batchnorm(net):
    """reference infer.py:105-109: BatchNorm2d layers use the statistics of the bag itself."""
    if isinstance(net, nn.BatchNorm2d):
        net.track_running_stats = False
        net.running_mean = None
        net.running_var = None


def _identity(down, x):
    """The block's shortcut: x, or downsample = Sequential(conv1x1, BatchNorm2d) (no ReLU)."""
    if down is None:
        return x
    if isinstance(down, nn.Sequential) and len(down) == 2 and isinstance(down[1], nn.BatchNorm2d):
        return conv_bn_act(down[0], down[1], x, False, as_residual=True)   # maybe deferred
    return down(x)


def _conv3x3(i, o, stride=1):
    return nn.Conv2d(i, o, 3, stride, 1, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        idt = _identity(self.downsample, x)
        y = conv_bn_act(self.conv1, self.bn1, x, True, consumer=self.conv2)   # maybe deferred
        return conv_bn_act(self.conv2, self.bn2, y, True, idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = _conv3x3(planes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = _identity(self.downsample, x)
        y = conv_bn_act(self.conv1, self.bn1, x, True, consumer=self.conv2)   # maybe deferred
        y = conv_bn_act(self.conv2, self.bn2, y, True, consumer=self.conv3)
        return conv_bn_act(self.conv3, self.bn3, y, True, idt)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def _make(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride,
                                           bias=False), nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = run_stem(self.conv1, self.bn1, self.maxpool, x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


_ARCH = {"r18": (BasicBlock, [2, 2, 2, 2]), "r34": (BasicBlock, [3, 4, 6, 3]),
         "r50": (Bottleneck, [3, 4, 6, 3])}


def build_backbone(backbone: str = "r18", pretrained: bool = True) -> ResNet:
    """The reference's feature_extractor (model.py:166-177), fc left for the caller to replace."""
    if backbone not in _ARCH:
        raise ValueError(f"unknown backbone {backbone!r} (expected r18, r34 or r50)")
    if pretrained:
        warnings.warn("ImageNet weights cannot be downloaded offline; the backbone is randomly "
                      "initialised -- load a checkpoint for trained weights", stacklevel=3)
    block, layers = _ARCH[backbone]
    return ResNet(block, layers)
