"""Test infrastructure: nn.Module restatement of torchvision 0.6.0 ``r2plus1d_18`` (absent from the
image), registered as ``torchvision.models.video`` so the reference's own
``src/model/R2plus1D_18_MotionNet.py`` can be imported and run when generating golden fixtures.
Module/parameter names follow torchvision (stem.0 ... layer4.1.conv2.1, fc), so state-dict keys
match the reference checkpoints. ``pretrained`` is ignored (no network)."""
import sys
import types

import torch.nn as nn


class Conv2Plus1D(nn.Sequential):
    def __init__(self, i, o, m, stride=1, padding=1):
        super().__init__(nn.Conv3d(i, m, (1, 3, 3), (1, stride, stride), (0, padding, padding), bias=False),
                         nn.BatchNorm3d(m), nn.ReLU(inplace=True),
                         nn.Conv3d(m, o, (3, 1, 1), (stride, 1, 1), (padding, 0, 0), bias=False))


class BasicBlock(nn.Module):
    def __init__(self, inp, planes, stride=1, downsample=None):
        super().__init__()
        mid = (inp * planes * 27) // (inp * 9 + 3 * planes)
        self.conv1 = nn.Sequential(Conv2Plus1D(inp, planes, mid, stride), nn.BatchNorm3d(planes), nn.ReLU(inplace=True))
        self.conv2 = nn.Sequential(Conv2Plus1D(planes, planes, mid), nn.BatchNorm3d(planes))
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        r = x
        o = self.conv2(self.conv1(x))
        if self.downsample is not None:
            r = self.downsample(x)
        return self.relu(o + r)


class R2Plus1dStem(nn.Sequential):
    def __init__(self):
        super().__init__(nn.Conv3d(3, 45, (1, 7, 7), (1, 2, 2), (0, 3, 3), bias=False), nn.BatchNorm3d(45),
                         nn.ReLU(inplace=True), nn.Conv3d(45, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0), bias=False),
                         nn.BatchNorm3d(64), nn.ReLU(inplace=True))


class VideoResNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.inplanes = 64
        self.stem = R2Plus1dStem()
        self.layer1 = self._make_layer(64, 1)
        self.layer2 = self._make_layer(128, 2)
        self.layer3 = self._make_layer(256, 2)
        self.layer4 = self._make_layer(512, 2)
        self.avgpool = nn.AdaptiveAvgPool3d((1, 1, 1))
        self.fc = nn.Linear(512, 400)

    def _make_layer(self, planes, stride):
        ds = None
        if stride != 1 or self.inplanes != planes:
            ds = nn.Sequential(nn.Conv3d(self.inplanes, planes, 1, (stride,) * 3, bias=False), nn.BatchNorm3d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, ds)]
        self.inplanes = planes
        layers.append(BasicBlock(planes, planes))
        return nn.Sequential(*layers)


def r2plus1d_18(pretrained=False, progress=True, **kw):
    return VideoResNet()


def install():
    tv = types.ModuleType("torchvision")
    models = types.ModuleType("torchvision.models")
    video = types.ModuleType("torchvision.models.video")
    video.r2plus1d_18 = r2plus1d_18
    tv.models = models
    models.video = video
    sys.modules.update({"torchvision": tv, "torchvision.models": models, "torchvision.models.video": video})
