"""Import shims that let the *reference* code under /root/reference be imported in
this container (CONTAINER-ONLY test infrastructure; never shipped, never imported by
the product path, never run on the GPU box).

The reference depends on packages that are absent here:
  * torchvision  -> ``models.resnet50`` (called at training/modify_models.py:446) and
                    ``ops.nms`` (called at training/yolopt/util.py:162).
  * pytorch_lightning, pycocotools, albumentations, cv2, wandb -> inert stubs, only so
    the Lightning modules that hold the eval-step post-processing can be imported
    (training/lightning/pose_estimation/module.py, face_detection/module_v2.py).

The two torchvision pieces are restated here from torchvision's *published* behaviour
(torchvision is unpinned in requirements.txt:6):
  * resnet50: ResNet v1.5 (stride on the 3x3 conv of the bottleneck), layers [3,4,6,3],
    BN eps 1e-5, identical state_dict keys.
  * nms: greedy, boxes sorted by score descending (stable), suppress j when
    IoU(i,j) > thr, area = (x2-x1)*(y2-y1); returns kept indices in score order.

``transformers`` must be imported before the torchvision shim is installed, because
its ``find_spec('torchvision')`` probe breaks on a module without a spec.
"""
from __future__ import annotations

import sys
import types

import numpy as np
import torch
import torch.nn as nn

REFERENCE_ROOT = "/root/reference"


# ----------------------------------------------------------------------------------
# torchvision.models.resnet50 (v1.5 bottleneck), state_dict-compatible
# ----------------------------------------------------------------------------------
class _Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            idt = self.downsample(x)
        return self.relu(out + idt)


class _ResNet50(nn.Module):
    def __init__(self):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make(64, 3, 1)
        self.layer2 = self._make(128, 4, 2)
        self.layer3 = self._make(256, 6, 2)
        self.layer4 = self._make(512, 3, 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(2048, 1000)

    def _make(self, planes, blocks, stride):
        ds = None
        if stride != 1 or self.inplanes != planes * 4:
            ds = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                               nn.BatchNorm2d(planes * 4))
        layers = [_Bottleneck(self.inplanes, planes, stride, ds)]
        self.inplanes = planes * 4
        layers += [_Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)


def _resnet50(pretrained=False, **kw):  # pretrained weights need the network: ignored
    return _ResNet50()


# torchvision.ops.nms: restated in oracle/model_ref.py (the oracle ships to the GPU box; this
# container-only shim module does not)
from oracle.model_ref import nms_restated  # noqa: E402


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def install():
    """Install the shims and put the reference's import roots on sys.path."""
    import transformers  # noqa: F401  (must precede the torchvision shim)
    from transformers import VitPoseForPoseEstimation  # noqa: F401

    if "torchvision" not in sys.modules or not hasattr(sys.modules["torchvision"], "_prpe_shim"):
        tv = _stub("torchvision", _prpe_shim=True)
        tv.models = _stub("torchvision.models", resnet50=_resnet50)
        tv.ops = _stub("torchvision.ops", nms=nms_restated)

    class _LM(nn.Module):
        def __init__(self, *a, **k):
            super().__init__()

        def log(self, *a, **k):
            pass

        def log_dict(self, *a, **k):
            pass

        def save_hyperparameters(self, *a, **k):
            pass

    pl = _stub("pytorch_lightning", LightningModule=_LM, LightningDataModule=object, Trainer=object,
               Callback=object)
    pl.callbacks = _stub("pytorch_lightning.callbacks", ModelCheckpoint=object,
                         LearningRateMonitor=object, Callback=object)
    pl.loggers = _stub("pytorch_lightning.loggers", WandbLogger=object)
    pc = _stub("pycocotools")
    pc.coco = _stub("pycocotools.coco", COCO=object)
    pc.cocoeval = _stub("pycocotools.cocoeval", COCOeval=object)
    _stub("albumentations")
    _stub("cv2")
    _stub("wandb")

    for p in (REFERENCE_ROOT + "/training", REFERENCE_ROOT + "/libs", REFERENCE_ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    sys.dont_write_bytecode = True
