"""``nn.Module`` surface of the combined model's branches (SURVEY.md §8b "What callers touch").

The reference's callers reach into the branches of ``CombinedModel`` (modify_models.py:462-494)
beyond ``forward``:
  * ``model.yolo_face.parameters()`` / ``model.yolo_person.parameters()``
    (face_detection/module_v2.py:510, person_detection/module_v2.py, ``configure_optimizers``);
  * ``model.vit_pose.adapter.parameters()`` and ``model.vit_pose.vit_pose.parameters()``
    (pose_estimation/module.py:655,664);
  * ``model.ada_face.adapter.parameters()`` and ``model.ada_face.parameters()``
    (face_recognition/module.py:179-180); ``model.ada_face.head.kernel`` (:137);
  * ``model.yolo_*.yolo.head.stride`` (a plain attribute of yolopt's ``Head``, nn.py:238).

``ParamTree`` rebuilds that hierarchy from the state_dict: one child module per dotted path
component (numeric names like ``adapter.0`` included), every tensor registered as a parameter
or, for the reference's buffers (BatchNorm running statistics, AdaFace head statistics), as a
buffer -- so ``named_parameters()`` / ``state_dict()`` of each branch carry the reference's
own names, sharing storage with the state_dict the engine packed. These trees are the
parameter surface only: the HIP engine computes from its packed copies, so a changed
parameter takes effect after ``CombinedModel.load_state_dict`` (eval hot path; training is
out of scope).
"""
from __future__ import annotations

import torch
import torch.nn as nn

# state_dict leaves that are buffers in the reference modules (BatchNorm*, AdaFace head)
_BUFFERS = {"running_mean", "running_var", "num_batches_tracked", "t", "batch_mean", "batch_std"}


class ParamTree(nn.Module):
    """A node of the parameter hierarchy; ``forward`` is not defined (no compute here)."""

    def child(self, name: str) -> "ParamTree":
        m = self._modules.get(name)
        if m is None:
            m = ParamTree()
            self.add_module(name, m)
        return m


def build_tree(sd: dict, prefix: str, root: nn.Module | None = None) -> nn.Module:
    """Module tree of every ``sd`` entry under ``prefix + '.'`` (names relative to it)."""
    root = ParamTree() if root is None else root
    pre = prefix + "."
    for key, t in sd.items():
        if not key.startswith(pre):
            continue
        parts = key[len(pre):].split(".")
        node = root
        for p in parts[:-1]:
            node = node.child(p) if isinstance(node, ParamTree) else _child(node, p)
        leaf = parts[-1]
        if leaf in _BUFFERS or not torch.is_floating_point(t):
            node.register_buffer(leaf, t)
        else:
            node.register_parameter(leaf, nn.Parameter(t, requires_grad=True))
    return root


def _child(node: nn.Module, name: str) -> nn.Module:
    m = node._modules.get(name)
    if m is None:
        m = ParamTree()
        node.add_module(name, m)
    return m


class VitPoseModule(ParamTree):
    """``model.vit_pose.vit_pose``: transformers' ``VitPoseForPoseEstimation`` as the reference
    wraps it (modify_models.py:383-385). Calling it runs the HIP ViTPose-B on ``pixel_values``
    [B,3,256,192] (BASELINE config 3) and returns an object with ``.heatmaps`` [B,17,64,48]
    (site-packages modeling_vitpose.py:190-278)."""

    def __init__(self, owner):
        super().__init__()
        object.__setattr__(self, "_owner", owner)   # the CombinedModel (not a submodule)

    def forward(self, pixel_values, labels=None, **kw):
        if labels is not None:
            raise NotImplementedError("training loss of VitPoseForPoseEstimation is out of scope (eval only)")
        return self._owner.vitpose_from_pixels(pixel_values)


class YoloModule(ParamTree):
    """``model.yolo_face.yolo`` / ``model.yolo_person.yolo``: the yolopt ``YOLO`` inside
    ``CustomYOLO`` (modify_models.py:61-106). Calling it runs the HIP YOLO v11n (net -> fpn ->
    head, eval) on frames [B,3,H,W] and returns [B, 4+nc, A] (nn.py:294-297; A = 8400 at
    640x640: the config-2 micro-bench variant), with ``head.stride`` as set on this module."""

    def __init__(self, owner, branch):
        super().__init__()
        object.__setattr__(self, "_owner", owner)
        object.__setattr__(self, "_branch", branch)

    def forward(self, x):
        return self._owner.yolo_from_frames(self._branch, x)


def branch_trees(sd: dict, owner) -> dict:
    """{'yolo_face', 'yolo_person', 'ada_face', 'vit_pose'} -> module trees (see module doc)."""
    out = {}
    for name in ("yolo_face", "yolo_person"):
        t = ParamTree()
        build_tree(sd, name + ".adapter", t.child("adapter"))
        t.add_module("yolo", build_tree(sd, name + ".yolo", YoloModule(owner, name)))
        out[name] = t
    out["ada_face"] = build_tree(sd, "ada_face")
    vit = ParamTree()
    build_tree(sd, "vit_pose.adapter", vit.child("adapter"))
    vit.add_module("vit_pose", build_tree(sd, "vit_pose.vit_pose", VitPoseModule(owner)))
    out["vit_pose"] = vit
    for name in ("yolo_face", "yolo_person"):
        head = out[name].child("yolo").child("head")
        # a plain attribute, not a buffer (nn.py:238): never in state_dict(), zeros after
        # modify_yolo's head swap (modify_models.py:168-178) -> eval boxes are 0
        object.__setattr__(head, "stride", torch.zeros(3))
    if "kernel" not in out["ada_face"].child("head")._parameters:
        object.__setattr__(out["ada_face"].child("head"), "kernel", None)
    return out
