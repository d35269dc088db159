"""ORACLE (test infrastructure only) — fp32 PyTorch-CPU restatement of the reference
per-frame inference hot path, written functionally over the reference state_dict.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / CPU baseline. The product path never imports it.

Pinning: oracle/make_golden.py runs the *reference's own classes* (imported with the
shims in oracle/ref_shims.py, container only) on the same seeded weights/inputs and
stores their outputs in tests/golden/; tests/test_oracle_golden.py checks this
restatement against those vectors (tolerance 1e-5 abs, typically bit-exact).

Every function cites the reference code it restates (paths relative to /root/reference;
``site-packages/`` = /usr/local/lib/python3.10/dist-packages/).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor


class Calib:
    """BN calibration recorder: when active, each BN sets its running stats from the
    batch statistics of its input (biased var) before normalising (used once by
    oracle/make_calibration.py to produce prpe/data/bn_calib_seed1.npz)."""

    def __init__(self):
        self.stats = {}


def _bn(sd, p, x, eps=1e-5, calib: Calib | None = None):
    """nn.BatchNorm2d / BatchNorm1d in eval mode (running statistics)."""
    if calib is not None:
        dims = [0] + list(range(2, x.dim()))
        mean = x.mean(dim=dims)
        var = x.var(dim=dims, unbiased=False)
        if x.dim() == 2:   # BatchNorm1d on a tiny batch: uniform variance across channels
            var = torch.full_like(var, float(var.mean()))
        sd[p + ".running_mean"] = mean.detach().clone()
        sd[p + ".running_var"] = var.detach().clone()
        calib.stats[p + ".running_mean"] = sd[p + ".running_mean"]
        calib.stats[p + ".running_var"] = sd[p + ".running_var"]
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"],
                        sd.get(p + ".weight"), sd.get(p + ".bias"), False, 0.0, eps)


def _conv(sd, p, x, stride=1, padding=0, groups=1):
    return F.conv2d(x, sd[p + ".weight"], sd.get(p + ".bias"), stride, padding, 1, groups)


# ----------------------------------------------------------------------------- trunk
def resnet50_trunk(sd, x, calib=None):
    """MultiTaskResNetFeatureExtractor.forward (training/modify_models.py:427-437) over
    torchvision resnet50 v1.5 (modify_models.py:446): stem 7x7/2, maxpool 3/2,
    bottlenecks [3,4,6,3], stride on the 3x3, BN eps 1e-5."""
    p = "backbone"
    x = F.relu(_bn(sd, p + ".bn1", _conv(sd, p + ".conv1", x, 2, 3), calib=calib))
    x = F.max_pool2d(x, 3, 2, 1)
    for li, (planes, blocks, stride) in enumerate(((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)), 1):
        for b in range(blocks):
            q = f"{p}.layer{li}.{b}"
            s = stride if b == 0 else 1
            o = F.relu(_bn(sd, q + ".bn1", _conv(sd, q + ".conv1", x), calib=calib))
            o = F.relu(_bn(sd, q + ".bn2", _conv(sd, q + ".conv2", o, s, 1), calib=calib))
            o = _bn(sd, q + ".bn3", _conv(sd, q + ".conv3", o), calib=calib)
            idt = x
            if b == 0:
                idt = _bn(sd, q + ".downsample.1", _conv(sd, q + ".downsample.0", x, s), calib=calib)
            x = F.relu(o + idt)
    return x


# ----------------------------------------------------------------------------- YOLO
def _yc(sd, p, x, k, s=1, g=1, act="silu", calib=None):
    """yolopt ``Conv``: conv(no bias) -> BN(eps 1e-3) -> act (nn.py:28-36)."""
    y = _bn(sd, p + ".norm", _conv(sd, p + ".conv", x, s, k // 2, g), eps=1e-3, calib=calib)
    return F.silu(y) if act == "silu" else y


def _residual(sd, p, x, calib):          # nn.py:42-49
    return x + _yc(sd, p + ".conv2", _yc(sd, p + ".conv1", x, 3, calib=calib), 3, calib=calib)


def _cspmodule(sd, p, x, calib):         # nn.py:52-63
    y = _yc(sd, p + ".conv1", x, 1, calib=calib)
    y = _residual(sd, p + ".res_m.1", _residual(sd, p + ".res_m.0", y, calib), calib)
    return _yc(sd, p + ".conv3", torch.cat((y, _yc(sd, p + ".conv2", x, 1, calib=calib)), 1), 1, calib=calib)


def _csp(sd, p, x, csp, calib):          # nn.py:66-80 (n = 1 everywhere in v11n)
    y = list(_yc(sd, p + ".conv1", x, 1, calib=calib).chunk(2, 1))
    m = _cspmodule if csp else _residual
    y.append(m(sd, p + ".res_m.0", y[-1], calib))
    return _yc(sd, p + ".conv2", torch.cat(y, 1), 1, calib=calib)


def _spp(sd, p, x, calib):               # nn.py:83-94
    x = _yc(sd, p + ".conv1", x, 1, calib=calib)
    y1 = F.max_pool2d(x, 5, 1, 2)
    y2 = F.max_pool2d(y1, 5, 1, 2)
    y3 = F.max_pool2d(y2, 5, 1, 2)
    return _yc(sd, p + ".conv2", torch.cat([x, y1, y2, y3], 1), 1, calib=calib)


def _psa_attention(sd, p, x, num_head, calib):   # nn.py:97-123
    b, c, h, w = x.shape
    dh = c // num_head
    dk = dh // 2
    scale = dk ** -0.5
    qkv = _yc(sd, p + ".qkv", x, 1, act=None, calib=calib).view(b, num_head, dk * 2 + dh, h * w)
    q, k, v = qkv.split([dk, dk, dh], dim=2)
    attn = ((q.transpose(-2, -1) @ k) * scale).softmax(dim=-1)
    y = (v @ attn.transpose(-2, -1)).view(b, c, h, w) + \
        _yc(sd, p + ".conv1", v.reshape(b, c, h, w), 3, g=c, act=None, calib=calib)
    return _yc(sd, p + ".conv2", y, 1, act=None, calib=calib)


def _psa(sd, p, x, calib):               # nn.py:139-148: PSABlock(ch // 2, num_head=ch // 128)
    a, y = _yc(sd, p + ".conv1", x, 1, calib=calib).chunk(2, 1)
    q = p + ".res_m.0"
    y = y + _psa_attention(sd, q + ".conv1", y, x.shape[1] // 128, calib)
    y = y + _yc(sd, q + ".conv2.1", _yc(sd, q + ".conv2.0", y, 1, calib=calib), 1, act=None, calib=calib)
    return _yc(sd, p + ".conv2", torch.cat((a, y), 1), 1, calib=calib)


def make_anchors(feats, strides, offset=0.5):    # yolopt/util.py:85-96
    anchors, stride_t = [], []
    for f, s in zip(feats, strides):
        _, _, h, w = f.shape
        sx = torch.arange(w, dtype=f.dtype) + offset
        sy = torch.arange(h, dtype=f.dtype) + offset
        sy, sx = torch.meshgrid(sy, sx, indexing="ij")
        anchors.append(torch.stack((sx, sy), -1).view(-1, 2))
        stride_t.append(torch.full((h * w, 1), float(s), dtype=f.dtype))
    return torch.cat(anchors), torch.cat(stride_t)


def yolo_branch(sd, p, feat, stride=(0.0, 0.0, 0.0), calib=None):
    """CustomYOLO.forward in eval mode (modify_models.py:76-106, 139-142) ->
    Head eval decode (nn.py:255-270). Returns [B, 4+1, A] = (cx,cy,w,h)*stride, sigmoid(cls).
    ``stride`` defaults to zeros: a fresh ``Head`` after ``modify_yolo`` (nn.py:238)."""
    a = p + ".adapter"
    x = F.silu(_bn(sd, a + ".1", _conv(sd, a + ".0", feat), calib=calib))
    x = F.interpolate(x, size=(160, 160), mode="bilinear", align_corners=True)
    x = F.silu(_bn(sd, a + ".5", _conv(sd, a + ".4", x, 1, 1), calib=calib))
    x = F.silu(_bn(sd, a + ".8", _conv(sd, a + ".7", x), calib=calib))
    x = F.silu(_bn(sd, a + ".11", _conv(sd, a + ".10", x, 1, 1), calib=calib))
    x = F.silu(_bn(sd, a + ".14", _conv(sd, a + ".13", x), calib=calib))
    x = F.silu(_bn(sd, a + ".17", _conv(sd, a + ".16", x, 1, 1), calib=calib))
    x = x - x.mean(dim=(2, 3), keepdim=True)                       # modify_models.py:84-86
    x = x / (x.std(dim=(2, 3), keepdim=True) + 1e-6)
    x = torch.sigmoid(x)
    return yolo_net(sd, p, x, stride, calib)


def yolo_net(sd, p, x, stride=(0.0, 0.0, 0.0), calib=None):
    """yolopt ``YOLO.forward`` in eval mode (nn.py:294-297: net -> fpn -> head) on NCHW input:
    the adapter's [B,3,160,160] (A = 525) or raw [B,3,640,640] frames (A = 8400, the config-2
    micro-bench variant)."""
    n = p + ".yolo.net"
    x = _yc(sd, n + ".p1.0", x, 3, 2, calib=calib)
    x = _csp(sd, n + ".p2.1", _yc(sd, n + ".p2.0", x, 3, 2, calib=calib), False, calib)
    p3 = _csp(sd, n + ".p3.1", _yc(sd, n + ".p3.0", x, 3, 2, calib=calib), False, calib)
    p4 = _csp(sd, n + ".p4.1", _yc(sd, n + ".p4.0", p3, 3, 2, calib=calib), True, calib)
    p5 = _csp(sd, n + ".p5.1", _yc(sd, n + ".p5.0", p4, 3, 2, calib=calib), True, calib)
    p5 = _psa(sd, n + ".p5.3", _spp(sd, n + ".p5.2", p5, calib), calib)
    f = p + ".yolo.fpn"                                             # nn.py:203-209
    up = lambda t: F.interpolate(t, scale_factor=2.0, mode="nearest")
    p4 = _csp(sd, f + ".h1", torch.cat([up(p5), p4], 1), False, calib)
    p3 = _csp(sd, f + ".h2", torch.cat([up(p4), p3], 1), False, calib)
    p4 = _csp(sd, f + ".h4", torch.cat([_yc(sd, f + ".h3", p3, 3, 2, calib=calib), p4], 1), False, calib)
    p5 = _csp(sd, f + ".h6", torch.cat([_yc(sd, f + ".h5", p4, 3, 2, calib=calib), p5], 1), True, calib)
    h = p + ".yolo.head"
    outs = []
    for i, xi in enumerate((p3, p4, p5)):
        bx = _yc(sd, f"{h}.box.{i}.1", _yc(sd, f"{h}.box.{i}.0", xi, 3, calib=calib), 3, calib=calib)
        bx = _conv(sd, f"{h}.box.{i}.2", bx)
        c = xi.shape[1]
        cl = _yc(sd, f"{h}.cls.{i}.0", xi, 3, g=c, calib=calib)
        cl = _yc(sd, f"{h}.cls.{i}.1", cl, 1, calib=calib)
        cl = _yc(sd, f"{h}.cls.{i}.2", cl, 3, g=80, calib=calib)
        cl = _yc(sd, f"{h}.cls.{i}.3", cl, 1, calib=calib)
        cl = _conv(sd, f"{h}.cls.{i}.4", cl)
        outs.append(torch.cat((bx, cl), 1))
    anchors, strides = (t.transpose(0, 1) for t in make_anchors(outs, stride))
    b = outs[0].shape[0]
    no = outs[0].shape[1]
    x = torch.cat([o.view(b, no, -1) for o in outs], 2)
    box, cls = x.split((64, no - 64), 1)
    # DFL (nn.py:212-225): softmax over 16 bins, 1x1 conv with weight arange(16)
    aa = box.shape[2]
    d = box.view(b, 4, 16, aa).transpose(2, 1).softmax(1)
    d = F.conv2d(d, sd[h + ".dfl.conv.weight"]).view(b, 4, aa)
    lt, rb = d.chunk(2, 1)
    a1 = anchors.unsqueeze(0) - lt
    b1 = anchors.unsqueeze(0) + rb
    box = torch.cat(((a1 + b1) / 2, b1 - a1), 1)
    return torch.cat((box * strides, cls.sigmoid()), 1)


# ----------------------------------------------------------------------------- AdaFace
# IR-50 unit list (libs/net_adaface.py:222-243, get_block: first unit strided)
_IR50_UNITS = []
for _cin, _d, _n in ((64, 64, 3), (64, 128, 4), (128, 256, 14), (256, 512, 3)):
    _IR50_UNITS += [(_cin, _d, 2)] + [(_d, _d, 1)] * (_n - 1)


def adaface_branch(sd, feat, calib=None):
    """CustomAdaFace.forward without labels (modify_models.py:288-297): adapter ->
    IR-50 (libs/net_adaface.py:144-167, 322-337) -> (x/||x||, ||x||)."""
    a = "ada_face.adapter"
    pr = lambda t, q: F.prelu(t, sd[q + ".weight"])
    x = pr(_bn(sd, a + ".1", _conv(sd, a + ".0", feat), calib=calib), a + ".2")
    x = F.interpolate(x, size=(112, 112), mode="bilinear", align_corners=True)
    x = pr(_bn(sd, a + ".5", _conv(sd, a + ".4", x, 1, 1), calib=calib), a + ".6")
    x = pr(_bn(sd, a + ".8", _conv(sd, a + ".7", x, 1, 1), calib=calib), a + ".9")
    x = pr(_bn(sd, a + ".11", _conv(sd, a + ".10", x, 1, 1), calib=calib), a + ".12")
    m = "ada_face.adaface_model"
    x = pr(_bn(sd, m + ".input_layer.1", _conv(sd, m + ".input_layer.0", x, 1, 1), calib=calib),
           m + ".input_layer.2")
    for i, (cin, d, st) in enumerate(_IR50_UNITS):
        p = f"{m}.body.{i}"
        if cin == d:
            sc = F.max_pool2d(x, 1, st)
        else:
            sc = _bn(sd, p + ".shortcut_layer.1", _conv(sd, p + ".shortcut_layer.0", x, st), calib=calib)
        r = _bn(sd, p + ".res_layer.0", x, calib=calib)
        r = _conv(sd, p + ".res_layer.1", r, 1, 1)
        r = pr(_bn(sd, p + ".res_layer.2", r, calib=calib), p + ".res_layer.3")
        r = _bn(sd, p + ".res_layer.5", _conv(sd, p + ".res_layer.4", r, st, 1), calib=calib)
        x = r + sc
    x = _bn(sd, m + ".output_layer.0", x, calib=calib)
    x = x.reshape(x.shape[0], -1)            # Dropout(0.4) is identity in eval
    x = F.linear(x, sd[m + ".output_layer.3.weight"], sd[m + ".output_layer.3.bias"])
    x = _bn(sd, m + ".output_layer.4", x, calib=calib)
    norm = torch.norm(x, 2, 1, True)
    return torch.div(x, norm), norm


# ----------------------------------------------------------------------------- ViTPose
def _ln(sd, p, x):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], 1e-12)


def vitpose_backbone(sd, pixel_values):
    """VitPoseForPoseEstimation.forward (site-packages transformers/models/vitpose/
    modeling_vitpose.py:190-278) with the simple decoder (:120-144); backbone
    modeling_vitpose_backbone.py:43-98 (embeddings), :100-182 (attention), :271-326
    (layer), :380-438 (final LN). Returns heatmaps [B,17,64,48]."""
    v = "vit_pose.vit_pose.backbone"
    x = F.conv2d(pixel_values, sd[v + ".embeddings.patch_embeddings.projection.weight"],
                 sd[v + ".embeddings.patch_embeddings.projection.bias"], 16, 2)
    b = x.shape[0]
    x = x.flatten(2).transpose(1, 2)
    pos = sd[v + ".embeddings.position_embeddings"]
    x = x + pos[:, 1:] + pos[:, :1]
    nh, dh = 12, 64
    for i in range(12):
        L = f"{v}.encoder.layer.{i}"
        hn = _ln(sd, L + ".layernorm_before", x)
        A = L + ".attention.attention"
        shp = (b, -1, nh, dh)
        k = F.linear(hn, sd[A + ".key.weight"], sd[A + ".key.bias"]).view(*shp).transpose(1, 2)
        vv = F.linear(hn, sd[A + ".value.weight"], sd[A + ".value.bias"]).view(*shp).transpose(1, 2)
        q = F.linear(hn, sd[A + ".query.weight"], sd[A + ".query.bias"]).view(*shp).transpose(1, 2)
        att = torch.matmul(q, k.transpose(2, 3)) * (dh ** -0.5)
        att = F.softmax(att, dim=-1)
        ctx = torch.matmul(att, vv).transpose(1, 2).contiguous().reshape(b, -1, nh * dh)
        ao = F.linear(ctx, sd[L + ".attention.output.dense.weight"], sd[L + ".attention.output.dense.bias"])
        x = ao + x
        hn = _ln(sd, L + ".layernorm_after", x)
        hn = F.gelu(F.linear(hn, sd[L + ".mlp.fc1.weight"], sd[L + ".mlp.fc1.bias"]))
        x = F.linear(hn, sd[L + ".mlp.fc2.weight"], sd[L + ".mlp.fc2.bias"]) + x
    x = _ln(sd, v + ".layernorm", x)
    x = x.permute(0, 2, 1).reshape(b, -1, 16, 12).contiguous()
    x = F.relu(x)
    x = F.interpolate(x, scale_factor=4.0, mode="bilinear", align_corners=False)
    return F.conv2d(x, sd["vit_pose.vit_pose.head.conv.weight"], sd["vit_pose.vit_pose.head.conv.bias"], 1, 1)


def vitpose_adapter(sd, feat, calib=None):
    """CustomVitPose.adapter (modify_models.py:352-374) -> pixel_values [B,3,256,192]."""
    a = "vit_pose.adapter"
    x = F.gelu(_bn(sd, a + ".1", _conv(sd, a + ".0", feat), calib=calib))
    x = F.interpolate(x, size=(256, 192), mode="bilinear", align_corners=True)
    x = F.gelu(_bn(sd, a + ".5", _conv(sd, a + ".4", x, 1, 1), calib=calib))
    x = F.gelu(_bn(sd, a + ".8", _conv(sd, a + ".7", x, 1, 1), calib=calib))
    x = F.gelu(_bn(sd, a + ".11", _conv(sd, a + ".10", x, 1, 1), calib=calib))
    return x


def vitpose_branch(sd, feat, calib=None):
    return vitpose_backbone(sd, vitpose_adapter(sd, feat, calib))


# ----------------------------------------------------------------------------- model
def combined_forward(sd, x, task, stride=(0.0, 0.0, 0.0)):
    """CombinedModel.forward (modify_models.py:482-494) for one task."""
    feat = resnet50_trunk(sd, x)
    if task == "pose_estimation":
        return vitpose_branch(sd, feat)
    if task == "person_detection":
        return yolo_branch(sd, "yolo_person", feat, stride)
    if task == "face_detection":
        return yolo_branch(sd, "yolo_face", feat, stride)
    return adaface_branch(sd, feat)


def forward_all(sd, x, stride=(8.0, 16.0, 32.0), calib=None):
    """Trunk once, then face-YOLO, AdaFace and ViTPose heads (config 4 of BASELINE.json)."""
    feat = resnet50_trunk(sd, x, calib)
    det = yolo_branch(sd, "yolo_face", feat, stride, calib)
    emb, norm = adaface_branch(sd, feat, calib)
    heat = vitpose_branch(sd, feat, calib)
    return {"feat": feat, "det": det, "emb": emb, "norm": norm, "heatmaps": heat}


# ----------------------------------------------------------------------------- post-proc
def nms_restated(boxes: Tensor, scores: Tensor, iou_threshold: float, max_keep: int | None = None) -> Tensor:
    """torchvision.ops.nms semantics (CPU kernel), restated in numpy float32.

    Greedy: visit boxes by descending score; keep a box unless an already-kept box
    has IoU > thr with it; IoU = inter / (area_i + area_j - inter), all in float32.
    Ties: torchvision sorts with ``scores.sort(descending=True)`` whose CPU order for
    equal scores is unspecified (not stable above ~16 elements); this restatement breaks
    ties by index (stable), which is the contract of the HIP kernel too.
    ``max_keep``: stop after that many kept boxes -- the greedy pass is sequential in score
    order, so the first max_keep kept indices are the same as the full result's.
    """
    b = boxes.detach().cpu().numpy().astype(np.float32)
    s = scores.detach().cpu().numpy().astype(np.float32)
    n = b.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.int64)
    order = np.argsort(-s, kind="stable")
    x1, y1, x2, y2 = (b[order, i] for i in range(4))
    areas = (x2 - x1) * (y2 - y1)
    alive = np.ones(n, dtype=bool)
    keep = []
    for i in range(n):
        if not alive[i]:
            continue
        keep.append(order[i])
        if max_keep is not None and len(keep) >= max_keep:
            break
        j = np.arange(i + 1, n)
        j = j[alive[i + 1:]]
        if j.size == 0:
            break
        xx1 = np.maximum(x1[i], x1[j]); yy1 = np.maximum(y1[i], y1[j])
        xx2 = np.minimum(x2[i], x2[j]); yy2 = np.minimum(y2[i], y2[j])
        w = np.maximum(np.float32(0), xx2 - xx1); h = np.maximum(np.float32(0), yy2 - yy1)
        inter = w * h
        with np.errstate(divide="ignore", invalid="ignore"):
            ovr = inter / (areas[i] + areas[j] - inter)
        alive[j[ovr > np.float32(iou_threshold)]] = False
    return torch.as_tensor(np.array(keep, dtype=np.int64))


def nms_single(boxes: Tensor, scores: Tensor, thr: float, max_keep: int | None = None) -> Tensor:
    """torchvision.ops.nms semantics (CPU kernel), called at yolopt/util.py:162:
    stable descending score order, suppress j iff IoU(i, j) > thr."""
    return nms_restated(boxes, scores, thr, max_keep)


def non_max_suppression(outputs: Tensor, confidence_threshold=0.001, iou_threshold=0.65):
    """yolopt.util.non_max_suppression (training/yolopt/util.py:123-169) without the
    wall-clock cut-off (:133-134,166-167, non-deterministic). outputs [B, 4+nc, N]."""
    max_wh, max_det, max_nms = 7680, 300, 30000
    bs = outputs.shape[0]
    nc = outputs.shape[1] - 4
    xc = outputs[:, 4:4 + nc].amax(1) > confidence_threshold
    out = [torch.zeros((0, 6))] * bs
    for i, x in enumerate(outputs):
        x = x.transpose(0, -1)[xc[i]]
        if not x.shape[0]:
            continue
        box, cls = x.split((4, nc), 1)
        xy = box.clone()
        xy[:, 0] = box[:, 0] - box[:, 2] / 2
        xy[:, 1] = box[:, 1] - box[:, 3] / 2
        xy[:, 2] = box[:, 0] + box[:, 2] / 2
        xy[:, 3] = box[:, 1] + box[:, 3] / 2
        if nc > 1:
            ii, jj = (cls > confidence_threshold).nonzero(as_tuple=False).T
            x = torch.cat((xy[ii], x[ii, 4 + jj, None], jj[:, None].float()), 1)
        else:
            conf, j = cls.max(1, keepdim=True)
            x = torch.cat((xy, conf, j.float()), 1)[conf.view(-1) > confidence_threshold]
        if not x.shape[0]:
            continue
        # stable descending sort: ties by index (the reference's torch CPU argsort
        # leaves tie order unspecified; identical for tie-free scores)
        x = x[torch.sort(x[:, 4], descending=True, stable=True)[1][:max_nms]]
        c = x[:, 5:6] * max_wh
        keep = nms_single(x[:, :4] + c, x[:, 4], iou_threshold, max_det)[:max_det]
        out[i] = x[keep]
    return out


def keypoints_from_heatmaps(heatmaps: Tensor, boxes: Tensor | None = None):
    """PoseEstimationModule._get_keypoints_from_heatmaps
    (training/lightning/pose_estimation/module.py:237-296): soft-argmax."""
    B, K, H, W = heatmaps.shape
    yg, xg = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32),
                            indexing="ij")
    prob = F.softmax(heatmaps.reshape(B, K, -1), dim=2).reshape(B, K, H, W)
    xe = (prob * xg[None, None]).sum(dim=(2, 3)) + 0.5
    ye = (prob * yg[None, None]).sum(dim=(2, 3)) + 0.5
    scores = prob.reshape(B, K, -1).max(dim=2)[0]
    coords = torch.stack([xe, ye], dim=-1)
    coords[..., 0] = coords[..., 0] / W
    coords[..., 1] = coords[..., 1] / H
    if boxes is not None:
        area = (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])
        sw = torch.clamp(torch.sqrt(area).view(-1, 1, 1) / 96.0, min=0.5, max=2.0)
        scores = scores * sw.squeeze(-1)
    return coords, scores


COCO_SIGMAS = [0.026, 0.025, 0.025, 0.035, 0.035, 0.079, 0.079, 0.072, 0.072,
               0.062, 0.062, 0.107, 0.107, 0.087, 0.087, 0.089, 0.089]


def oks_delta(coords_a: Tensor, coords_b: Tensor, h=256, w=192) -> float:
    """1 - OKS between two keypoint sets in [0,1] crop coordinates."""
    s = torch.tensor(COCO_SIGMAS, dtype=torch.float64)
    da = coords_a.double() * torch.tensor([w, h], dtype=torch.float64)
    db = coords_b.double() * torch.tensor([w, h], dtype=torch.float64)
    d2 = ((da - db) ** 2).sum(-1)
    area = float(h * w)
    oks = torch.exp(-d2 / (2 * area * (2 * s) ** 2)).mean(-1)
    return float((1 - oks).max())


# ---------------------------------------------------------------- eval steps
COCO_FLIP_PAIRS = [(1, 2), (3, 4), (5, 6), (7, 8), (9, 10), (11, 12), (13, 14), (15, 16)]  # datamodule.py:25-34


def pose_flip_average(pred_heatmaps: Tensor, flipped_output_heatmaps: Tensor, mode: str = "reference") -> Tensor:
    """pose_estimation/module.py:476-484: flip the flipped pass's heatmaps back along W, apply
    the pair handling, average. ``reference`` keeps the code's ``[:, pair].flip(0)`` (a batch
    reversal of the paired channels); ``swap`` exchanges the pair's channels instead."""
    flipped = torch.flip(flipped_output_heatmaps, dims=[-1])
    for pair in COCO_FLIP_PAIRS:
        if mode == "reference":
            flipped[:, pair] = flipped[:, pair].flip(0)
        else:
            flipped[:, pair] = flipped[:, pair].flip(1)
    return (pred_heatmaps + flipped) * 0.5


def face_recognition_eval(embeddings: Tensor, head_kernel: Tensor, labels: Tensor, s: float = 64.0):
    """face_recognition/module.py:137-145: cosine logits against the row-normalised head
    kernel (F.normalize default dim=1 on the [512, classes] kernel), scaled by s, then
    cross-entropy and top-1 accuracy. Returns (loss, acc, output, argmax)."""
    kernel = F.normalize(head_kernel)
    cosine = F.linear(F.normalize(embeddings), kernel.t())
    output = cosine * s
    loss = F.cross_entropy(output, labels)
    amax = output.max(1)[1]
    acc = (amax == labels).float().mean()
    return loss, acc, output, amax


class DetectionMetricsRef:
    """DetectionMetrics (training/lightning/face_detection/module_v2.py:13-127) restated, as
    driven by FaceDetectionModule.validation_step (:480-499): test infrastructure only."""

    def __init__(self):
        self.tp = self.fp = self.gt = 0
        self.records = []                      # (score, is_tp, iou), insertion order

    @staticmethod
    def box_iou(b1: Tensor, b2: Tensor) -> Tensor:                    # :27-45
        a1 = (b1[:, 2] - b1[:, 0]) * (b1[:, 3] - b1[:, 1])
        a2 = (b2[:, 2] - b2[:, 0]) * (b2[:, 3] - b2[:, 1])
        lt = torch.max(b1[:, None, :2], b2[:, :2])
        rb = torch.min(b1[:, None, 2:], b2[:, 2:])
        wh = (rb - lt).clamp(min=0)
        inter = wh[:, :, 0] * wh[:, :, 1]
        union = a1[:, None] + a2 - inter
        return inter / (union + 1e-6)

    def update_batch(self, preds: list, gt_boxes: Tensor, batch_idx: Tensor):   # :480-499 + :47-78
        for i, pred in enumerate(preds):
            if len(pred) == 0:
                continue
            g = gt_boxes[batch_idx == i]
            if len(g) == 0:
                continue
            best = self.box_iou(pred[:, :4], g).max(dim=1)[0]
            for s, v in zip(pred[:, 4].tolist(), best.tolist()):
                t = v > 0.5
                self.tp += int(t)
                self.fp += int(not t)
                self.records.append((s, t, v))
            self.gt += len(g)

    def compute(self) -> dict:                                          # :80-127
        precision = self.tp / (self.tp + self.fp + 1e-6)
        recall = self.tp / (self.gt + 1e-6)
        f1 = 2 * (precision * recall) / (precision + recall + 1e-6)
        aps = []
        for thr in torch.linspace(0.5, 0.95, 10):
            kept = [r for r in self.records if r[2] >= thr]
            if not kept:
                aps.append(0.0)
                continue
            kept = sorted(kept, key=lambda x: x[0], reverse=True)
            tp = torch.tensor([x[1] for x in kept])
            tpc, fpc = torch.cumsum(tp, 0), torch.cumsum(~tp, 0)
            rec = torch.cat((torch.tensor([0]), tpc / (self.gt + 1e-6), torch.tensor([1])))
            prec = torch.cat((torch.tensor([1]), tpc / (tpc + fpc + 1e-6), torch.tensor([0])))
            aps.append(torch.trapz(prec, rec).item())
        return {"precision": precision, "recall": recall, "f1": f1, "mAP50": aps[0], "mAP75": aps[5],
                "mAP": sum(aps) / len(aps)}


def compute_iou_ref(box1: Tensor, box2: Tensor, eps=1e-7, CIoU=False) -> Tensor:
    """training/lightning/utils.py:8-76 restated (pairwise [N, M])."""
    b1 = box1.unsqueeze(1)
    b2 = box2.unsqueeze(0)
    b1x1, b1y1, b1x2, b1y2 = b1.split(1, dim=-1)
    b2x1, b2y1, b2x2, b2y2 = b2.split(1, dim=-1)
    w1, h1, w2, h2 = b1x2 - b1x1, b1y2 - b1y1, b2x2 - b2x1, b2y2 - b2y1
    area1 = w1.clamp(min=0) * h1.clamp(min=0)
    area2 = w2.clamp(min=0) * h2.clamp(min=0)
    iw = (torch.minimum(b1x2, b2x2) - torch.maximum(b1x1, b2x1)).clamp(min=0)
    ih = (torch.minimum(b1y2, b2y2) - torch.maximum(b1y1, b2y1)).clamp(min=0)
    inter = iw * ih
    iou = inter / (area1 + area2 - inter + eps)
    if not CIoU:
        return iou.squeeze(-1)
    cw = torch.maximum(b1x2, b2x2) - torch.minimum(b1x1, b2x1)
    ch = torch.maximum(b1y2, b2y2) - torch.minimum(b1y1, b2y1)
    c2 = (cw ** 2 + ch ** 2) + eps
    rho2 = ((b1x1 + b1x2 - b2x1 - b2x2) ** 2 + (b1y1 + b1y2 - b2y1 - b2y2) ** 2) / 4
    v = (4 / (math.pi ** 2)) * torch.pow(torch.atan(w2 / (h2 + eps)) - torch.atan(w1 / (h1 + eps)), 2)
    alpha = v / (v - iou + (1 + eps))
    return (iou - (rho2 / c2 + v * alpha)).squeeze(-1)


def detection_eval_loss_ref(pred_boxes: Tensor, pred_scores: Tensor, gt_boxes: Tensor, gt_labels: Tensor,
                            batch_idx: Tensor):
    """FaceDetectionModule.compute_loss (module_v2.py:178-303) restated: returns (avg_loss,
    {image: (loss_b, box, cls, bg)}) with NaN for terms the reference does not compute."""
    B = pred_boxes.shape[0]
    if pred_boxes.shape[1] == 4:
        pred_boxes = pred_boxes.transpose(1, 2)
        pred_scores = pred_scores.transpose(1, 2)
    max_scores, _ = pred_scores.max(dim=-1)
    total = 0
    per = {}
    nan = float("nan")
    for b in range(B):
        mask = batch_idx == b
        if not mask.any():
            continue
        g, gl = gt_boxes[mask], gt_labels[mask]
        conf = max_scores[b] > 0.01
        pb, ps = pred_boxes[b, conf], pred_scores[b, conf]
        if len(pb) == 0 or len(g) == 0:
            if len(pb) > 0:
                bg = F.binary_cross_entropy_with_logits(ps.max(dim=-1)[0], torch.zeros_like(ps.max(dim=-1)[0]))
                total += bg
                per[b] = (bg.item(), nan, nan, bg.item())
            continue
        ious = compute_iou_ref(pb, g)
        best, idx = ious.max(dim=1)
        pos = best > 0.5
        if pos.any():
            box = -compute_iou_ref(pb[pos], g[idx[pos]], CIoU=True).mean()
            cls = F.cross_entropy(ps[pos], gl[idx[pos]])
            bgv = ps[~pos].max(dim=-1)[0]
            bg = F.binary_cross_entropy_with_logits(bgv, torch.zeros_like(bgv))
            lb = box + cls + 0.5 * bg
            total += lb
            per[b] = (lb.item(), box.item(), cls.item(), bg.item())
        else:
            bg = F.binary_cross_entropy_with_logits(ps.max(dim=-1)[0], torch.zeros_like(ps.max(dim=-1)[0]))
            total += bg
            per[b] = (bg.item(), nan, nan, bg.item())
    return total / B, per
