"""Torch-tensor level wrappers over the C ABI (device buffers come from PyTorch-ROCm).

Tensors are float32 on the GPU with a *logical NHWC* shape [N, H, W, C] and arbitrary
strides (channel slices of concat buffers, NCHW inputs via ``permute``, broadcast
residuals with stride 0 ...). Every call launches on the current torch stream.
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import ACT, RES_NONE, BneckDesc, ConvDesc, PrpeError, StemDesc, View, check, lib


def _stream() -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t) -> int | None:
    return None if t is None else _gpu(t).data_ptr()


def _gpu(*ts):
    """Every tensor handed to the library must live in device memory: a host pointer in a
    kernel is a GPU memory fault, so it is refused here, before the C ABI."""
    for t in ts:
        if t is not None and not (isinstance(t, torch.Tensor) and t.is_cuda):
            raise ValueError(f"prpe: expected a HIP device tensor, got {type(t).__name__} on "
                             f"{getattr(t, 'device', '?')}")
    return ts[0] if len(ts) == 1 else ts


def view(t: torch.Tensor | None) -> View:
    """prpe_view of a 4-D logical-NHWC tensor (or a null view for None)."""
    if t is None:
        return View()
    assert t.dim() == 4 and t.dtype == torch.float32 and t.is_cuda, (t.shape, t.dtype, t.device)
    n, h, w, c = t.shape
    sn, sh, sw, sc = t.stride()
    return View(t.data_ptr(), n, h, w, c, sn, sh, sw, sc)


def nhwc(t: torch.Tensor) -> torch.Tensor:
    """Logical NHWC view of an NCHW tensor (no copy)."""
    return t.permute(0, 2, 3, 1)


def _check_slots(what, n, *slots):
    """max|x| / max|y| slot arrays: contiguous float32 device tensors of at least n (frames)
    entries -- the kernels index them by frame, so a short array would be read or raised out of
    bounds on the device."""
    for a in slots:
        if a is not None and (not isinstance(a, torch.Tensor) or a.dtype != torch.float32 or not a.is_cuda or
                              a.numel() < n or not a.is_contiguous()):
            raise ValueError(f"{what}: max|x| slots must be a contiguous float32 device [N >= {n}]")


def conv2d(x, pack, y, *, res=None, res_mode=RES_NONE, act=None, precision=0, tile=0, x_amax=None,
           y_amax=None, x2=None, x2_amax=None, x_planes=False, y_planes=False, w2=None, y2=None, w3=None,
           scale2=None, bias2=None, act2="none"):
    """y = EPI(conv(PRO(x))) with a ``ConvPack`` (see prpe.pack).

    precision 3 (split fp16) and 4 (one fp16 plane) need ``x_amax``: a [N] device tensor,
    x_amax[n] bounding max|x[n]| per frame (e.g. the ``y_amax`` its producer raised). ``y_amax``
    (any precision): [N] device tensor the kernel raises to max|y[n]| per frame (zero it first)."""
    d = ConvDesc()
    _gpu(pack.w_hi)
    _check_slots(f"prpe_conv2d[{pack.name}]", x.shape[0], x_amax, y_amax, x2_amax)
    if precision in (3, 4):
        h16, l16, s16 = pack.f16_planes()
        d.w_h16, d.w_l16, d.scale16 = h16.data_ptr(), l16.data_ptr(), s16.data_ptr()
        d.x_amax = _ptr(x_amax)
    d.y_amax = _ptr(y_amax)
    d.x_planes, d.y_planes = int(x_planes), int(y_planes)   # planes format, see prpe.h
    if w2 is not None:                 # epilogue 1x1 GEMM (w2 fp32 [n2][Co]) into y2, see prpe.h
        _gpu(w2, y2)
        n_mid = y2.shape[3] if w3 is None else w3.shape[1]
        if w2.dtype != torch.float32 or not w2.is_contiguous() or w2.shape != (n_mid, y.shape[3]):
            raise ValueError(f"prpe_conv2d[{pack.name}]: w2 must be contiguous float32 [n2, Co]")
        d.w2 = w2.data_ptr()
        d.y2 = view(y2)
        if w3 is not None:             # second stage: z1 = act2(scale2 (y' w2^T) + bias2), z = z1 w3^T
            for t, shp in ((w3, (y2.shape[3], n_mid)), (scale2, (n_mid,)), (bias2, (n_mid,))):
                if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.shape != shp):
                    raise ValueError(f"prpe_conv2d[{pack.name}]: w3 [n3, n2] / scale2, bias2 [n2] float32")
            d.w3, d.scale2, d.bias2 = w3.data_ptr(), _ptr(scale2), _ptr(bias2)
            d.act2, d.n2 = ACT[act2], n_mid
    if x2 is not None:                 # second 1x1 input, see prpe.h (dual input)
        d.x2 = view(x2)
        d.x2_amax = _ptr(x2_amax)
    d.x = view(x)
    d.y = view(y)
    d.res = view(res)
    d.kh, d.kw, d.stride, d.pad = pack.kh, pack.kw, pack.stride, pack.pad
    d.w_hi, d.w_lo, d.w_lo2 = pack.w_hi.data_ptr(), pack.w_lo.data_ptr(), pack.w_lo2.data_ptr()
    d.k_pad, d.co_pad = pack.k_pad, pack.co_pad
    d.scale, d.bias, d.slope = _ptr(pack.scale), _ptr(pack.bias), _ptr(pack.slope)
    d.in_scale, d.in_bias = _ptr(pack.in_scale), _ptr(pack.in_bias)
    d.act = ACT[act if act is not None else pack.act]
    d.res_mode = res_mode
    d.precision = precision
    d.tile = tile
    d.k_order = pack.k_order
    # caller-owned scratch (the split-K partial sums; 0 bytes on every other path), from the
    # caching allocator on the current stream, so concurrent streams never share one
    nbytes = lib().prpe_conv2d_workspace_bytes(C.byref(d))
    if nbytes < 0:
        raise PrpeError(f"prpe_conv2d[{pack.name}]: descriptor rejected (status {nbytes})")
    ws = None
    if nbytes:
        ws = torch.empty((nbytes + 255) // 256 * 64, device=y.device, dtype=torch.float32)
        d.workspace, d.workspace_bytes = ws.data_ptr(), nbytes
    check(lib().prpe_conv2d(C.byref(d), _stream()), f"prpe_conv2d[{pack.name}]")
    return y


def bottleneck(x, packs, y, x_amax, y_amax=None):
    """Fused identity-shortcut ResNet bottleneck at precision 3 (prpe_bottleneck, include/prpe.h):
    y = relu(bn3(conv3(relu(bn2(conv2(relu(bn1(conv1 x))))))) + x); ``packs`` = the three
    ConvPacks (BN folded, conv2 chunk-major), x_amax [N] per-frame max|x|, y_amax [N] raised."""
    _gpu(x, y, x_amax)
    if x_amax is None:
        raise ValueError("prpe_bottleneck: x_amax (per-frame max|x| of the block input) is required")
    _check_slots("prpe_bottleneck", x.shape[0], x_amax, y_amax)
    d = BneckDesc()
    d.x, d.y = view(x), view(y)
    d.x_amax, d.y_amax = x_amax.data_ptr(), _ptr(y_amax)
    d.mid = packs[0].co
    keep = []
    for i, pk in enumerate(packs):
        h16, l16, s16 = pk.f16_planes()
        b = pk.bias if pk.bias is not None else torch.zeros(pk.co, device=x.device)
        keep.append(b)
        d.w_h16[i], d.w_l16[i], d.scale16[i], d.bias[i] = h16.data_ptr(), l16.data_ptr(), s16.data_ptr(), b.data_ptr()
        d.k_pad[i] = pk.k_pad
    check(lib().prpe_bottleneck(C.byref(d), _stream()), "prpe_bottleneck")
    return y


def stem_maxpool(buf, h, w, x_amax, pack, y, y_amax=None):
    """ResNet-50 stem conv (7x7/2, BN, ReLU) + max-pool 3x3/2 in one launch (prpe_stem_maxpool,
    include/prpe.h). ``buf``: the zero-bordered NHWC4 frames [N, h+6, w+8, 4] (Engine.stem's
    buffer, image at rows / columns 3..); ``pack``: the stem's chunked precision-3 ConvPack
    (k_pad 224); y [N, h/4, w/4, 64]."""
    _gpu(buf, y, x_amax)
    if not buf.is_contiguous() or buf.dim() != 4 or buf.shape[3] != 4:
        raise PrpeError("stem_maxpool: buf must be a contiguous [N, H+6, W+8, 4] buffer")
    if x_amax is None:
        raise ValueError("prpe_stem_maxpool: x_amax (per-frame max|x| of the frames) is required")
    _check_slots("prpe_stem_maxpool", buf.shape[0], x_amax, y_amax)
    d = StemDesc()
    d.x, d.xsn, d.xsh = buf.data_ptr(), buf.stride(0), buf.stride(1)
    d.n, d.h, d.w = buf.shape[0], h, w
    d.x_amax = x_amax.data_ptr()
    h16, l16, s16 = pack.f16_planes()
    b = pack.bias if pack.bias is not None else torch.zeros(pack.co, device=buf.device)
    d.w_h16, d.w_l16, d.k_pad, d.scale16, d.bias = h16.data_ptr(), l16.data_ptr(), pack.k_pad, s16.data_ptr(), b.data_ptr()
    d.y = view(y)
    d.y_amax = _ptr(y_amax)
    check(lib().prpe_stem_maxpool(C.byref(d), _stream()), "prpe_stem_maxpool")
    return y


def upconv3x3(z, y, align_corners, scale=None, bias=None, slope=None, act="none", separable=False,
              y_planes=False, y_amax=None):
    """Fused one-pass kernel by default; ``separable=True`` runs the two-pass workspace form.
    ``y_amax`` ([N] device, zeroed): raised to max|y[n]| per frame (one-pass kernels only)."""
    _check_slots("prpe_upconv3x3", y.shape[0], y_amax)
    zv, yv = view(z), view(y)
    ws, nbytes = None, 0
    if separable:
        nbytes = lib().prpe_upconv3x3_workspace_bytes(C.byref(zv), C.byref(yv))
        ws = torch.empty((nbytes + 3) // 4, device=z.device, dtype=torch.float32)
    check(lib().prpe_upconv3x3(C.byref(zv), C.byref(yv), 1 if align_corners else 0, _ptr(scale), _ptr(bias),
                               _ptr(slope), ACT[act], int(y_planes), _ptr(y_amax), _ptr(ws), nbytes, _stream()),
          "prpe_upconv3x3")
    return y


def dwconv(x, y, w, k, stride, pad, scale, bias, act="none", res=None):
    check(lib().prpe_dwconv(C.byref(view(x)), C.byref(view(y)), C.byref(view(res)), _ptr(w), k, stride, pad,
                            _ptr(scale), _ptr(bias), ACT[act], _stream()), "prpe_dwconv")
    return y


def maxpool(x, y, k, stride, pad):
    check(lib().prpe_maxpool(C.byref(view(x)), C.byref(view(y)), k, stride, pad, _stream()), "prpe_maxpool")
    return y


def copy_pad(x, y, flip_w=False, y_amax=None):
    """y = x zero-padded in C; ``flip_w`` reads x mirrored along W (a negative-stride view,
    so the flip-test pass needs no flipped copy of the frames); ``y_amax`` ([N] device tensor,
    zeroed) is raised to max|y[n]| per frame."""
    xv = view(x)
    if flip_w:
        xv.ptr = x.data_ptr() + (x.shape[2] - 1) * x.stride(2) * x.element_size()
        xv.sw = -x.stride(2)
    check(lib().prpe_copy_pad(C.byref(xv), C.byref(view(y)), _ptr(y_amax), _stream()), "prpe_copy_pad")
    return y


def upsample_nearest2x(x, y):
    check(lib().prpe_upsample_nearest2x(C.byref(view(x)), C.byref(view(y)), _stream()), "prpe_upsample_nearest2x")
    return y


def norm_sigmoid(x, y):
    check(lib().prpe_norm_sigmoid(C.byref(view(x)), C.byref(view(y)), _stream()), "prpe_norm_sigmoid")
    return y


def layernorm(x2d, y2d, gamma, beta, eps=1e-12, relu=False, planes=False):
    """planes: write y2d in the planes format (prpe.h) for a precision-0 GEMM consumer."""
    _gpu(x2d, y2d, gamma, beta)
    rows, c = x2d.shape
    check(lib().prpe_layernorm(x2d.data_ptr(), x2d.stride(0), y2d.data_ptr(), y2d.stride(0), rows, c,
                               gamma.data_ptr(), beta.data_ptr(), eps, (1 if relu else 0) | (2 if planes else 0),
                               _stream()), "prpe_layernorm")
    return y2d


def attention(qkv, out, B, L, H, D, scale):
    _gpu(qkv, out)
    check(lib().prpe_attention(qkv.data_ptr(), out.data_ptr(), B, L, H, D, scale, _stream()), "prpe_attention")
    return out


def attention_strided(qkv, strides, out, B, L, H, D, scale, out_planes=False):
    """qkv: tensor holding q/k/v at element strides (frame, which, head, token), e.g. a
    head-major [B, 3, H, L, D] buffer: (3*H*L*D, H*L*D, L*D, D); the row-major [B*L, 3*H*D]
    operand of prpe_attention is (L*3*H*D, H*D, D, 3*H*D). out_planes: write out in the planes
    format (prpe.h) for a precision-0 GEMM consumer."""
    _gpu(qkv, out)
    sf, sw, sh, st = (int(v) for v in strides)
    check(lib().prpe_attention_strided(qkv.data_ptr(), sf, sw, sh, st, out.data_ptr(), B, L, H, D, scale,
                                       1 if out_planes else 0, _stream()), "prpe_attention_strided")
    return out


def psa_attention(qkv, out, vout, nh, dk, dh, scale):
    check(lib().prpe_psa_attention(C.byref(view(qkv)), C.byref(view(out)), C.byref(view(vout)), nh, dk, dh, scale,
                                   _stream()), "prpe_psa_attention")
    return out


def dfl_decode(head, out, nc, level_hw, strides):
    _gpu(head, out)
    B = head.shape[0]
    hw = (C.c_int32 * (2 * len(level_hw)))(*[v for hw_ in level_hw for v in hw_])
    st = (C.c_float * len(strides))(*[float(s) for s in strides])
    check(lib().prpe_dfl_decode(head.data_ptr(), out.data_ptr(), B, nc, len(level_hw), hw, st, _stream()),
          "prpe_dfl_decode")
    return out


def l2norm(x, emb, norm, eps=0.0):
    """emb = x / max(||x||, eps) per row, norm = ||x||. eps 0: torch.div(x, norm) (IR-50 output);
    eps 1e-12: F.normalize."""
    _gpu(x, emb, norm)
    rows, c = x.shape
    check(lib().prpe_l2norm(x.data_ptr(), emb.data_ptr(), norm.data_ptr(), rows, c, float(eps), _stream()),
          "prpe_l2norm")
    return emb, norm


def nms(pred, layout, conf=0.001, iou=0.65, max_nms=30000, max_det=300):
    """Batched device NMS -> (out [B,max_det,6], count [B] int32). layout 0: [B,4+nc,N]; 1: [B,N,4+nc]."""
    pred = _gpu(pred).contiguous()
    B = pred.shape[0]
    if layout == 0:
        nc, N = pred.shape[1] - 4, pred.shape[2]
    else:
        N, nc = pred.shape[1], pred.shape[2] - 4
    out = torch.empty(B, max_det, 6, device=pred.device, dtype=torch.float32)
    cnt = torch.empty(B, device=pred.device, dtype=torch.int32)
    # N*nc above the kernel's LDS key capacity: keys + a radix sort per image in a global workspace
    nbytes = lib().prpe_nms_workspace_bytes(B, N, nc, max_nms)
    if nbytes < 0:
        raise RuntimeError("prpe_nms_workspace_bytes failed")
    ws = torch.empty((nbytes + 7) // 8, device=pred.device, dtype=torch.int64) if nbytes else None
    check(lib().prpe_nms(pred.data_ptr(), B, N, nc, layout, conf, iou, max_nms, max_det, out.data_ptr(),
                         cnt.data_ptr(), _ptr(ws), nbytes, _stream()), "prpe_nms")
    return out, cnt


def softargmax(heat, boxes=None, want_argmax=False):
    heat = _gpu(heat).contiguous()
    B, K, H, W = heat.shape
    coords = torch.empty(B, K, 2, device=heat.device, dtype=torch.float32)
    scores = torch.empty(B, K, device=heat.device, dtype=torch.float32)
    am = torch.empty(B, K, device=heat.device, dtype=torch.int32) if want_argmax else None
    bx = boxes.contiguous().float() if boxes is not None else None
    check(lib().prpe_softargmax(heat.data_ptr(), B, K, H, W, _ptr(bx), coords.data_ptr(), scores.data_ptr(),
                                _ptr(am), _stream()), "prpe_softargmax")
    return (coords, scores, am) if want_argmax else (coords, scores)


def flip_average(heat, heat_flipped, partner, mode=0):
    """Pose flip test: (heat + flipback(heat_flipped)) * 0.5 (pose_estimation/module.py:470-484)."""
    heat, heat_flipped = (t.contiguous() for t in _gpu(heat, heat_flipped))
    B, K, H, W = heat.shape
    out = torch.empty_like(heat)
    pa = (C.c_int32 * K)(*[int(v) for v in partner])
    check(lib().prpe_flip_average(heat.data_ptr(), heat_flipped.data_ptr(), out.data_ptr(), B, K, H, W, pa, mode,
                                  _stream()), "prpe_flip_average")
    return out


def ce_argmax(logits, labels=None):
    """Per-row argmax (+ cross-entropy and the [mean loss, acc] summary when labels given)."""
    _gpu(logits)
    B, Cn = logits.shape
    assert logits.stride(1) == 1
    amax = torch.empty(B, device=logits.device, dtype=torch.int32)
    loss = summary = None
    if labels is not None:
        labels = labels.to(device=logits.device, dtype=torch.int64).contiguous()
        loss = torch.empty(B, device=logits.device, dtype=torch.float32)
        summary = torch.empty(2, device=logits.device, dtype=torch.float32)
    check(lib().prpe_ce_argmax(logits.data_ptr(), logits.stride(0), B, Cn, _ptr(labels), _ptr(loss), amax.data_ptr(),
                               _ptr(summary), _stream()), "prpe_ce_argmax")
    return loss, amax, summary


def det_metrics_update(dets, counts, gt_boxes, gt_batch, counters, records):
    """Append one batch to the device DetectionMetrics state (see include/prpe.h)."""
    _gpu(dets, counts, counters, records)
    B, max_det, six = dets.shape
    assert six == 6 and dets.is_contiguous() and counts.dtype == torch.int32
    gt = gt_boxes.to(device=dets.device, dtype=torch.float32).contiguous().view(-1, 4)
    gb = gt_batch.to(device=dets.device, dtype=torch.int64).contiguous().view(-1)
    nbytes = lib().prpe_det_metrics_update_workspace_bytes(B)
    ws = torch.empty(max(1, (nbytes + 3) // 4), device=dets.device, dtype=torch.float32)
    check(lib().prpe_det_metrics_update(dets.data_ptr(), counts.contiguous().data_ptr(), B, max_det, gt.data_ptr(),
                                        gb.data_ptr(), gt.shape[0], counters.data_ptr(), records.data_ptr(),
                                        records.shape[0], ws.data_ptr(), nbytes, _stream()), "prpe_det_metrics_update")


def det_metrics_compute(counters, records, n, thresholds):
    """(precision, recall, f1, mAP50, mAP75, mAP) as a float64 device tensor [6]."""
    _gpu(counters, records)
    nbytes = lib().prpe_det_metrics_compute_workspace_bytes(n)
    ws = torch.empty((nbytes + 3) // 4, device=counters.device, dtype=torch.float32)
    out = torch.empty(6, device=counters.device, dtype=torch.float64)
    thr = (C.c_float * len(thresholds))(*[float(t) for t in thresholds])
    check(lib().prpe_det_metrics_compute(counters.data_ptr(), records.data_ptr(), n, C.cast(thr, C.c_void_p),
                                         out.data_ptr(), ws.data_ptr(), nbytes, _stream()), "prpe_det_metrics_compute")
    return out


def det_eval_loss(boxes, scores, gt_boxes, gt_batch, gt_classes=None):
    """Detection eval loss (see include/prpe.h): boxes [B,4,N], scores [B,C,N] (any strides).
    Returns (loss [1], per_image [B,4] = (loss_b, box, cls, bg))."""
    _gpu(boxes, scores)
    B, four, N = boxes.shape
    Cn = scores.shape[1]
    assert four == 4 and scores.shape[0] == B and scores.shape[2] == N
    dev = boxes.device
    gt = gt_boxes.to(device=dev, dtype=torch.float32).contiguous().view(-1, 4)
    gb = gt_batch.to(device=dev, dtype=torch.int64).contiguous().view(-1)
    gc = None if gt_classes is None else gt_classes.to(device=dev, dtype=torch.int64).contiguous().view(-1)
    bs = (C.c_int64 * 3)(*boxes.stride())
    ss = (C.c_int64 * 3)(*scores.stride())
    per = torch.empty(B, 4, device=dev, dtype=torch.float32)
    loss = torch.empty(1, device=dev, dtype=torch.float32)
    check(lib().prpe_det_eval_loss(boxes.data_ptr(), C.cast(bs, C.c_void_p), scores.data_ptr(), C.cast(ss, C.c_void_p),
                                   B, Cn, N, gt.data_ptr(), gb.data_ptr(), _ptr(gc), gt.shape[0], per.data_ptr(),
                                   loss.data_ptr(), _stream()), "prpe_det_eval_loss")
    return loss, per
