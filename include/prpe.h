/*
 * prpe.h — C ABI of the MI355X-native per-frame inference hot path of the
 * Person-Recognition-for-Pose-Estimation combined multi-task model.
 *
 * The reference (100 % Python, /root/reference) has no native boundary: its device work
 * is PyTorch/cuDNN operators called from nn.Modules. These entry points
 * are what a ctypes/FFI binding of that path binds; each cites the reference interface
 * (file:line) whose arithmetic it replaces. The Python host side
 * (person-recognition-for-pose-estimation_amd/prpe) mirrors the reference module API.
 *
 * Rules (all entry points):
 *   - Every buffer is caller-allocated device memory; the library never allocates.
 *   - Tensors are strided float32 views: element strides, any layout (NHWC/NCHW/...).
 *   - Calls are stream-ordered on the given hipStream_t (passed as void*), no implicit
 *     synchronisation; safe to call concurrently on different streams/devices.
 *   - Return 0 on success, a negative errno-style code (-22 = EINVAL) for bad
 *     arguments (checked before any launch), or a positive hipError_t from the launch.
 *   - Nothing throws across the ABI.
 */
#ifndef PRPE_H_
#define PRPE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRPE_ABI_VERSION 10

/* activations (epilogues/prologues) */
enum prpe_act {
  PRPE_ACT_NONE = 0,
  PRPE_ACT_RELU = 1,   /* torch.nn.ReLU */
  PRPE_ACT_SILU = 2,   /* torch.nn.SiLU  (yolopt/nets/nn.py:28-36) */
  PRPE_ACT_PRELU = 3,  /* torch.nn.PReLU, per-channel slope (libs/net_adaface.py:153-160) */
  PRPE_ACT_GELU = 4,   /* exact erf GELU (modify_models.py:356, ViT MLP) */
  PRPE_ACT_SIGMOID = 5
};

/* residual modes of the conv epilogue */
enum prpe_res_mode {
  PRPE_RES_NONE = 0,
  PRPE_RES_PRE_ACT = 1,  /* y = act(acc*scale + bias + r)   ResNet bottleneck / IR unit / ViT */
  PRPE_RES_POST_ACT = 2  /* y = act(acc*scale + bias) + r   yolopt Residual (nn.py:48-49) */
};

/* A strided 4-D float32 view, logical shape [n, h, w, c]. */
typedef struct prpe_view {
  float* ptr;
  int32_t n, h, w, c;
  int64_t sn, sh, sw, sc;
} prpe_view;

/*
 * Convolution (groups = 1) as an implicit GEMM on MFMA with split-bf16 operands
 * (fp32 accumulate): see ``precision``.
 *   y[n,oh,ow,co] = EPI( sum_{kh,kw,ci} PRO(x[n, oh*s-p+kh, ow*s-p+kw, ci]) * W[co,kh,kw,ci] )
 * PRO(v) = v*in_scale[ci] + in_bias[ci] for in-bounds taps, 0 for padding (IR-50 pre-BN,
 * libs/net_adaface.py:159). EPI = folded BN / bias (scale, bias), residual, activation.
 * Weights are packed by the host: bf16 planes [co_pad][k_pad], w = plane0 + plane1 + plane2
 * (RNE splits), with k in the order ``k_order`` names:
 *   0: k = (kh*KW+kw)*Ci + ci                          (any Ci)
 *   1: k = ((ci/32)*KH*KW + kh*KW+kw)*32 + ci%32       (Ci % 32 == 0, channel-contiguous x:
 *      the taps of one 32-channel chunk are consecutive K-steps -> input re-reads hit L1)
 * Replaces: torch.nn.Conv2d + BatchNorm2d (+act, +residual) in training/modify_models.py,
 * yolopt/nets/nn.py:28-39, libs/net_adaface.py:144-167, torchvision resnet50 (:446),
 * nn.Linear in ViTPose and IR-50 output_layer (as a 1x1 / 7x7 "conv").
 */
typedef struct prpe_conv_desc {
  prpe_view x;            /* input  [N, Hi, Wi, Ci] */
  prpe_view y;            /* output [N, Ho, Wo, Co] */
  prpe_view res;          /* residual [N, Ho, Wo, Co] (ptr may be NULL) */
  int32_t kh, kw, stride, pad;
  const uint16_t* w_hi;   /* bf16 bits, plane 0 */
  const uint16_t* w_lo;   /* plane 1 (precision 0, 2) */
  const uint16_t* w_lo2;  /* plane 2 (precision 2) */
  int32_t k_pad, co_pad;  /* packed extents (k_pad % 32 == 0, co_pad % 128 == 0) */
  const float* scale;     /* [Co] or NULL (= 1) */
  const float* bias;      /* [Co] or NULL (= 0) */
  const float* slope;     /* [Co] PReLU slopes or NULL */
  const float* in_scale;  /* [Ci] or NULL; needs the vector path (x.sc == 1, Ci % 4 == 0, 16-B rows) */
  const float* in_bias;   /* [Ci] or NULL */
  int32_t act;            /* prpe_act */
  int32_t res_mode;       /* prpe_res_mode */
  int32_t precision;      /* 0 = 2-plane split-bf16, 3 MFMA terms (~2^-17);
                             2 = 3-plane split (exact fp32 operands), 6 terms;
                             3 = 2-plane split-fp16 with power-of-2 scaling, 3 terms (~2^-21
                                 per operand: below fp32 accumulation error for K >= 64);
                                 needs w_h16/w_l16/scale16/x_amax, no in_scale, and a
                                 channel-chunked input (Ci % 32 == 0, k_order 1 or 1x1);
                             4 = ONE fp16 plane per operand with the same power-of-2 scaling,
                                 RNE, 1 term (~2^-12 per operand); needs w_h16/scale16/x_amax
                                 (w_l16 unused), a channel-chunked input, no dual input / planes;
                                 in_scale allowed (the kernel bounds max|PRO(x)| by
                                 x_amax max|in_scale| + max|in_bias|); the AdaFace branch's policy;
                             1 = plain bf16 (1 term; diagnostics only) */
  int32_t tile;           /* 0 = auto; 1..6 = 128x128, 128x64, 128x32, 128x16, 256x128, 256x64
                             (register-staged); 10..12 LDS-DMA staged; 21..25 wave-row */
  int32_t k_order;        /* weight K order, see above */
  /* precision 3 operands: fp16 planes [co_pad][k_pad] of w[co][k] * 2^e[co] (w = (h16 + l16)
   * * 2^-e[co] to ~2^-22), the epilogue scale with 2^-e[co] folded in, and PER-FRAME bounds
   * x_amax[n] >= max|x[n]| (n < N; the producer's y_amax) that set each frame's power-of-2
   * activation scale -- a frame's arithmetic never depends on the other frames of the batch */
  const uint16_t* w_h16;
  const uint16_t* w_l16;
  const float* scale16;   /* [Co] */
  const float* x_amax;    /* [N] device */
  float* y_amax;          /* optional (any precision): device [N], y_amax[n] raised to max|y[n]|
                             (atomic; zero it before the producing launch) */
  /* optional second input (x2.ptr != NULL): y = EPI(W[:, :Ci] x + W[:, Ci:] x2), a 1x1 unpadded
   * conv over both; x2 is [N, Ho, Wo, C2] on the output's pixel grid (any strides, e.g. a
   * stride-2 subsampling view), channel-contiguous, C2 % 32 == 0 and Ci % 32 == 0; weights
   * packed [co_pad][k_pad] with k = Ci + C2 columns; precision 0/2/3 (3 also needs x2_amax [N];
   * one activation scale per frame for both inputs). Replaces a ResNet bottleneck's conv3 + downsample
   * projection + residual add (torchvision resnet50 Bottleneck.forward) with one GEMM. */
  prpe_view x2;
  const float* x2_amax;
  /* planes format: a tensor of fp32 shape [N,H,W,C] whose bytes hold, per pixel and per
   * group of 8 channels, the 8 bf16 hi planes then the 8 bf16 lo planes of the two-plane split
   * (hi = RNE(v), lo = RNE(v - hi)): what precision 0 would compute from the fp32 values, so a
   * producer that writes it saves the consumer's split, bit for bit. x_planes: x is in it
   * (precision 0, channel-chunked 1x1/3x3, wave-row kernel); y_planes: write y in it
   * (channel-contiguous, C % 8 == 0, 32-B aligned). */
  int32_t x_planes;
  int32_t y_planes;
  /* optional 1x1 GEMM in the epilogue (w2 != NULL): after scale/bias/act, z = y' W2^T with W2
   * fp32 [y2.c][Co], written to y2 [N, Ho, Wo, y2.c] (channel-contiguous, y2.c <= 32) instead
   * of y (not written). Split-bf16 matrix-core products (two planes per operand, three
   * products: the precision-0 split) on the tile held in LDS. The 3x3 conv -> Co <= 4 3x3 conv
   * pairs of the adapters (the second conv as its 1x1 tap GEMM + shifted tap sum,
   * prpe_upconv3x3 at unit scale): the intermediate tensor never reaches HBM. Haloed-tile 3x3
   * kernel only (3x3 / s1 / p1, Co <= 128, precision 0 or 3, no residual / planes / max|y|). */
  const float* w2;
  prpe_view y2;
  /* optional second stage (w3 != NULL, with w2): z1 = act2(scale2 * (y' W2^T) + bias2) with
   * W2 fp32 [n2][Co], n2 <= 64 (scale2 / bias2 [n2] or NULL for 1 / 0), then z = z1 W3^T with
   * W3 fp32 [y2.c][n2] into y2 (a conv -> 1x1 conv -> tap GEMM chain, YOLO adapter .10/.13/.16) */
  const float* w3;
  const float* scale2;
  const float* bias2;
  int32_t act2;
  int32_t n2;
  /* caller-owned device scratch, >= prpe_conv2d_workspace_bytes(d) bytes, 256-B aligned (NULL and
   * 0 when that is 0). Only the split-K path of full-window linears uses it (the IR-50 output
   * layer: partial sums per K-slice); a call that needs more than it is given returns -EINVAL.
   * Concurrent calls on different streams must pass different workspaces. */
  void* workspace;
  int64_t workspace_bytes;
} prpe_conv_desc;

/* Scratch bytes prpe_conv2d(d) needs (0 for every path but split-K), or -EINVAL for a descriptor
 * prpe_conv2d would reject. Host-only: no launch, no allocation. */
int64_t prpe_conv2d_workspace_bytes(const prpe_conv_desc* d);
int prpe_conv2d(const prpe_conv_desc* d, void* stream);

/*
 * Fused ResNet bottleneck with identity shortcut, precision 3 (torchvision Bottleneck.forward,
 * v1.5; the reference trunk's layer1 blocks 1-2, modify_models.py:413-446):
 *   y = relu(bn3(conv3(relu(bn2(conv2_3x3(relu(bn1(conv1(x)))))))) + x)
 * x, y: [N, H, W, 4*mid] channel-contiguous (x 16-B aligned rows; x [N, H, W, mid] for the
 * projection block below); x_amax [N] per-frame max|x|
 * (as prpe_conv2d precision 3); y_amax (optional) raised to max|y[n]|. Weights as prpe_conv2d's
 * precision-3 packs: fp16 planes w_h16 / w_l16 [co_pad][k_pad] (conv1 k = 4 mid, conv2 chunk-major
 * k = 9 mid, conv3 k = mid), scale16 (the planes' 2^-e folded in) and bias [Co]. The two inner
 * activations never reach HBM; they are rounded to fp16 planes with one power-of-2 scale per
 * 8 x 16 output tile (per frame and tile: frames stay independent). mid = 64 (layer1) or 128
 * (layer2, identity blocks only).
 * Projection block (layer1.0, stride 1): x has mid channels (x.c == mid, y.c == 4 mid) and
 *   y = relu(bn3(conv3(t2)) + bn_d(downsample(x)))
 * with conv3 and the downsample 1x1 as ONE dual GEMM over [t2 | x]: weight slot 2 is then the
 * [4 mid][2 mid] matrix [s3 W3 | sd Wd] (both BN scales folded into its rows, k_pad = 2 mid) and
 * bias[2] = b3 + bd; t2 and x share one power-of-2 scale (max of the tile's max|t2| and the
 * frame's max|x|), as prpe_conv2d's dual-input GEMM.
 * x, y, the weight planes, scale16 and bias 16-B aligned, x / y pixel strides multiples of 4
 * floats, one frame of x and of y < 2^31 bytes; anything else returns -EINVAL. Not in place: y
 * must not overlap x (other tiles read x's halo and residual while y is written) -> -EINVAL.
 */
typedef struct prpe_bneck_desc {
  prpe_view x;
  prpe_view y;
  const float* x_amax;
  float* y_amax;
  int32_t mid;
  const uint16_t* w_h16[3];
  const uint16_t* w_l16[3];
  int32_t k_pad[3];
  const float* scale16[3];
  const float* bias[3];
} prpe_bneck_desc;
int prpe_bottleneck(const prpe_bneck_desc* d, void* stream);

/*
 * ResNet-50 stem + max-pool in one launch, precision 3 (torchvision resnet50 conv1 7x7/2 pad 3
 * -> bn1 -> relu -> maxpool 3x3/2 pad 1; the reference trunk, modify_models.py:413-446):
 *   y[n, py, px, c] = max over the 3x3 / 2 window of relu(bn1(conv1(x)))
 * x: the frames as a zero-bordered NHWC4 buffer, element (n, h, w, c) at x + n*xsn + h*xsh + 4*w + c,
 * h < H + 6, w < W + 8, the image at rows / columns 3 .. (prpe_copy_pad writes it; the 4th
 * channel and the border are zero); x_amax [N] per-frame max|x|. The weight pack is the stem's
 * precision-3 pack of prpe_conv2d's chunked form: W'[64][224], k = kh*32 + kw*4 + c (zero for
 * kw = 7, c = 3), fp16 planes w_h16 / w_l16 with scale16 (2^-e folded in) and bias [64]. Every
 * stem value equals prpe_conv2d's on the same view bit for bit; the stem map never reaches HBM.
 * y: [N, H/4, W/4, 64], channel-contiguous, 16-B aligned; y_amax (optional) raised to max|y[n]|
 * (= the stem map's max: every stem output lies in some window). H, W multiples of 4, one frame
 * of x < 2^31 bytes, y not overlapping x's N frames; anything else returns -EINVAL.
 */
typedef struct prpe_stem_desc {
  const float* x;
  int64_t xsn, xsh;
  int32_t n, h, w;
  const float* x_amax;
  const uint16_t* w_h16;
  const uint16_t* w_l16;
  int32_t k_pad;
  const float* scale16;
  const float* bias;
  prpe_view y;
  float* y_amax;
} prpe_stem_desc;
int prpe_stem_maxpool(const prpe_stem_desc* d, void* stream);

/*
 * conv3x3(pad 1) o bilinear-upsample, second stage of the exact algebraic rewrite
 *   conv3x3(U(x)) = sum_tap shift_tap(U(Z_tap)),   Z_tap = W_tap . x  (low-res 1x1 GEMM)
 * z: [N, Hi, Wi, 9*Co] low-res per-tap products (channel = tap*Co + co, tap = kh*3+kw).
 * y[n,oy,ox,co] = act( (sum_tap valid * bilerp(Z_tap, src(oy+kh-1, ox+kw-1))) * scale + bias )
 * align_corners = 1: src = dst*(in-1)/(out-1);  0: src = max(0,(dst+0.5)*in/out-0.5).
 * Replaces nn.Upsample(bilinear) + Conv2d(3x3) + BN + act in modify_models.py:47-52,
 * :237-242, :359-364 and the ViTPose simple decoder (modeling_vitpose.py:120-144).
 * workspace = NULL (the product path) selects the fused one-pass kernel: x-interpolated
 * source rows are kept in rolling registers, HBM traffic = y write + z read. With a workspace
 * of >= prpe_upconv3x3_workspace_bytes(z, y) bytes the sum is instead evaluated in two passes
 * through it (x-interpolation, then y; kept for ablation). Both agree to fp32 rounding.
 * y_planes: write y in the planes format described at prpe_conv_desc: fused path, C % 8 == 0,
 * channel-contiguous, 32-B aligned; for a precision-0 consumer conv.
 * y_amax (optional, ABI 8): device [N], y_amax[n] raised to max|y[n]| (zeroed by the caller;
 * the per-frame bound a precision-3/4 consumer conv reads as its x_amax); fused path only.
 */
int64_t prpe_upconv3x3_workspace_bytes(const prpe_view* z, const prpe_view* y);
int prpe_upconv3x3(const prpe_view* z, const prpe_view* y, int32_t align_corners,
                   const float* scale, const float* bias, const float* slope, int32_t act,
                   int32_t y_planes, float* y_amax, void* workspace, int64_t workspace_bytes,
                   void* stream);

/* Depthwise kxk conv (groups = C) + folded BN + act (+ post-act residual add when res.ptr).
 * Replaces yolopt Conv(g=ch) (nn.py:108, :248-250). */
int prpe_dwconv(const prpe_view* x, const prpe_view* y, const prpe_view* res,
                const float* w /* [C][k][k] */, int32_t k, int32_t stride, int32_t pad,
                const float* scale, const float* bias, int32_t act, void* stream);

/* Max pooling, k x k / stride / pad (-inf padding). torchvision resnet maxpool,
 * yolopt SPP (nn.py:88-94), IR-50 MaxPool2d(1, s) shortcut (net_adaface.py:148). */
int prpe_maxpool(const prpe_view* x, const prpe_view* y, int32_t k, int32_t stride,
                 int32_t pad, void* stream);

/* Strided copy with channel zero-padding: y[...,c] = c < x.c ? x[...,c] : 0 (e.g. NCHW frames
 * -> NHWC4 for the vectorised stem conv; the 4th channel meets a zero weight column).
 * y_amax (optional): device [N], y_amax[n] raised to max|y[n]| (zeroed by the caller). */
int prpe_copy_pad(const prpe_view* x, const prpe_view* y, float* y_amax /* optional */, void* stream);

/* Nearest x2 upsample (yolopt DarkFPN nn.Upsample(scale_factor=2), nn.py:195). */
int prpe_upsample_nearest2x(const prpe_view* x, const prpe_view* y, void* stream);

/* Per-sample, per-channel standardisation + sigmoid (modify_models.py:84-86):
 * y = sigmoid((x - mean_hw) / (std_hw_unbiased + 1e-6)). */
int prpe_norm_sigmoid(const prpe_view* x, const prpe_view* y, void* stream);

/* LayerNorm over the last dim of rows (ViTPose, eps 1e-12). x/y: [rows][C] with row strides.
 * flags: bit 0 = ReLU on the output (simple decoder's ReLU, modeling_vitpose.py:139); bit 1 =
 * write y in the planes format described at prpe_conv_desc: C % 8 == 0, C <= 1024, 16-B aligned x rows,
 * 32-B aligned y rows; the input format of the precision-0 GEMM that consumes it. */
int prpe_layernorm(const float* x, int64_t x_row_stride, float* y, int64_t y_row_stride,
                   int64_t rows, int32_t C, const float* gamma, const float* beta,
                   float eps, int32_t flags, void* stream);

/* ViT multi-head self-attention, softmax(Q K^T * scale) V per (frame, head).
 * qkv: [B*L][3*H*D] rows (q | k | v, head-major inside each), out: [B*L][H*D].
 * Replaces eager_attention_forward (modeling_vitpose_backbone.py:100-126). */
int prpe_attention(const float* qkv, float* out, int32_t B, int32_t L, int32_t H, int32_t D,
                   float scale, void* stream);

/* The same attention on a strided q/k/v operand: element (frame b, which w = 0 q / 1 k / 2 v,
 * head h, token t, channel d) at qkv[b*s_frame + w*s_which + h*s_head + t*s_tok + d]; all
 * strides multiples of 4 elements, qkv 16-B aligned. prpe_attention is the row-major case
 * (s_frame = L*3*H*D, s_which = H*D, s_head = D, s_tok = 3*H*D); a head-major QKV GEMM output
 * [B][3][H][L][D] (s_frame = 3*H*L*D, s_which = H*L*D, s_head = L*D, s_tok = D) gives every
 * head's K and V as one contiguous 48-KB block. out: [B*L][H*D], in the planes format of
 * prpe_conv_desc when out_planes != 0 (the input format of the precision-0 projection GEMM). */
int prpe_attention_strided(const float* qkv, int64_t s_frame, int64_t s_which, int64_t s_head,
                           int64_t s_tok, float* out, int32_t B, int32_t L, int32_t H, int32_t D,
                           float scale, int32_t out_planes, void* stream);

/* YOLO PSA attention core (nn.py:111-122): per frame, per head:
 *   out[c, i] = sum_j v[c, j] softmax_j(q[:, i] . k[:, j] * scale)
 * qkv view [N, h, w, nh*(2*dk+dh)] (per head: q dk | k dk | v dh), out view [N,h,w,nh*dh].
 * vout (optional, ptr may be NULL): v gathered head-major [N,h,w,nh*dh] — the
 * ``v.reshape(b, c, h, w)`` operand of the depthwise positional conv (nn.py:122). */
int prpe_psa_attention(const prpe_view* qkv, const prpe_view* out, const prpe_view* vout,
                       int32_t nh, int32_t dk, int32_t dh, float scale, void* stream);

/* YOLO Head eval decode (nn.py:255-270 + DFL nn.py:212-225 + make_anchors util.py:85-96).
 * head: [B, A, 64+nc] rows (per anchor: 64 DFL logits, nc class logits), levels given by
 * (h_l, w_l, stride_l) in anchor order; out: [B, 4+nc, A] = (cx,cy,w,h)*stride, sigmoid(cls). */
int prpe_dfl_decode(const float* head, float* out, int32_t B, int32_t nc, int32_t nlevels,
                    const int32_t* level_hw /* [nlevels*2] host */, const float* strides /* host */,
                    void* stream);

/* Row-wise L2 normalisation: norm = ||x||_2, emb = x / max(norm, eps).
 * eps = 0: IR-50 output torch.div(x, norm) (net_adaface.py:334-337; a zero row gives NaN as there);
 * eps = 1e-12: F.normalize (face_recognition/module.py:137-138; a zero row gives 0). */
int prpe_l2norm(const float* x, float* emb, float* norm, int32_t rows, int32_t C, float eps, void* stream);

/*
 * yolopt.util.non_max_suppression (training/yolopt/util.py:123-169), batched, on device.
 * pred: [B, 4+nc, N] when layout = 0; [B, N, 4+nc] when layout = 1 (same arithmetic as the
 * reference on a transposed tensor). Candidates: max class score > conf; boxes cxcywh ->
 * xyxy; nc==1: best class; nc>1: every (box, class) with score > conf; stable descending
 * score order (ties by index), <= max_nms candidates, class offset 7680*cls,
 * greedy suppression IoU > iou (torchvision.ops.nms), <= max_det kept.
 * out: [B, max_det, 6] (x1,y1,x2,y2,conf,cls), count: [B] int32. No host sync.
 * workspace: >= prpe_nms_workspace_bytes(B, N, nc, max_nms) bytes, 256-B aligned (0 bytes and
 * NULL allowed when N*nc <= 16384: candidates sorted in LDS; above that the keys and one
 * rocPRIM radix sort per image go through the workspace).
 * The reference's wall-clock cut-off (util.py:133-134,166-167) is not reproduced.
 */
int64_t prpe_nms_workspace_bytes(int32_t B, int32_t N, int32_t nc, int32_t max_nms);
int prpe_nms(const float* pred, int32_t B, int32_t N, int32_t nc, int32_t layout,
             float conf, float iou, int32_t max_nms, int32_t max_det,
             float* out, int32_t* count, void* workspace, int64_t workspace_bytes, void* stream);

/*
 * PoseEstimationModule._get_keypoints_from_heatmaps (pose_estimation/module.py:237-296):
 * per (frame, keypoint) softmax over H*W, coords = (E[x]+0.5)/W, (E[y]+0.5)/H, score =
 * max prob (* clamp(sqrt(box area)/96, .5, 2) when boxes != NULL, boxes [B,4] x1y1x2y2).
 * heat: [B, K, H, W] contiguous. argmax (optional, may be NULL): [B,K] int32 flat index of
 * the max (first occurrence) = the hard-argmax keypoint.
 */
int prpe_softargmax(const float* heat, int32_t B, int32_t K, int32_t H, int32_t W,
                    const float* boxes, float* coords, float* scores, int32_t* argmax,
                    void* stream);

/*
 * Pose flip test, device half (pose_estimation/module.py:470-484):
 *   out = (heat + F) * 0.5,  F[b,k,h,w] = heat_flipped[b', k', h, W-1-w]
 * heat_flipped = heatmaps of the W-flipped frames. partner[k] (host, K <= 64) = the other
 * keypoint of k's flip pair or -1. mode 0 = the reference's arithmetic: for paired channels
 * ``flipped[:, pair].flip(0)`` reverses the BATCH order (b' = B-1-b, k' = k); mode 1 = the
 * channel swap the code intends (b' = b, k' = partner[k]). out must not alias heat_flipped.
 */
int prpe_flip_average(const float* heat, const float* heat_flipped, float* out, int32_t B, int32_t K,
                      int32_t H, int32_t W, const int32_t* partner, int32_t mode, void* stream);

/*
 * Face-recognition eval head, row reductions (face_recognition/module.py:141-145):
 * logits [B, C] (row stride ld) = s * cos(normalize(emb), normalize(kernel)) from prpe_conv2d.
 * argmax[b] = first index of the row max (torch.max(1)[1]); with labels (int64 [B]):
 * loss[b] = logsumexp(row) - row[label]; summary (optional, [2]) = mean loss
 * (F.cross_entropy) and mean(argmax == label) (the reference's acc).
 */
int prpe_ce_argmax(const float* logits, int64_t ld, int32_t B, int32_t C, const int64_t* labels,
                   float* loss, int32_t* argmax, float* summary, void* stream);

/*
 * Detection eval metrics (DetectionMetrics, training/lightning/face_detection/module_v2.py:13-127,
 * as driven by validation_step :458-499). State is caller-allocated on
 * the device: counters uint64 [4] = (tp, fp, gt, records), zeroed to reset; records float
 * [capacity][2] = (score, best IoU) appended in image, then prediction order.
 * update: dets [B, max_det, 6] (x1,y1,x2,y2,conf,cls) + counts [B] from prpe_nms, ground truth
 * gt_boxes [G, 4] xyxy with gt_batch [G] (int64 image index, the reference's targets['batch_idx']);
 * images with no prediction or no ground truth are skipped (validation_step's `continue`s);
 * each prediction's best IoU over its image's boxes (box_iou: inter / (union + 1e-6), fp32),
 * tp if > 0.5. Records past capacity are dropped (counters[3] still counts them).
 * compute (epoch end): n = counters[3] (host value), thresholds = host float[10]
 * (torch.linspace(0.5, 0.95, 10)); out double[6] = precision, recall, f1, mAP50, mAP75, mAP
 * (compute(): stable descending sort by score, per-threshold cumulative tp/fp, torch.trapz).
 */
int64_t prpe_det_metrics_update_workspace_bytes(int32_t B);
int prpe_det_metrics_update(const float* dets, const int32_t* counts, int32_t B, int32_t max_det,
                            const float* gt_boxes, const int64_t* gt_batch, int32_t G, uint64_t* counters,
                            float* records, int64_t capacity, void* workspace, int64_t workspace_bytes,
                            void* stream);
int64_t prpe_det_metrics_compute_workspace_bytes(int64_t n);
int prpe_det_metrics_compute(const uint64_t* counters, const float* records, int64_t n,
                             const float* thresholds, double* out, void* workspace, int64_t workspace_bytes,
                             void* stream);

/*
 * Detection eval loss (FaceDetectionModule.compute_loss, module_v2.py:178-303, as validation_step
 * :467 calls it on the eval head output): boxes [B, 4, N] and scores [B, C, N] as strided views
 * (element strides [3] each, host arrays), ground truth gt_boxes [G, 4] / gt_batch [G] / optional
 * gt_classes [G] (int64). per_image [B][4] = (loss_b, box, cls, bg) (NaN where the reference
 * computes no such term), loss [1] = sum_b loss_b / B. N <= 1024. See csrc/detmetrics.hip.
 */
int prpe_det_eval_loss(const float* boxes, const int64_t* box_strides, const float* scores,
                       const int64_t* score_strides, int32_t B, int32_t C, int32_t N, const float* gt_boxes,
                       const int64_t* gt_batch, const int64_t* gt_classes, int32_t G, float* per_image,
                       float* loss, void* stream);

/* ABI version / build info. prpe_source_hash: sha256 (hex) of the sources the library was built
 * from (csrc/*.hip, csrc/*.h, include/prpe.h; computed by build.py), so a host binding can refuse
 * a library built from other sources than the ones beside it. */
int prpe_abi_version(void);
const char* prpe_build_info(void);
const char* prpe_source_hash(void);

#ifdef __cplusplus
}
#endif
#endif /* PRPE_H_ */
