// Full-window convolutions with one output pixel per frame (a linear over the flattened frame:
// M = frames, K = KH*KW*Ci, N = Co), split along K. The IR-50 output layer (BN2d -> Flatten ->
// Linear(25088 -> 512) -> BN1d, net_adaface.py output_layer) is this shape: M = 256, N = 512,
// K = 25,088. Tiled only over M x N it has 8..64 workgroups for 256 CUs (0.65 ms at bs = 256,
// 10 TF/s, profiles/r02_layer_profile_*); split into one K-slice per (kh, kw) tap it has
// ceil(M/64) x Co/64 x KH*KW workgroups.
//
// Stage 1 (linear_splitk_kernel): workgroup (n-tile, m-tile, slice s) = 4 waves, each 16 frames
// x 64 output channels over the slice's K range; A straight from global (the frame's contiguous
// NHWC row, the prologue BN applied, split into two bf16 planes), B = the weights' hi / lo
// planes (tap-major pack, k = (kh*KW + kw)*Ci + ci = the NHWC flatten order), three products per
// pair as at precision 0 everywhere. Raw partial sums -> workspace [S][M][Co].
// Stage 2 (linear_splitk_reduce): y = EPI(sum_s part[s]) in slice order (deterministic), with
// the epilogue's scale / bias / activation.
// The partial sums go to the caller's workspace (prpe_conv2d_workspace_bytes; the library
// never allocates), so concurrent calls on different streams use different buffers.
#include "conv.h"

namespace prpe_k {
namespace {

__global__ __launch_bounds__(256) void linear_splitk_kernel(ConvK p, float* __restrict__ part, int kslice) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int n0 = blockIdx.x * 64, m0 = blockIdx.y * 64 + wave * 16, s = blockIdx.z;
  const int m = min(m0 + fr, p.M - 1);                  // clamped rows are computed, not stored
  const float* xr = p.x + (int64_t)m * p.xsn;
  const int k0 = s * kslice;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint16_t* bh = p.whi + (int64_t)(n0 + fr) * p.k_pad;
  const uint16_t* bl = p.wlo + (int64_t)(n0 + fr) * p.k_pad;
  const int64_t bstep = (int64_t)16 * p.k_pad;          // next 16 output channels
  for (int kk = 0; kk < kslice; kk += 32) {
    const int k = k0 + kk + fg * 8;
    f4 v0 = *reinterpret_cast<const f4*>(xr + k);
    f4 v1 = *reinterpret_cast<const f4*>(xr + k + 4);
    if (p.in_scale) {
      const int ci = k % p.Ci;                          // 8 consecutive channels (Ci % 8 == 0)
      v0 = v0 * *reinterpret_cast<const f4*>(p.in_scale + ci) + *reinterpret_cast<const f4*>(p.in_bias + ci);
      v1 = v1 * *reinterpret_cast<const f4*>(p.in_scale + ci + 4) + *reinterpret_cast<const f4*>(p.in_bias + ci + 4);
    }
    bf16x4 p0[2], p1[2];
    split_planes<2>(v0, p0);
    split_planes<2>(v1, p1);
    bf16x8 a[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) a[q] = bf16x8{p0[q][0], p0[q][1], p0[q][2], p0[q][3], p1[q][0], p1[q][1], p1[q][2], p1[q][3]};
    bf16x8 b0[4], b1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      b0[j] = *reinterpret_cast<const bf16x8*>(bh + j * bstep + k);
      b1[j] = *reinterpret_cast<const bf16x8*>(bl + j * bstep + k);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] = mfma16(a[1], b0[j], acc[j]);
      acc[j] = mfma16(a[0], b1[j], acc[j]);
      acc[j] = mfma16(a[0], b0[j], acc[j]);
    }
  }
  // C layout of the 16x16 MFMA: rows fg*4 + r, column fr
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int mm = m0 + fg * 4 + r;
    if (mm >= p.M) continue;
    float* o = part + ((int64_t)s * p.M + mm) * p.Co + n0 + fr;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j * 16] = acc[j][r];
  }
}

__global__ __launch_bounds__(256) void linear_splitk_reduce(ConvK p, const float* __restrict__ part, int S) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;   // one float4 of y
  const int64_t total4 = (int64_t)p.M * p.Co / 4;
  if (i >= total4) return;
  const int m = (int)(i * 4 / p.Co), c = (int)(i * 4 - (int64_t)m * p.Co);
  f4 v = {0.f, 0.f, 0.f, 0.f};
  const int64_t plane = (int64_t)p.M * p.Co;
  for (int s = 0; s < S; ++s) v += *reinterpret_cast<const f4*>(part + s * plane + i * 4);
  f4 sc = {1.f, 1.f, 1.f, 1.f}, bi = {0.f, 0.f, 0.f, 0.f}, sl = {0.f, 0.f, 0.f, 0.f};
  if (p.scale) sc = *reinterpret_cast<const f4*>(p.scale + c);
  if (p.bias) bi = *reinterpret_cast<const f4*>(p.bias + c);
  if (p.slope) sl = *reinterpret_cast<const f4*>(p.slope + c);
  v = v * sc + bi;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = apply_act(v[q], p.act, sl[q]);
  *reinterpret_cast<f4*>(p.y + (int64_t)m * p.ysn + c) = v;
}

}  // namespace

bool conv_splitk_eligible(const ConvK& kp, int prec, int k_order) {
  // one output pixel per frame over the whole (unpadded) input, frames' NHWC rows contiguous,
  // tap-major weights, 64-column tiles, plain fp32 output, precision 0
  return prec == 0 && k_order == 0 && kp.Ho == 1 && kp.Wo == 1 && kp.pad == 0 && kp.KH == kp.Hi &&
         kp.KW == kp.Wi && kp.xsc == 1 && (kp.Wi == 1 || kp.xsw == kp.Ci) &&
         (kp.Hi == 1 || kp.xsh == (int64_t)kp.Wi * kp.Ci) && kp.Ci % 32 == 0 &&   // size-1 dims: any stride
         kp.Co % 64 == 0 && kp.ysc == 1 && kp.res_mode == PRPE_RES_NONE && !kp.x_planes && !kp.y_planes &&
         !kp.y_amax && !kp.x2 && !kp.w2 && kp.K == kp.k_pad && (uintptr_t)kp.x % 16 == 0 &&
         (uintptr_t)kp.y % 16 == 0 && kp.ysn % 4 == 0 && kp.xsn % 4 == 0 &&
         (!kp.in_scale || (kp.in_bias && (uintptr_t)kp.in_scale % 16 == 0 && (uintptr_t)kp.in_bias % 16 == 0)) &&
         (!kp.scale || (uintptr_t)kp.scale % 16 == 0) && (!kp.bias || (uintptr_t)kp.bias % 16 == 0) &&
         (!kp.slope || (uintptr_t)kp.slope % 16 == 0);
}

// one K-slice per tap when the taps are >= 256 deep, else slices of 8 K-steps
static int splitk_slice(const ConvK& kp) {
  int kslice = kp.KH * kp.KW > 1 && kp.Ci >= 256 ? kp.Ci : 256;
  if (kp.K % kslice) kslice = 32;
  return kslice;
}

int64_t conv_splitk_workspace_bytes(const ConvK& kp) {
  const int64_t S = kp.K / splitk_slice(kp);
  return S * kp.M * kp.Co * (int64_t)sizeof(float);
}

int conv_splitk_launch(const ConvK& kp, float* ws, hipStream_t st) {
  const int kslice = splitk_slice(kp);
  const int S = kp.K / kslice;
  const dim3 g1(kp.Co / 64, (kp.M + 63) / 64, S);
  hipLaunchKernelGGL(linear_splitk_kernel, g1, dim3(256), 0, st, kp, ws, kslice);
  const int64_t total4 = (int64_t)kp.M * kp.Co / 4;
  hipLaunchKernelGGL(linear_splitk_reduce, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, st, kp,
                     (const float*)ws, S);
  return launch_status();
}

}  // namespace prpe_k
