// Attention kernels.
//
// prpe_attention — ViTPose-B self-attention (L = 192 tokens, D = 64, 12 heads), one
// workgroup per (frame, head), one wave per 16-query tile (12 waves = 768 threads).
// K and V of the head are staged once in LDS as split-bf16 (hi, lo) planes; V is stored
// transposed so its B-fragments are contiguous. S = Q K^T and O = P V run on
// v_mfma_f32_16x16x32_bf16 with the 3-pass split (lo*hi + hi*lo + hi*hi), fp32 softmax in
// registers (row = 4*(lane>>4)+r of the 16x16 accumulator, 16 lanes per row), P re-staged
// through a per-wave LDS slab 32 keys at a time as the A operand of PV.
// Reference: eager_attention_forward (modeling_vitpose_backbone.py:100-126):
//   softmax(matmul(q, k^T) * scaling) @ v.
//
// prpe_psa_attention — YOLO v11 PSA attention core (nn.py:111-122), 25 tokens, 2 heads;
// tiny, VALU fp32, one workgroup per frame.
#include "common.h"

namespace {

constexpr int AL = 192;        // tokens
constexpr int AD = 64;         // head dim
constexpr int KROW = AD + 8;   // bf16 per K row in LDS (pad 16 B)
constexpr int VROW = AL + 8;   // bf16 per V^T row in LDS (pad 16 B)
constexpr int NWAVE = AL / 16; // 12

__global__ __launch_bounds__(NWAVE * 64) void vit_attention_kernel(const float* __restrict__ qkv,
                                                                   float* __restrict__ out, int H, float scale) {
  __shared__ __attribute__((aligned(16))) __bf16 Kh[AL * KROW];
  __shared__ __attribute__((aligned(16))) __bf16 Kl[AL * KROW];
  __shared__ __attribute__((aligned(16))) __bf16 Vh[AD * VROW];
  __shared__ __attribute__((aligned(16))) __bf16 Vl[AD * VROW];
  __shared__ __attribute__((aligned(16))) __bf16 Ph[NWAVE][16 * 40];
  __shared__ __attribute__((aligned(16))) __bf16 Pl[NWAVE][16 * 40];

  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int HD = H * AD;
  const int64_t rs = 3 * (int64_t)HD;             // qkv row stride
  const float* base = qkv + (int64_t)b * AL * rs;

  // stage K (row-major [key][d]) and V^T ([d][key]) as hi/lo bf16
  for (int i = tid; i < AL * AD / 4; i += NWAVE * 64) {
    const int key = i / (AD / 4), d4 = (i % (AD / 4)) * 4;
    const float4 k4 = *reinterpret_cast<const float4*>(base + key * rs + HD + h * AD + d4);
    const float4 v4 = *reinterpret_cast<const float4*>(base + key * rs + 2 * HD + h * AD + d4);
    const float kv[4] = {k4.x, k4.y, k4.z, k4.w};
    const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
    bf16x4 khi, klo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      __bf16 hi, lo;
      split_bf16(kv[j], hi, lo);
      khi[j] = hi; klo[j] = lo;
      split_bf16(vv[j], hi, lo);
      Vh[(d4 + j) * VROW + key] = hi; Vl[(d4 + j) * VROW + key] = lo;
    }
    *reinterpret_cast<bf16x4*>(Kh + key * KROW + d4) = khi;     // one 8-B LDS write per plane
    *reinterpret_cast<bf16x4*>(Kl + key * KROW + d4) = klo;
  }

  // Q fragments straight from global: A[row = query][k = d]
  const int fr = lane & 15, fg = lane >> 4;
  const int q0 = wave * 16;
  bf16x8 qh[2], ql[2];
  {
    const float* qr = base + (int64_t)(q0 + fr) * rs + h * AD;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const float4 a = *reinterpret_cast<const float4*>(qr + ks * 32 + fg * 8);
      const float4 c = *reinterpret_cast<const float4*>(qr + ks * 32 + fg * 8 + 4);
      const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 hi, lo;
        split_bf16(v[j], hi, lo);
        qh[ks][j] = hi; ql[ks][j] = lo;
      }
    }
  }
  __syncthreads();

  // S = Q K^T : 12 key tiles of 16
  f32x4 s[NWAVE];
#pragma unroll
  for (int t = 0; t < NWAVE; ++t) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int off = (t * 16 + fr) * KROW + ks * 32 + fg * 8;
      const bf16x8 kh = *reinterpret_cast<const bf16x8*>(Kh + off);
      const bf16x8 kl = *reinterpret_cast<const bf16x8*>(Kl + off);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ql[ks], kh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qh[ks], kl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qh[ks], kh, acc, 0, 0, 0);
    }
    s[t] = acc;
  }
  // softmax over keys, rows r: query q0 + 4*fg + r; a row's 192 values = 12 tiles x 16 lanes
  float rmax[4], rsum[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < NWAVE; ++t) { s[t][r] *= scale; m = fmaxf(m, s[t][r]); }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    rmax[r] = m;
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < NWAVE; ++t) { const float e = exp_hw(s[t][r] - m); s[t][r] = e; sum += e; }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 64);
    rsum[r] = __builtin_amdgcn_rcpf(sum);     // P = e * (1 / sum): one rcp per row
  }
  (void)rmax;
  // O = P V, P chunks of 32 keys (2 tiles) through the per-wave LDS slab
  f32x4 o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __bf16* ph = Ph[wave];
  __bf16* pl = Pl[wave];
#pragma unroll
  for (int c = 0; c < NWAVE / 2; ++c) {
    // write P[16 q][32 keys] (normalised) as hi/lo, row stride 40 bf16
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = s[2 * c + tt][r] * rsum[r];
        __bf16 hi, lo;
        split_bf16(pv, hi, lo);
        const int off = (fg * 4 + r) * 40 + tt * 16 + fr;
        ph[off] = hi; pl[off] = lo;
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): slab writes landed
    __builtin_amdgcn_wave_barrier();
    const bf16x8 ah = *reinterpret_cast<const bf16x8*>(ph + fr * 40 + fg * 8);
    const bf16x8 alo = *reinterpret_cast<const bf16x8*>(pl + fr * 40 + fg * 8);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int off = (j * 16 + fr) * VROW + c * 32 + fg * 8;
      const bf16x8 vh = *reinterpret_cast<const bf16x8*>(Vh + off);
      const bf16x8 vl = *reinterpret_cast<const bf16x8*>(Vl + off);
      o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, vh, o[j], 0, 0, 0);
      o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, vl, o[j], 0, 0, 0);
      o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, vh, o[j], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
  // out[b*L + q][h*D + d]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + fg * 4 + r;
      out[((int64_t)b * AL + q) * HD + h * AD + j * 16 + fr] = o[j][r];
    }
}

// ----------------------------------------------------------------------------- PSA
__device__ __forceinline__ int64_t voff(const prpe_view& v, int n, int hh, int ww, int c) {
  return (int64_t)n * v.sn + (int64_t)hh * v.sh + (int64_t)ww * v.sw + (int64_t)c * v.sc;
}

__global__ __launch_bounds__(256) void psa_attention_kernel(prpe_view qkv, prpe_view out, prpe_view vout, int nh,
                                                            int dk, int dh, float scale) {
  extern __shared__ float sm[];
  const int n = blockIdx.x;
  const int W = qkv.w, L = qkv.h * qkv.w;
  const int per = 2 * dk + dh;
  float* S = sm;                       // [nh][L][L]
  for (int e = threadIdx.x; e < nh * L * L; e += blockDim.x) {
    const int hd = e / (L * L), i = (e / L) % L, j = e % L;
    float acc = 0.f;
    for (int d = 0; d < dk; ++d)
      acc += qkv.ptr[voff(qkv, n, i / W, i % W, hd * per + d)] * qkv.ptr[voff(qkv, n, j / W, j % W, hd * per + dk + d)];
    S[e] = acc * scale;
  }
  __syncthreads();
  for (int row = threadIdx.x; row < nh * L; row += blockDim.x) {
    float* sr = S + (int64_t)row * L;
    float m = -INFINITY;
    for (int j = 0; j < L; ++j) m = fmaxf(m, sr[j]);
    float sum = 0.f;
    for (int j = 0; j < L; ++j) { sr[j] = expf(sr[j] - m); sum += sr[j]; }
    for (int j = 0; j < L; ++j) sr[j] = sr[j] / sum;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nh * dh * L; e += blockDim.x) {
    const int hd = e / (dh * L), d = (e / L) % dh, i = e % L;
    const float* pr = S + ((int64_t)hd * L + i) * L;
    float acc = 0.f;
    for (int j = 0; j < L; ++j) acc += qkv.ptr[voff(qkv, n, j / W, j % W, hd * per + 2 * dk + d)] * pr[j];
    out.ptr[voff(out, n, i / W, i % W, hd * dh + d)] = acc;
    if (vout.ptr)
      vout.ptr[voff(vout, n, i / W, i % W, hd * dh + d)] =
          qkv.ptr[voff(qkv, n, i / W, i % W, hd * per + 2 * dk + d)];
  }
}

}  // namespace

extern "C" int prpe_attention(const float* qkv, float* out, int32_t B, int32_t L, int32_t H, int32_t D,
                              float scale, void* stream) {
  if (!qkv || !out || B <= 0 || H <= 0 || L != AL || D != AD) return PRPE_EINVAL;
  if ((uintptr_t)qkv % 16) return PRPE_EINVAL;
  hipLaunchKernelGGL(vit_attention_kernel, dim3(B * H), dim3(NWAVE * 64), 0, as_stream(stream), qkv, out, H, scale);
  return launch_status();
}

extern "C" int prpe_psa_attention(const prpe_view* qkv, const prpe_view* out, const prpe_view* vout, int32_t nh,
                                  int32_t dk, int32_t dh, float scale, void* stream) {
  if (!view_ok(qkv) || !view_ok(out) || nh <= 0 || dk <= 0 || dh <= 0) return PRPE_EINVAL;
  if (qkv->c != nh * (2 * dk + dh) || out->c != nh * dh || qkv->n != out->n) return PRPE_EINVAL;
  const int L = qkv->h * qkv->w;
  const size_t shm = sizeof(float) * (size_t)nh * L * L;
  if (shm > 64 * 1024) return PRPE_EINVAL;
  prpe_view vo{};
  if (vout && vout->ptr) {
    if (vout->c != out->c || vout->n != out->n || vout->h != out->h || vout->w != out->w) return PRPE_EINVAL;
    vo = *vout;
  }
  hipLaunchKernelGGL(psa_attention_kernel, dim3(qkv->n), dim3(256), shm, as_stream(stream), *qkv, *out, vo, nh, dk,
                     dh, scale);
  return launch_status();
}
