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
#include <stdlib.h>

namespace {

constexpr int AL = 192;        // tokens
constexpr int AD = 64;         // head dim
// bf16 per K row in LDS: a 160-B pitch (10 16-B slots). A ds_read_b128 of the K fragment is
// serviced in 16-lane groups holding rows fr = {0-3, 12-15} at slot fg and rows {4-11} at slot
// fg + 1 (MI355X_MICROARCH.md, LDS); with 10 slots per row the first set lands on the even
// slots and the second on the odd ones: conflict-free (the 144-B pitch was 2-way)
constexpr int KROW = AD + 16;
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

// ----------------------------------------------------------------------------- v2
// vit_attention_t_kernel — the same function computed transposed, in key chunks:
//   S^T = K Q^T   (A = K rows from LDS, B = Q^T: the wave's queries, in registers)
//   O^T = V^T P^T (A = V^T from LDS, B = P^T straight from the S^T accumulators)
// The S^T accumulator of a 16-key tile gives lane (fr, fg) keys 4 fg + r of query fr, which is
// exactly a B-fragment of P^T once the K index of a 32-key PV step is taken in the order
// (tile 2c: keys 4 fg .. 4 fg + 3, tile 2c + 1: keys 16 + 4 fg .. 16 + 4 fg + 3) -- so P never
// goes through LDS, and the A-fragment of V^T reads the same two 4-key runs (two 8-B reads).
// Softmax runs over the rows of S^T (a query's keys: 4 r x 4 lane groups x tiles): two
// shuffles per reduction. Keys are processed KC at a time with an online-softmax merge
// (running max m, sum l, rescale of O by exp(m_old - m_new)), so only one chunk of K and V^T is
// staged: 2 x (KC x 72 + 64 x (KC + 8)) bf16 = 36 KB at KC = 64 instead of 137 KB. A wave owns
// QT 16-query tiles (each K / V^T fragment read from LDS feeds QT MFMAs); with QT = 2 a
// workgroup is 6 waves and two or more workgroups share a CU, one staging while another
// computes. 1 / l once per query at the end; O^T rows are d, so each lane stores 4
// consecutive channels (16-B stores).
template <int KC, int QT>
__global__ __launch_bounds__(AL / 16 / QT * 64) __attribute__((amdgpu_waves_per_eu(QT == 2 ? 3 : 4))) void vit_attention_t_kernel(const float* __restrict__ qkv,
                                                                           float* __restrict__ out, int H,
                                                                           float scale) {
  static_assert(AL % KC == 0 && KC % 32 == 0, "key chunk");
  constexpr int NW = AL / 16 / QT;         // waves
  constexpr int NT = NW * 64;
  constexpr int KT = KC / 16;              // 16-key tiles per chunk
  constexpr int VR = KC + 8;               // bf16 per V^T row (pad 16 B)
  constexpr int KSZ = KC * KROW, VSZ = AD * VR;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * KSZ + 2 * VSZ];
  __bf16* Kh = lds;
  __bf16* Kl = lds + KSZ;
  __bf16* Vh = lds + 2 * KSZ;
  __bf16* Vl = lds + 2 * KSZ + VSZ;

  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int HD = H * AD;
  const int64_t rs = 3 * (int64_t)HD;
  const float* base = qkv + (int64_t)b * AL * rs;
  const int q0 = wave * 16 * QT;

  // Q^T B-fragments: lane (fr = query, fg) holds d = 32 ks + 8 fg .. + 7
  bf16x8 qh[QT][2], ql[QT][2];
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    const float* qr = base + (int64_t)(q0 + u * 16 + fr) * rs + h * AD;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const float4 a = *reinterpret_cast<const float4*>(qr + ks * 32 + fg * 8);
      const float4 c = *reinterpret_cast<const float4*>(qr + ks * 32 + fg * 8 + 4);
      const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 hi, lo;
        split_bf16(v[j], hi, lo);
        qh[u][ks][j] = hi; ql[u][ks][j] = lo;
      }
    }
  }

  float m[QT], l[QT];                      // running max / sum of query fr of tile u
  f32x4 o[QT][4];
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    m[u] = -1e30f; l[u] = 0.f;          // finite: exp_hw(-inf) would be NaN
#pragma unroll
    for (int j = 0; j < 4; ++j) o[u][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  for (int c0 = 0; c0 < AL; c0 += KC) {
    __builtin_amdgcn_sched_barrier(0);     // the previous chunk's reads stay above the barrier,
    if (c0) __syncthreads();               // every wave done with the previous chunk
    __builtin_amdgcn_sched_barrier(0);     // this chunk's below it
    // K rows [key][d] as hi/lo: one float4 per item, 8-B LDS writes
    for (int i = tid; i < KC * (AD / 4); i += NT) {
      const int key = i / (AD / 4), d4 = (i % (AD / 4)) * 4;
      const float4 k4 = *reinterpret_cast<const float4*>(base + (c0 + key) * rs + HD + h * AD + d4);
      const float kv[4] = {k4.x, k4.y, k4.z, k4.w};
      bf16x4 khi, klo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        __bf16 hi, lo;
        split_bf16(kv[j], hi, lo);
        khi[j] = hi; klo[j] = lo;
      }
      *reinterpret_cast<bf16x4*>(Kh + key * KROW + d4) = khi;
      *reinterpret_cast<bf16x4*>(Kl + key * KROW + d4) = klo;
    }
    // V^T [d][key]: an item is 4 keys x 4 channels (four float4 loads; 16 consecutive threads
    // cover one key's 64 channels), transposed in registers, 8-B LDS writes of 4 keys
    for (int i = tid; i < (KC / 4) * (AD / 4); i += NT) {
      const int k4 = i / (AD / 4), d4 = (i % (AD / 4)) * 4;
      float v[4][4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const float4 t = *reinterpret_cast<const float4*>(base + (c0 + k4 * 4 + kk) * rs + 2 * HD + h * AD + d4);
        v[kk][0] = t.x; v[kk][1] = t.y; v[kk][2] = t.z; v[kk][3] = t.w;
      }
#pragma unroll
      for (int dd = 0; dd < 4; ++dd) {
        bf16x4 vhi, vlo;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          __bf16 hi, lo;
          split_bf16(v[kk][dd], hi, lo);
          vhi[kk] = hi; vlo[kk] = lo;
        }
        *reinterpret_cast<bf16x4*>(Vh + (d4 + dd) * VR + k4 * 4) = vhi;
        *reinterpret_cast<bf16x4*>(Vl + (d4 + dd) * VR + k4 * 4) = vlo;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);

    // S^T tiles: rows = keys c0 + 16 t + 4 fg + r, column = query q0 + 16 u + fr
    f32x4 s[QT][KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
#pragma unroll
      for (int u = 0; u < QT; ++u) s[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int off = (t * 16 + fr) * KROW + ks * 32 + fg * 8;
        const bf16x8 kh = *reinterpret_cast<const bf16x8*>(Kh + off);
        const bf16x8 kl = *reinterpret_cast<const bf16x8*>(Kl + off);
#pragma unroll
        for (int u = 0; u < QT; ++u) {
          s[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kl, qh[u][ks], s[u][t], 0, 0, 0);
          s[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kh, ql[u][ks], s[u][t], 0, 0, 0);
          s[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kh, qh[u][ks], s[u][t], 0, 0, 0);
        }
      }
    }
    // online softmax over this chunk's keys, per query
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) { s[u][t][r] *= scale; mx = fmaxf(mx, s[u][t][r]); }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[u], mx);
      const float alpha = exp_hw(m[u] - mn);   // 0 on the first chunk (m = -1e30)
      m[u] = mn;
      float sum = 0.f;
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) { const float e = exp_hw(s[u][t][r] - mn); s[u][t][r] = e; sum += e; }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      l[u] = l[u] * alpha + sum;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[u][j] *= alpha;
    }

    // O^T += V^T P^T, 32 keys per step
#pragma unroll
    for (int c = 0; c < KT / 2; ++c) {
      bf16x8 ph[QT], pl[QT];
#pragma unroll
      for (int u = 0; u < QT; ++u)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          __bf16 hi, lo;
          split_bf16(s[u][2 * c + (jj >> 2)][jj & 3], hi, lo);
          ph[u][jj] = hi; pl[u][jj] = lo;
        }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int off = (j * 16 + fr) * VR + c * 32 + fg * 4;
        const bf16x4 h0 = *reinterpret_cast<const bf16x4*>(Vh + off);
        const bf16x4 h1 = *reinterpret_cast<const bf16x4*>(Vh + off + 16);
        const bf16x4 l0 = *reinterpret_cast<const bf16x4*>(Vl + off);
        const bf16x4 l1 = *reinterpret_cast<const bf16x4*>(Vl + off + 16);
        const bf16x8 vh = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        const bf16x8 vl = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
#pragma unroll
        for (int u = 0; u < QT; ++u) {
          o[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vl, ph[u], o[u][j], 0, 0, 0);
          o[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh, pl[u], o[u][j], 0, 0, 0);
          o[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh, ph[u], o[u][j], 0, 0, 0);
        }
      }
    }
  }
  // out[b*L + q][h*D + d], d = 16 j + 4 fg + r: one 16-B store per tile
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    const float inv = __builtin_amdgcn_rcpf(l[u]);
    float* orow = out + ((int64_t)b * AL + q0 + u * 16 + fr) * HD + h * AD + fg * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4*>(orow + j * 16) = o[u][j] * inv;
  }
}

// ----------------------------------------------------------------------------- v3
// vit_attention_s_kernel — the transposed chunked kernel above (QT = 1, 12 waves) as a
// software pipeline over a STREAM of (head, key-chunk) items: a workgroup owns `hpw` heads of
// one frame and walks their 192 / KC chunks each; the fp32 K / V (and, at a head's first
// chunk, Q) of item i + 1 are loaded into registers while item i computes, and written to LDS
// (split into planes) after the barrier that retires item i's reads. Only the very first
// item's loads are exposed; the kernel reads q, k, v once and writes o once, so it is bound by
// that HBM traffic (4 x 4 B x L x H x D per frame), not by the MFMAs.
// element strides of the q / k / v operand: frame, q->k->v, head, token (channel stride 1)
struct AttnStrides {
  int64_t frame, which, head, tok;
};

template <int KC, bool OPL>
__global__ __launch_bounds__(NWAVE * 64) void vit_attention_s_kernel(const float* __restrict__ qkv, AttnStrides sd,
                                                                    float* __restrict__ out, int H, int hpw,
                                                                    float scale) {
  static_assert(AL % KC == 0 && KC % 32 == 0, "key chunk");
  constexpr int NT = NWAVE * 64;
  constexpr int NCH = AL / KC;
  constexpr int KT = KC / 16;
  constexpr int VR = KC + 8;
  constexpr int KSZ = KC * KROW, VSZ = AD * VR;
  constexpr int KN = KC * (AD / 4);                      // float4 of K per chunk
  constexpr int VN = (KC / 4) * (AD / 4);                // 4x4 V items per chunk
  constexpr int KPT = (KN + NT - 1) / NT, VPT = (VN + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * KSZ + 2 * VSZ];
  __bf16* Kh = lds;
  __bf16* Kl = lds + KSZ;
  __bf16* Vh = lds + 2 * KSZ;
  __bf16* Vl = lds + 2 * KSZ + VSZ;

  const int groups = H / hpw;
  const int b = blockIdx.x / groups, h0 = (blockIdx.x % groups) * hpw;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int HD = H * AD;
  const int64_t rs = sd.tok;
  const float* base = qkv + (int64_t)b * sd.frame;
  const int q0 = wave * 16;
  const int nit = hpw * NCH;

  // register stage of one item
  float4 kr[KPT], vr[VPT][4], qr[4];
  auto fetch = [&](int it) {
    const int hh = h0 + it / NCH, c0 = (it % NCH) * KC;
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const int i = tid + j * NT;
      if (i < KN) {
        const int key = i / (AD / 4), d4 = (i % (AD / 4)) * 4;
        kr[j] = *reinterpret_cast<const float4*>(base + (c0 + key) * rs + sd.which + hh * sd.head + d4);
      }
    }
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int i = tid + j * NT;
      if (i < VN) {
        const int k4 = i / (AD / 4), d4 = (i % (AD / 4)) * 4;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          vr[j][kk] = *reinterpret_cast<const float4*>(base + (c0 + k4 * 4 + kk) * rs + 2 * sd.which + hh * sd.head +
                                                      d4);
      }
    }
    if (it % NCH == 0) {
      const float* q = base + (int64_t)(q0 + fr) * rs + hh * sd.head;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        qr[2 * ks] = *reinterpret_cast<const float4*>(q + ks * 32 + fg * 8);
        qr[2 * ks + 1] = *reinterpret_cast<const float4*>(q + ks * 32 + fg * 8 + 4);
      }
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const int i = tid + j * NT;
      if (i < KN) {
        const int key = i / (AD / 4), d4 = (i % (AD / 4)) * 4;
        const float kv[4] = {kr[j].x, kr[j].y, kr[j].z, kr[j].w};
        bf16x4 khi, klo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          __bf16 hi, lo;
          split_bf16(kv[e], hi, lo);
          khi[e] = hi; klo[e] = lo;
        }
        *reinterpret_cast<bf16x4*>(Kh + key * KROW + d4) = khi;
        *reinterpret_cast<bf16x4*>(Kl + key * KROW + d4) = klo;
      }
    }
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int i = tid + j * NT;
      if (i < VN) {
        const int k4 = i / (AD / 4), d4 = (i % (AD / 4)) * 4;
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) {
          bf16x4 vhi, vlo;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            __bf16 hi, lo;
            split_bf16(vr[j][kk][dd], hi, lo);
            vhi[kk] = hi; vlo[kk] = lo;
          }
          *reinterpret_cast<bf16x4*>(Vh + (d4 + dd) * VR + k4 * 4) = vhi;
          *reinterpret_cast<bf16x4*>(Vl + (d4 + dd) * VR + k4 * 4) = vlo;
        }
      }
    }
  };

  bf16x8 qh[2], ql[2];
  float m = -1e30f, l = 0.f;                             // finite: exp_hw(-inf) would be NaN
  f32x4 o[4];
  fetch(0);
  for (int it = 0; it < nit; ++it) {
    const int c = it % NCH;
    if (c == 0) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const float v[8] = {qr[2 * ks].x, qr[2 * ks].y, qr[2 * ks].z, qr[2 * ks].w,
                            qr[2 * ks + 1].x, qr[2 * ks + 1].y, qr[2 * ks + 1].z, qr[2 * ks + 1].w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 hi, lo;
          split_bf16(v[j], hi, lo);
          qh[ks][j] = hi; ql[ks][j] = lo;
        }
      }
      m = -1e30f; l = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();                                     // item it-1's LDS reads retired
    stage();
    if (it + 1 < nit) fetch(it + 1);                     // in flight across this item's MFMAs
    __syncthreads();

    f32x4 s[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int off = (t * 16 + fr) * KROW + ks * 32 + fg * 8;
        const bf16x8 kh = *reinterpret_cast<const bf16x8*>(Kh + off);
        const bf16x8 kl = *reinterpret_cast<const bf16x8*>(Kl + off);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kl, qh[ks], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kh, ql[ks], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kh, qh[ks], acc, 0, 0, 0);
      }
      s[t] = acc;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s[t][r] *= scale; mx = fmaxf(mx, s[t][r]); }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = exp_hw(m - mn);
    m = mn;
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) { const float e = exp_hw(s[t][r] - mn); s[t][r] = e; sum += e; }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    l = l * alpha + sum;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] *= alpha;
#pragma unroll
    for (int cc = 0; cc < KT / 2; ++cc) {
      bf16x8 ph, pl;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        __bf16 hi, lo;
        split_bf16(s[2 * cc + (jj >> 2)][jj & 3], hi, lo);
        ph[jj] = hi; pl[jj] = lo;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int off = (j * 16 + fr) * VR + cc * 32 + fg * 4;
        const bf16x4 a0 = *reinterpret_cast<const bf16x4*>(Vh + off);
        const bf16x4 a1 = *reinterpret_cast<const bf16x4*>(Vh + off + 16);
        const bf16x4 b0 = *reinterpret_cast<const bf16x4*>(Vl + off);
        const bf16x4 b1 = *reinterpret_cast<const bf16x4*>(Vl + off + 16);
        const bf16x8 vh = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        const bf16x8 vl = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vl, ph, o[j], 0, 0, 0);
        o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh, pl, o[j], 0, 0, 0);
        o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh, ph, o[j], 0, 0, 0);
      }
    }
    if (c == NCH - 1) {
      const float inv = __builtin_amdgcn_rcpf(l);
      float* prow = out + ((int64_t)b * AL + q0 + fr) * HD;
      const int c0 = (h0 + it / NCH) * AD + fg * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (OPL) store_planes4(reinterpret_cast<uint16_t*>(prow), c0 + j * 16, o[j] * inv);
        else *reinterpret_cast<f32x4*>(prow + c0 + j * 16) = o[j] * inv;
      }
    }
  }
}

// ----------------------------------------------------------------------------- v4
// vit_attention_h_kernel (round 5) -- whole heads: a workgroup owns `hpw` heads of one frame and
// stages each head's K and V^T for ALL 192 keys once (split-bf16 planes, 110 KB of LDS), so a
// head costs two barriers (v3: two per 64-key chunk, six per head) and the softmax runs over two
// 96-key halves in registers (one online merge; the whole row would be 48 score registers per lane
// and spill beside the next head's prefetch). The
// fp32 K / V of head h + 1 are loaded into registers while head h computes (issued right after
// head h's staging, consumed by the next staging; Q at the top of its own head), so the HBM
// reads -- the kernel's bound:
// q, k, v read once, o written once -- overlap the MFMAs. Products as v3 (3 bf16 terms for S and
// for PV, transposed: S^T = K Q^T, O^T = V^T P^T with P taken straight from the S^T accumulators).
template <bool OPL>
__global__ __launch_bounds__(NWAVE * 64) void vit_attention_h_kernel(const float* __restrict__ qkv, AttnStrides sd,
                                                                    float* __restrict__ out, int H, int hpw,
                                                                    float scale) {
  constexpr int NT = NWAVE * 64;
  constexpr int KT = AL / 16;                             // 12 key tiles
  // V^T rows of AL + 16 bf16 with the 4-key chunk index XOR-swizzled by (d >> 2) & 15 (d = the
  // row): the staging writes (16 lanes = 16 rows four apart, one chunk) were 8-way bank conflicts
  // on the unswizzled 200-wide rows -- 448 extra LDS cycles per head and wave group, the bulk of
  // SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 0.475 (profiles/r05_attn_pmc.txt) -- and are
  // conflict-free now, as the PV fragment reads stay (simulated with the MI355X_MICROARCH bank
  // rules: ds_write_b64 4 x 16 lanes mod 32, ds_read_b64 2 x 32 lanes mod 64)
  constexpr int VR = AL + 16;
  auto vsw = [](int d, int k4) { return (k4 ^ ((d >> 2) & 15)) * 4; };
  constexpr int KSZ = AL * KROW, VSZ = AD * VR;
  constexpr int KN = AL * (AD / 4);                       // float4 of K per head: 3072
  constexpr int VN = (AL / 4) * (AD / 4);                 // 4 keys x 4 channels V items: 768
  constexpr int KPT = KN / NT, VPT = VN / NT;             // 4, 1 per thread
  static_assert(KN % NT == 0 && VN % NT == 0, "whole items per thread");
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * KSZ + 2 * VSZ];
  __bf16* Kh = lds;
  __bf16* Kl = lds + KSZ;
  __bf16* Vh = lds + 2 * KSZ;
  __bf16* Vl = lds + 2 * KSZ + VSZ;

  const int groups = H / hpw;
  const int b = blockIdx.x / groups, h0 = (blockIdx.x % groups) * hpw;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t rs = sd.tok;
  const float* base = qkv + (int64_t)b * sd.frame;
  const int q0 = wave * 16;

  // the frame's q / k / v through one buffer descriptor: ONE 32-bit per-thread offset per operand
  // kind, the head / key-block / kk parts as scalar offsets (64-bit per-item pointers needed ~40
  // VGPRs beside the prefetch registers and spilled)
  const int frame_bytes = (int)(((int64_t)(AL - 1) * rs + 2 * sd.which + (int64_t)(H - 1) * sd.head + AD) * 4);
  const __amdgpu_buffer_rsrc_t fr_rsrc = buf_rsrc(base, frame_bytes);
  const unsigned kvo = (unsigned)(((int64_t)(tid / (AD / 4)) * rs + (tid % (AD / 4)) * 4) * 4);      // K item j: + 48 j keys
  const unsigned vvo = (unsigned)(((int64_t)(tid / (AD / 4)) * 4 * rs + (tid % (AD / 4)) * 4) * 4);  // V item: keys 4 k4 + kk
  const unsigned qvo = (unsigned)(((int64_t)(q0 + fr) * rs + fg * 8) * 4);
  static_assert(KPT * NT / (AD / 4) == AL && VPT == 1, "item maps");
  f32x4 kr[KPT], vr[VPT][4], qr[4];   // native vectors (arrays of HIP float4 structs go to scratch)
  auto ld4 = [&](unsigned vo, int64_t so) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(fr_rsrc, vo, (int)so, 0));
  };
  auto fetch = [&](int hh) {
    const int64_t hb = (int64_t)hh * sd.head * 4;
#pragma unroll
    for (int j = 0; j < KPT; ++j) kr[j] = ld4(kvo, hb + sd.which * 4 + (int64_t)j * (NT / (AD / 4)) * rs * 4);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) vr[0][kk] = ld4(vvo, hb + 2 * sd.which * 4 + (int64_t)kk * rs * 4);
  };
  // the wave's 16 queries of head hh: loaded at the top of the head's iteration (their latency
  // runs under the first barrier and the staging), so they are not live across the MFMAs
  auto fetch_q = [&](int hh) {
    const int64_t hb = (int64_t)hh * sd.head * 4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qr[2 * ks] = ld4(qvo, hb + ks * 128);
      qr[2 * ks + 1] = ld4(qvo, hb + ks * 128 + 16);
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const int i = tid + j * NT;
      const int key = i / (AD / 4), d4 = (i % (AD / 4)) * 4;
      const float kv[4] = {kr[j][0], kr[j][1], kr[j][2], kr[j][3]};
      bf16x4 khi, klo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __bf16 hi, lo;
        split_bf16(kv[e], hi, lo);
        khi[e] = hi; klo[e] = lo;
      }
      *reinterpret_cast<bf16x4*>(Kh + key * KROW + d4) = khi;
      *reinterpret_cast<bf16x4*>(Kl + key * KROW + d4) = klo;
    }
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int i = tid + j * NT;
      const int k4 = i / (AD / 4), d4 = (i % (AD / 4)) * 4;
#pragma unroll
      for (int dd = 0; dd < 4; ++dd) {
        bf16x4 vhi, vlo;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          __bf16 hi, lo;
          split_bf16(vr[j][kk][dd], hi, lo);
          vhi[kk] = hi; vlo[kk] = lo;
        }
        *reinterpret_cast<bf16x4*>(Vh + (d4 + dd) * VR + vsw(d4 + dd, k4)) = vhi;
        *reinterpret_cast<bf16x4*>(Vl + (d4 + dd) * VR + vsw(d4 + dd, k4)) = vlo;
      }
    }
  };

  fetch(h0);
  for (int it = 0; it < hpw; ++it) {
    const int hh = h0 + it;
    fetch_q(hh);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();                                     // head it - 1's K / V reads retired
    __builtin_amdgcn_sched_barrier(0);
    stage();
    // the next head's K / V, in flight across this head's MFMAs. Unconditional (the last head
    // re-reads its own, unused): behind a branch, the compiler's waits for the Q loads merged both
    // paths and drained this prefetch (vmcnt(0)) before the MFMAs
    fetch(it + 1 < hpw ? hh + 1 : hh);
    bf16x8 qh[2], ql[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // q pre-scaled by scale * log2(e): the scores come out in base-2 units, so the softmax
      // is v_exp_f32 of (s - max) directly (no per-score scale multiply, no two-part exp(x)
      // argument: ~6 VALU per score less; the fp32 product adds 2^-24 relative to q, far below
      // the 3-term bf16 split's own error)
      const float qs = scale * 1.44269504088896340736f;
      const float v[8] = {qr[2 * ks][0] * qs, qr[2 * ks][1] * qs, qr[2 * ks][2] * qs, qr[2 * ks][3] * qs,
                          qr[2 * ks + 1][0] * qs, qr[2 * ks + 1][1] * qs, qr[2 * ks + 1][2] * qs,
                          qr[2 * ks + 1][3] * qs};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 hi, lo;
        split_bf16(v[j], hi, lo);
        qh[ks][j] = hi; ql[ks][j] = lo;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);

    // two halves of 96 keys (register budget: 24 score registers per lane instead of 48), one
    // online-softmax merge between them: S^T tiles rows = keys 16 t + 4 fg + r, column = query
    // q0 + fr
    float m = -1e30f, sum = 0.f;                         // finite: (-inf) - (-inf) would be NaN
    f32x4 o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int hf = 0; hf < 2; ++hf) {
      constexpr int HT = KT / 2;
      f32x4 sc[HT];
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int off = ((hf * HT + t) * 16 + fr) * KROW + ks * 32 + fg * 8;
          const bf16x8 kh = *reinterpret_cast<const bf16x8*>(Kh + off);
          const bf16x8 kl = *reinterpret_cast<const bf16x8*>(Kl + off);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kl, qh[ks], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kh, ql[ks], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kh, qh[ks], acc, 0, 0, 0);
        }
        sc[t] = acc;
        // (keeps the compiler from hoisting every tile's K fragment reads ahead of the MFMAs)
        if (t % 2 == 1) __builtin_amdgcn_sched_barrier(0);
      }
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, sc[t][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - mn); // 0 for the first half
      m = mn;
      float hs = 0.f;
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) { const float e = __builtin_amdgcn_exp2f(sc[t][r] - mn); sc[t][r] = e; hs += e; }
      hs += __shfl_xor(hs, 16, 64);
      hs += __shfl_xor(hs, 32, 64);
      sum = sum * alpha + hs;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] *= alpha;
      // O^T += V^T P^T, 32 keys per step
#pragma unroll
      for (int cc = 0; cc < HT / 2; ++cc) {
        bf16x8 ph, pl;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          __bf16 hi, lo;
          split_bf16(sc[2 * cc + (jj >> 2)][jj & 3], hi, lo);
          ph[jj] = hi; pl[jj] = lo;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int d = j * 16 + fr, k4 = hf * (AL / 8) + cc * 8 + fg;
          const int off0 = d * VR + vsw(d, k4), off1 = d * VR + vsw(d, k4 + 4);
          const bf16x4 a0 = *reinterpret_cast<const bf16x4*>(Vh + off0);
          const bf16x4 a1 = *reinterpret_cast<const bf16x4*>(Vh + off1);
          const bf16x4 b0 = *reinterpret_cast<const bf16x4*>(Vl + off0);
          const bf16x4 b1 = *reinterpret_cast<const bf16x4*>(Vl + off1);
          const bf16x8 vh = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          const bf16x8 vl = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
          o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vl, ph, o[j], 0, 0, 0);
          o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh, pl, o[j], 0, 0, 0);
          o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh, ph, o[j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const float inv = __builtin_amdgcn_rcpf(sum);
    float* prow = out + ((int64_t)b * AL + q0 + fr) * (H * AD);
    const int c0 = hh * AD + fg * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (OPL) store_planes4(reinterpret_cast<uint16_t*>(prow), c0 + j * 16, o[j] * inv);
      else *reinterpret_cast<f32x4*>(prow + c0 + j * 16) = o[j] * inv;
    }
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

// The same PSA core for token counts whose score matrix does not fit LDS (the yolopt net on raw
// 640x640 frames: P5 20x20 = 400 tokens; the config-2 micro-bench variant): one thread per
// (frame, head, query), keys and values staged through LDS 64 at a time, two passes over the keys
// (the row maximum, then exp(s - max) and the weighted sum of v), the reference's softmax order
// of operations (nn.py:115-118: max-subtracted exp, sum, divide) with the same expf. dk <= 32,
// dh <= 64 (host-checked).
constexpr int PSA_KC = 64;
__global__ __launch_bounds__(256) void psa_attention_stream_kernel(prpe_view qkv, prpe_view out, prpe_view vout,
                                                                   int nh, int dk, int dh, float scale) {
  __shared__ float Ks[PSA_KC][33];
  __shared__ float Vs[PSA_KC][65];
  const int n = blockIdx.x / nh, hd = blockIdx.x - (blockIdx.x / nh) * nh;
  const int W = qkv.w, L = qkv.h * qkv.w;
  const int per = 2 * dk + dh;
  const int i = blockIdx.y * 256 + threadIdx.x;
  const bool live = i < L;
  float q[32];
#pragma unroll
  for (int d = 0; d < 32; ++d)
    q[d] = live && d < dk ? qkv.ptr[voff(qkv, n, i / W, i % W, hd * per + d)] : 0.f;
  auto stage = [&](int j0, bool with_v) {
    __syncthreads();
    for (int e = threadIdx.x; e < PSA_KC * 32; e += 256) {
      const int jj = e / 32, d = e % 32, j = j0 + jj;
      Ks[jj][d] = j < L && d < dk ? qkv.ptr[voff(qkv, n, j / W, j % W, hd * per + dk + d)] : 0.f;
    }
    if (with_v)
      for (int e = threadIdx.x; e < PSA_KC * 64; e += 256) {
        const int jj = e / 64, d = e % 64, j = j0 + jj;
        Vs[jj][d] = j < L && d < dh ? qkv.ptr[voff(qkv, n, j / W, j % W, hd * per + 2 * dk + d)] : 0.f;
      }
    __syncthreads();
  };
  auto score = [&](int jj) {
    float a = 0.f;
    for (int d = 0; d < dk; ++d) a += q[d] * Ks[jj][d];
    return a * scale;
  };
  float m = -INFINITY;
  for (int j0 = 0; j0 < L; j0 += PSA_KC) {
    stage(j0, false);
    const int nj = L - j0 < PSA_KC ? L - j0 : PSA_KC;
    for (int jj = 0; jj < nj; ++jj) m = fmaxf(m, score(jj));
  }
  float sum = 0.f, o[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) o[d] = 0.f;
  for (int j0 = 0; j0 < L; j0 += PSA_KC) {
    stage(j0, true);
    const int nj = L - j0 < PSA_KC ? L - j0 : PSA_KC;
    for (int jj = 0; jj < nj; ++jj) {
      const float pexp = expf(score(jj) - m);
      sum += pexp;
#pragma unroll
      for (int d = 0; d < 64; ++d) o[d] += pexp * Vs[jj][d];
    }
  }
  if (!live) return;
#pragma unroll
  for (int d = 0; d < 64; ++d) {
    if (d >= dh) break;
    out.ptr[voff(out, n, i / W, i % W, hd * dh + d)] = o[d] / sum;
    if (vout.ptr)
      vout.ptr[voff(vout, n, i / W, i % W, hd * dh + d)] = qkv.ptr[voff(qkv, n, i / W, i % W, hd * per + 2 * dk + d)];
  }
}

int attention_launch(const float* qkv, AttnStrides sd, float* out, int32_t B, int32_t L, int32_t H, int32_t D,
                     float scale, int out_planes, void* stream) {
  if (!qkv || !out || B <= 0 || H <= 0 || L != AL || D != AD) return PRPE_EINVAL;
  if ((uintptr_t)qkv % 16 || (uintptr_t)out % 16) return PRPE_EINVAL;
  if (sd.frame % 4 || sd.which % 4 || sd.head % 4 || sd.tok % 4) return PRPE_EINVAL;
  // negative strides are not a layout this entry point takes (prpe.h); the whole-head kernel
  // addresses a frame through one buffer descriptor with 32-bit offsets, so it only takes frames
  // whose q / k / v extent (and therefore every per-thread and scalar offset inside it) is below
  // 2^31 bytes -- a frame-interleaved layout (s_tok = B * 3HD, ...) beyond that goes to the
  // streaming kernel, which addresses with 64-bit pointers
  if (sd.frame < 0 || sd.which < 0 || sd.head < 0 || sd.tok < 0) return PRPE_EINVAL;
  const int64_t frame_extent = ((int64_t)(L - 1) * sd.tok + 2 * sd.which + (int64_t)(H - 1) * sd.head + D) * 4;
  const bool desc_ok = frame_extent < (1LL << 31);
  // PRPE_ATTN selects the kernel for A/B runs: 1 = the round-1 kernel (P through LDS, all 192
  // keys staged, 12 waves), KC*10 + QT = transposed kernel with KC-key chunks and QT query tiles
  // per wave (322, 641, 642, 962); 32 / 64 / 96 = the streaming kernel with that chunk;
  // 4 = the whole-head kernel (v4, round 5); default 4. The streaming and whole-head kernels take
  // strided (e.g. head-major) operands.
  static const int sel = [] {
    const char* e = getenv("PRPE_ATTN");
    return e ? atoi(e) : 4;
  }();
  const bool rowmajor = sd.frame == (int64_t)L * 3 * H * D && sd.which == (int64_t)H * D && sd.head == D &&
                        sd.tok == (int64_t)3 * H * D;
  const dim3 g(B * H);
  hipStream_t st = as_stream(stream);
  // streaming kernel: heads per workgroup = the largest divisor of H that still gives every CU
  // a workgroup (one 12-wave workgroup per CU at its register count)
  int hpw = H;
  while (hpw > 1 && ((int64_t)B * H / hpw < 256 || H % hpw)) --hpw;
  const dim3 gs(B * H / hpw);
  if (out_planes) {
    if ((uintptr_t)out % 32) return PRPE_EINVAL;
    if (sel == 4 && desc_ok) hipLaunchKernelGGL((vit_attention_h_kernel<true>), gs, dim3(NWAVE * 64), 0, st, qkv, sd, out, H, hpw, scale);
    else hipLaunchKernelGGL((vit_attention_s_kernel<64, true>), gs, dim3(NWAVE * 64), 0, st, qkv, sd, out, H, hpw, scale);
    return launch_status();
  }
  if (sel == 4 && desc_ok) {
    hipLaunchKernelGGL((vit_attention_h_kernel<false>), gs, dim3(NWAVE * 64), 0, st, qkv, sd, out, H, hpw, scale);
    return launch_status();
  }
  switch (rowmajor ? sel : 64) {
    case 1: hipLaunchKernelGGL(vit_attention_kernel, g, dim3(NWAVE * 64), 0, st, qkv, out, H, scale); break;
    case 322: hipLaunchKernelGGL((vit_attention_t_kernel<32, 2>), g, dim3(6 * 64), 0, st, qkv, out, H, scale); break;
    case 641: hipLaunchKernelGGL((vit_attention_t_kernel<64, 1>), g, dim3(12 * 64), 0, st, qkv, out, H, scale); break;
    case 642: hipLaunchKernelGGL((vit_attention_t_kernel<64, 2>), g, dim3(6 * 64), 0, st, qkv, out, H, scale); break;
    case 962: hipLaunchKernelGGL((vit_attention_t_kernel<96, 2>), g, dim3(6 * 64), 0, st, qkv, out, H, scale); break;
    case 32: hipLaunchKernelGGL((vit_attention_s_kernel<32, false>), gs, dim3(NWAVE * 64), 0, st, qkv, sd, out, H, hpw, scale); break;
    case 96: hipLaunchKernelGGL((vit_attention_s_kernel<96, false>), gs, dim3(NWAVE * 64), 0, st, qkv, sd, out, H, hpw, scale); break;
    default: hipLaunchKernelGGL((vit_attention_s_kernel<64, false>), gs, dim3(NWAVE * 64), 0, st, qkv, sd, out, H, hpw, scale); break;
  }
  return launch_status();
}

}  // namespace

extern "C" int prpe_attention(const float* qkv, float* out, int32_t B, int32_t L, int32_t H, int32_t D,
                              float scale, void* stream) {
  const int64_t HD = (int64_t)H * D;
  return attention_launch(qkv, AttnStrides{(int64_t)L * 3 * HD, HD, D, 3 * HD}, out, B, L, H, D, scale, 0, stream);
}

extern "C" int prpe_attention_strided(const float* qkv, int64_t s_frame, int64_t s_which, int64_t s_head,
                                      int64_t s_tok, float* out, int32_t B, int32_t L, int32_t H, int32_t D,
                                      float scale, int32_t out_planes, void* stream) {
  return attention_launch(qkv, AttnStrides{s_frame, s_which, s_head, s_tok}, out, B, L, H, D, scale, out_planes,
                          stream);
}

extern "C" int prpe_psa_attention(const prpe_view* qkv, const prpe_view* out, const prpe_view* vout, int32_t nh,
                                  int32_t dk, int32_t dh, float scale, void* stream) {
  if (!view_ok(qkv) || !view_ok(out) || nh <= 0 || dk <= 0 || dh <= 0) return PRPE_EINVAL;
  if (qkv->c != nh * (2 * dk + dh) || out->c != nh * dh || qkv->n != out->n) return PRPE_EINVAL;
  const int L = qkv->h * qkv->w;
  const size_t shm = sizeof(float) * (size_t)nh * L * L;
  prpe_view vo{};
  if (vout && vout->ptr) {
    if (vout->c != out->c || vout->n != out->n || vout->h != out->h || vout->w != out->w) return PRPE_EINVAL;
    vo = *vout;
  }
  if (shm > 64 * 1024) {                   // scores do not fit LDS: the streaming form
    if (dk > 32 || dh > 64 || (int64_t)qkv->n * nh >= (1LL << 31)) return PRPE_EINVAL;
    hipLaunchKernelGGL(psa_attention_stream_kernel, dim3(qkv->n * nh, (L + 255) / 256), dim3(256), 0,
                       as_stream(stream), *qkv, *out, vo, nh, dk, dh, scale);
    return launch_status();
  }
  hipLaunchKernelGGL(psa_attention_kernel, dim3(qkv->n), dim3(256), shm, as_stream(stream), *qkv, *out, vo, nh, dk,
                     dh, scale);
  return launch_status();
}
