// Implicit-GEMM convolution on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), split-bf16 x3.
//
// GEMM view: M = N*Ho*Wo output pixels, N_gemm = Co, K = KH*KW*Ci (k = (kh*KW+kw)*Ci+ci).
//   A[m,k] = PRO(x[n, oh*s-p+kh, ow*s-p+kw, ci])   (gathered on the fly, strided view)
//   B[k,co] = W[co, kh, kw, ci]                    (host-packed bf16 hi/lo planes [co][k])
// Each fp32 operand is split into NP bf16 planes a = a0 + a1 (+ a2) and the wave issues the
// partial products with plane-index sum < NP, smallest first, fp32 accumulate:
//   precision 0 (NP=2): a1*b0 + a0*b1 + a0*b0            ~16-bit operands, 2^-17 rel/product,
//                        1/3 of the dense bf16 MFMA rate (~830 TF/s ceiling)
//   precision 2 (NP=3): a2*b0 + a1*b1 + a0*b2 + a1*b0 + a0*b1 + a0*b0
//                        the 3-way split is exact for fp32 operands: fp32-faithful products
//                        at 1/6 of the bf16 rate (~415 TF/s ceiling vs 157 for f32 MFMA)
//   precision 1 (NP=1): a0*b0 plain bf16 (diagnostics / ablation only)
//
// Tiling: BM x BN x 32, 256 threads = 4 waves (WM x WN), each wave a (BM/WM)x(BN/WN) tile of
// 16x16 MFMA blocks. Global->register prefetch of tile k+1 overlaps the MFMAs of tile k;
// LDS double buffer, one barrier per K-step. LDS rows are 64 B (32 bf16); the 4 16-B slots
// of row r are XOR-permuted by F[(r>>2)&3] = {0,2,3,1}, which makes every ds_read_b128
// lane group of the fragment read hit 16 distinct slots (conflict-free).
// Grid: 1-D, XCD-remapped so the Co-tiles sharing one A panel run on one XCD (shared L2).
//
// Reference arithmetic replaced: torch Conv2d (+BatchNorm2d eval +act +residual) at every
// call site listed in include/prpe.h (prpe_conv2d).
#include "common.h"

namespace {

constexpr int BK = 32;
constexpr int NTHREADS = 256;

struct ConvK {
  const float* x; int64_t xsn, xsh, xsw, xsc; int Hi, Wi, Ci;
  float* y; int64_t ysn, ysh, ysw, ysc; int Ho, Wo, Co;
  const float* r; int64_t rsn, rsh, rsw, rsc;
  int KH, KW, stride, pad, K, k_pad, nk;
  const uint16_t* whi; const uint16_t* wlo; const uint16_t* wlo2;
  const float* scale; const float* bias; const float* slope;
  const float* in_scale; const float* in_bias;
  int act, res_mode;
  int M, HoWo, tiles_n, nwg;
};

__device__ __forceinline__ int swzF(int row) {
  const int q = (row >> 2) & 3;
  return q == 0 ? 0 : q == 1 ? 2 : q == 2 ? 3 : 1;
}

template <int BM, int BN, int WM, int WN, bool VEC, int PREC>
__global__ __launch_bounds__(NTHREADS) void conv_igemm_kernel(ConvK p) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_ROWS_PT = BM / 32;                 // VEC: rows per thread (8 float4 per row)
  constexpr int B_CHUNKS = BN * 4;                   // 16-B chunks per plane per K-step
  constexpr int B_PT = (B_CHUNKS + NTHREADS - 1) / NTHREADS;
  static_assert(WM * WN == 4, "4 waves");
  constexpr int NP = PREC == 1 ? 1 : (PREC == 0 ? 2 : 3);   // bf16 planes per operand
  static_assert(TM >= 1 && TN >= 1, "tile");

  // LDS: [buf][plane][rows][32] bf16 (u16), A then B.
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * NP * (BM + BN) * BK];
  __shared__ int klut[VEC ? 1 : 1024];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int L = xcd_remap(blockIdx.x, p.nwg);
  const int tile_m = L / p.tiles_n, tile_n = L % p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  auto A_at = [&](int buf, int plane) -> uint16_t* { return lds + ((buf * NP + plane) * (BM + BN)) * BK; };
  auto B_at = [&](int buf, int plane) -> uint16_t* { return lds + ((buf * NP + plane) * (BM + BN) + BM) * BK; };

  // ---------------- A-load state
  // VEC: thread -> k chunk c4 = tid&7 (4 floats), rows tid/8 + 32*i.
  // scalar: thread -> row tid % BM, k columns kk0 + (256/BM)*j.
  constexpr int S_ROWS = 1;
  constexpr int S_KPT = (BM * BK) / NTHREADS;          // k elements per thread per step (scalar)
  int64_t rowoff[VEC ? A_ROWS_PT : S_ROWS];
  int ih0[VEC ? A_ROWS_PT : S_ROWS], iw0[VEC ? A_ROWS_PT : S_ROWS];

  auto decode_row = [&](int m, int64_t& off, int& ih, int& iw) {
    if (m < p.M) {
      int n = m / p.HoWo;
      int rem = m - n * p.HoWo;
      int oh = rem / p.Wo;
      int ow = rem - oh * p.Wo;
      off = (int64_t)n * p.xsn;
      ih = oh * p.stride - p.pad;
      iw = ow * p.stride - p.pad;
    } else {
      off = 0; ih = -(1 << 28); iw = -(1 << 28);
    }
  };

  if constexpr (VEC) {
#pragma unroll
    for (int i = 0; i < A_ROWS_PT; ++i) decode_row(m0 + (tid >> 3) + 32 * i, rowoff[i], ih0[i], iw0[i]);
  } else {
    decode_row(m0 + (tid % BM), rowoff[0], ih0[0], iw0[0]);
    // k -> packed (dh, dw, ci) table for this layer (k_pad <= 1024 checked on host)
    for (int k = tid; k < p.k_pad; k += NTHREADS) {
      int v = -1;
      if (k < p.K) {
        int tap = k / p.Ci, ci = k - tap * p.Ci;
        int dh = tap / p.KW, dw = tap - dh * p.KW;
        v = (dh << 24) | (dw << 16) | ci;
      }
      klut[k] = v;
    }
    __syncthreads();
  }

  // VEC incremental (kh, kw, ci) of this thread's chunk
  int c_ci = (tid & 7) * 4, c_kh = 0, c_kw = 0;
  if constexpr (VEC) {
    while (c_ci >= p.Ci) { c_ci -= p.Ci; if (++c_kw == p.KW) { c_kw = 0; ++c_kh; } }
  }

  float4 areg[VEC ? A_ROWS_PT : 1];
  float sreg[VEC ? 1 : S_KPT];
  uint4 breg[NP][B_PT];

  auto load_tile = [&](int kt) {
    if constexpr (VEC) {
      const bool kval = c_kh < p.KH;
      float4 s4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p.in_scale && kval) {
        s4 = *reinterpret_cast<const float4*>(p.in_scale + c_ci);
        b4 = *reinterpret_cast<const float4*>(p.in_bias + c_ci);
      }
#pragma unroll
      for (int i = 0; i < A_ROWS_PT; ++i) {
        const int ih = ih0[i] + c_kh, iw = iw0[i] + c_kw;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (kval && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi) {
          v = *reinterpret_cast<const float4*>(p.x + rowoff[i] + ih * p.xsh + iw * p.xsw + c_ci);
          if (p.in_scale) {
            v.x = v.x * s4.x + b4.x; v.y = v.y * s4.y + b4.y;
            v.z = v.z * s4.z + b4.z; v.w = v.w * s4.w + b4.w;
          }
        }
        areg[i] = v;
      }
      // advance this thread's k by BK
      c_ci += BK;
      while (c_ci >= p.Ci && c_kh < p.KH) { c_ci -= p.Ci; if (++c_kw == p.KW) { c_kw = 0; ++c_kh; } }
    } else {
      const int kk0 = tid / BM;
      constexpr int KSTEP = NTHREADS / BM;
#pragma unroll
      for (int j = 0; j < S_KPT; ++j) {
        const int k = kt * BK + kk0 + KSTEP * j;
        const int e = klut[k];
        float v = 0.f;
        if (e >= 0) {
          const int dh = e >> 24, dw = (e >> 16) & 0xFF, ci = e & 0xFFFF;
          const int ih = ih0[0] + dh, iw = iw0[0] + dw;
          if ((unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi) {
            v = p.x[rowoff[0] + ih * p.xsh + iw * p.xsw + ci * p.xsc];
            if (p.in_scale) v = v * p.in_scale[ci] + p.in_bias[ci];
          }
        }
        sreg[j] = v;
      }
    }
    // B: packed planes [co_pad][k_pad] bf16
#pragma unroll
    for (int j = 0; j < B_PT; ++j) {
      const int c = tid + NTHREADS * j;
      if (B_CHUNKS % NTHREADS == 0 || c < B_CHUNKS) {
        const int row = c >> 2, ch = c & 3;
        const int64_t off = (int64_t)(n0 + row) * p.k_pad + kt * BK + ch * 8;
        breg[0][j] = *reinterpret_cast<const uint4*>(p.whi + off);
        if (NP > 1) breg[1][j] = *reinterpret_cast<const uint4*>(p.wlo + off);
        if (NP > 2) breg[NP - 1][j] = *reinterpret_cast<const uint4*>(p.wlo2 + off);
      }
    }
  };

  auto store_tile = [&](int buf) {
    if constexpr (VEC) {
      const int c4 = tid & 7;
#pragma unroll
      for (int i = 0; i < A_ROWS_PT; ++i) {
        const int row = (tid >> 3) + 32 * i;
        const int slot = (c4 >> 1) ^ swzF(row);
        const int off = row * BK + slot * 8 + (c4 & 1) * 4;
        bf16x4 pl[NP];
        const float4 v = areg[i];
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float r = vv[e];
#pragma unroll
          for (int q = 0; q < NP; ++q) {
            const __bf16 t = (__bf16)r;
            pl[q][e] = t;
            r -= (float)t;
          }
        }
#pragma unroll
        for (int q = 0; q < NP; ++q) *reinterpret_cast<bf16x4*>(A_at(buf, q) + off) = pl[q];
      }
    } else {
      const int row = tid % BM, kk0 = tid / BM;
      constexpr int KSTEP = NTHREADS / BM;
#pragma unroll
      for (int j = 0; j < S_KPT; ++j) {
        const int kk = kk0 + KSTEP * j;
        const int slot = (kk >> 3) ^ swzF(row);
        const int off = row * BK + slot * 8 + (kk & 7);
        float r = sreg[j];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          const __bf16 t = (__bf16)r;
          reinterpret_cast<__bf16*>(A_at(buf, q))[off] = t;
          r -= (float)t;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < B_PT; ++j) {
      const int c = tid + NTHREADS * j;
      if (B_CHUNKS % NTHREADS == 0 || c < B_CHUNKS) {
        const int row = c >> 2, ch = c & 3;
        const int off = row * BK + (ch ^ swzF(row)) * 8;
#pragma unroll
        for (int q = 0; q < NP; ++q) *reinterpret_cast<uint4*>(B_at(buf, q) + off) = breg[q][j];
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;

  auto compute = [&](int buf) {
    bf16x8 af[NP][TM], bfr[NP][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WTM + i * 16 + fr;
      const int off = row * BK + (fg ^ swzF(row)) * 8;
#pragma unroll
      for (int q = 0; q < NP; ++q) af[q][i] = *reinterpret_cast<const bf16x8*>(A_at(buf, q) + off);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn * WTN + j * 16 + fr;
      const int off = row * BK + (fg ^ swzF(row)) * 8;
#pragma unroll
      for (int q = 0; q < NP; ++q) bfr[q][j] = *reinterpret_cast<const bf16x8*>(B_at(buf, q) + off);
    }
    // partial products smallest first; terms with plane-index sum >= NP are dropped
    // (NP=2: lo*hi + hi*lo + hi*hi; NP=3: 2*0 + 1*1 + 0*2 + 1*0 + 0*1 + 0*0)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int s = NP - 1; s >= 0; --s)
#pragma unroll
          for (int qa = s; qa >= 0; --qa)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[qa][i], bfr[s - qa][j], acc[i][j], 0, 0, 0);
      }
  };

  // ---------------- main loop
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < p.nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < p.nk) load_tile(kt + 1);
    compute(cur);
    if (kt + 1 < p.nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue
  float sc[TN], bi[TN], sl[TN];
  int cols[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WTN + j * 16 + fr;
    cols[j] = col;
    const bool cv = col < p.Co;
    sc[j] = (cv && p.scale) ? p.scale[col] : 1.f;
    bi[j] = (cv && p.bias) ? p.bias[col] : 0.f;
    sl[j] = (cv && p.slope) ? p.slope[col] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WTM + i * 16 + fg * 4 + r;
      if (m >= p.M) continue;
      const int n = m / p.HoWo;
      const int rem = m - n * p.HoWo;
      const int oh = rem / p.Wo;
      const int ow = rem - oh * p.Wo;
      const int64_t yo = (int64_t)n * p.ysn + (int64_t)oh * p.ysh + (int64_t)ow * p.ysw;
      const int64_t ro = (int64_t)n * p.rsn + (int64_t)oh * p.rsh + (int64_t)ow * p.rsw;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = cols[j];
        if (col >= p.Co) continue;
        float v = acc[i][j][r] * sc[j] + bi[j];
        if (p.res_mode == PRPE_RES_PRE_ACT) v += p.r[ro + col * p.rsc];
        v = apply_act(v, p.act, sl[j]);
        if (p.res_mode == PRPE_RES_POST_ACT) v += p.r[ro + col * p.rsc];
        p.y[yo + col * p.ysc] = v;
      }
    }
  }
}

template <int BM, int BN, int WM, int WN>
int launch_cfg(const ConvK& kp0, bool vec, int prec, hipStream_t st) {
  ConvK kp = kp0;
  const int tiles_m = (kp.M + BM - 1) / BM;
  kp.tiles_n = (kp.Co + BN - 1) / BN;
  kp.nwg = tiles_m * kp.tiles_n;
  dim3 grid(kp.nwg), block(NTHREADS);
  if (vec) {
    if (prec == 0) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, true, 0>), grid, block, 0, st, kp);
    else if (prec == 1) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, true, 1>), grid, block, 0, st, kp);
    else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, true, 2>), grid, block, 0, st, kp);
  } else {
    if (prec == 0) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, false, 0>), grid, block, 0, st, kp);
    else if (prec == 1) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, false, 1>), grid, block, 0, st, kp);
    else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, false, 2>), grid, block, 0, st, kp);
  }
  return launch_status();
}

}  // namespace

extern "C" int prpe_conv2d(const prpe_conv_desc* d, void* stream) {
  if (!d || !view_ok(&d->x) || !view_ok(&d->y) || !d->w_hi) return PRPE_EINVAL;
  if (d->precision < 0 || d->precision > 2) return PRPE_EINVAL;
  if (d->precision != 1 && !d->w_lo) return PRPE_EINVAL;
  if (d->precision == 2 && !d->w_lo2) return PRPE_EINVAL;
  if (d->kh <= 0 || d->kw <= 0 || d->stride <= 0 || d->pad < 0) return PRPE_EINVAL;
  const prpe_view& x = d->x; const prpe_view& y = d->y;
  if (x.n != y.n) return PRPE_EINVAL;
  const int Ho = (x.h + 2 * d->pad - d->kh) / d->stride + 1;
  const int Wo = (x.w + 2 * d->pad - d->kw) / d->stride + 1;
  if (Ho != y.h || Wo != y.w) return PRPE_EINVAL;
  const int K = d->kh * d->kw * x.c;
  if (d->k_pad % BK || d->k_pad < K || d->co_pad % 128 || d->co_pad < y.c) return PRPE_EINVAL;
  if (d->res_mode != PRPE_RES_NONE && !d->res.ptr) return PRPE_EINVAL;
  if (d->in_scale && !d->in_bias) return PRPE_EINVAL;
  if (d->act == PRPE_ACT_PRELU && !d->slope) return PRPE_EINVAL;
  const int64_t M64 = (int64_t)x.n * Ho * Wo;
  if (M64 >= (1LL << 31)) return PRPE_EINVAL;
  // vector path: contiguous channels, Ci % 4 == 0, 16-B aligned rows
  const bool vec = x.sc == 1 && (x.c % 4) == 0 && (x.sw % 4) == 0 && (x.sh % 4) == 0 &&
                   (x.sn % 4) == 0 && ((uintptr_t)x.ptr % 16) == 0;
  if (!vec && d->k_pad > 1024) return PRPE_EINVAL;

  ConvK kp{};
  kp.x = x.ptr; kp.xsn = x.sn; kp.xsh = x.sh; kp.xsw = x.sw; kp.xsc = x.sc;
  kp.Hi = x.h; kp.Wi = x.w; kp.Ci = x.c;
  kp.y = y.ptr; kp.ysn = y.sn; kp.ysh = y.sh; kp.ysw = y.sw; kp.ysc = y.sc;
  kp.Ho = Ho; kp.Wo = Wo; kp.Co = y.c;
  kp.r = d->res.ptr; kp.rsn = d->res.sn; kp.rsh = d->res.sh; kp.rsw = d->res.sw; kp.rsc = d->res.sc;
  kp.KH = d->kh; kp.KW = d->kw; kp.stride = d->stride; kp.pad = d->pad;
  kp.K = K; kp.k_pad = d->k_pad; kp.nk = (K + BK - 1) / BK;
  kp.whi = d->w_hi; kp.wlo = d->w_lo; kp.wlo2 = d->w_lo2;
  kp.scale = d->scale; kp.bias = d->bias; kp.slope = d->slope;
  kp.in_scale = d->in_scale; kp.in_bias = d->in_bias;
  kp.act = d->act; kp.res_mode = d->res_mode;
  kp.M = (int)M64; kp.HoWo = Ho * Wo;
  hipStream_t st = as_stream(stream);
  const int prec = d->precision;
  int tile = d->tile;
  if (tile == 0) tile = y.c > 64 ? 1 : y.c > 32 ? 2 : y.c > 16 ? 3 : 4;
  switch (tile) {
    case 1: return launch_cfg<128, 128, 2, 2>(kp, vec, prec, st);
    case 2: return launch_cfg<128, 64, 2, 2>(kp, vec, prec, st);
    case 3: return launch_cfg<128, 32, 4, 1>(kp, vec, prec, st);
    case 4: return launch_cfg<128, 16, 4, 1>(kp, vec, prec, st);
    default: return PRPE_EINVAL;
  }
}
