// Implicit-GEMM convolution on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), split-bf16 operands.
//
// GEMM view: M = N*Ho*Wo output pixels, N_gemm = Co, K = KH*KW*Ci.
//   A[m,k] = PRO(x[n, oh*s-p+kh, ow*s-p+kw, ci])   (gathered on the fly, strided view)
//   B[k,co] = W[co, kh, kw, ci]                    (host-packed bf16 planes [co][k])
// K order (``k_order``): 0 = tap-major k = (kh*KW+kw)*Ci + ci; 1 = chunk-major
// k = ((ci/32)*KH*KW + kh*KW+kw)*32 + ci%32 (Ci % 32 == 0): the KH*KW taps of one 32-channel
// chunk are consecutive K-steps, so the overlapping input windows they gather are re-read
// from L1 instead of L2.
// Each fp32 operand is split into NP bf16 planes a = a0 + a1 (+ a2) and the wave issues the
// partial products with plane-index sum < NP, smallest first, fp32 accumulate:
//   precision 0 (NP=2): a1*b0 + a0*b1 + a0*b0            ~16-bit operands, 2^-17 rel/product,
//                        1/3 of the dense bf16 MFMA rate (~830 TF/s ceiling)
//   precision 2 (NP=3): a2*b0 + a1*b1 + a0*b2 + a1*b0 + a0*b1 + a0*b0
//                        the 3-way split is exact for fp32 operands: fp32-faithful products
//                        at 1/6 of the bf16 rate (~415 TF/s ceiling vs 157 for f32 MFMA)
//   precision 1 (NP=1): a0*b0 plain bf16 (diagnostics / ablation only)
//
// Tiling: BM x BN x 32, NT = 64*WM*WN threads, each wave a (BM/WM)x(BN/WN) tile of 16x16 MFMA
// blocks. Global->register prefetch of tile k+1 overlaps the MFMAs of tile k (A is split into
// planes in registers, then written to LDS); LDS double buffer, one barrier per K-step. LDS
// rows are 64 B (32 bf16); the 4 16-B slots of row r are XOR-permuted by F[(r>>2)&3] =
// {0,2,3,1}, which makes every ds_read_b128 lane group of the fragment read hit 16 distinct
// slots. Epilogue: the accumulator tile is staged through the (then free) LDS ring and written
// as whole-row 16-B vectors with coalesced residual loads. Grid: 1-D, XCD-remapped so the
// Co-tiles sharing one A panel run on one XCD (shared L2).
//
// Reference arithmetic replaced: torch Conv2d (+BatchNorm2d eval +act +residual) at every
// call site listed in include/prpe.h (prpe_conv2d).
#include "conv.h"
#include <stdlib.h>

namespace {

constexpr int BK = 32;

// 32 zero bytes: the gather source of out-of-bounds taps (padding), so a loaded value never
// needs a select afterwards (conv_wave reads 32 B per lane and row)
__device__ __attribute__((aligned(32))) float g_zero8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

using namespace prpe_k;

// KM: 0 = scalar gather through a k -> (kh,kw,ci) LUT (any Ci, e.g. 3-channel inputs)
//     1 = vector loads, tap-major K (Ci % 4 == 0)
//     2 = vector loads, chunk-major K (Ci % 32 == 0, weights packed with k_order 1)
// PRO: input-side affine (IR-50 pre-BN) compiled in; vector paths only.
// VALU budget (the MFMAs of a K-step are 48 / 96 per wave at 2 / 3 planes): the per-row gather
// costs a bit test, a select and one 64-bit add -- row bases and the tap validity of every row
// (one bit per kh and per kw) are computed once, the K-step offset is wave-uniform (KM 2) or
// advanced incrementally (KM 1).
template <int BM, int BN, int WM, int WN, int KM, int PREC, bool PRO>
__global__ __launch_bounds__(64 * WM * WN, 2) void conv_igemm_kernel(ConvK p) {
  constexpr int NT = 64 * WM * WN;
  constexpr bool VEC = KM != 0;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int RPASS = NT / 8;                      // VEC: rows per pass (8 float4 per row)
  constexpr int A_ROWS_PT = BM / RPASS;
  constexpr int B_CHUNKS = BN * 4;                   // 16-B chunks per plane per K-step
  constexpr int B_PT = (B_CHUNKS + NT - 1) / NT;
  constexpr int NP = PREC == 1 ? 1 : (PREC == 0 ? 2 : 3);   // bf16 planes per operand
  static_assert(TM >= 1 && TN >= 1 && A_ROWS_PT >= 1, "tile");
  static_assert(KM != 0 || (NT % BM == 0), "scalar path: NT multiple of BM");

  // staging ring: [buf][plane][A rows | B rows][32] bf16; re-used for the epilogue's C tile
  constexpr int LDS_U16 = 2 * NP * (BM + BN) * BK;
  constexpr int CS = BN + 4;                          // C-tile row pitch (floats)
  constexpr int CH_FIT = (LDS_U16 * 2) / (CS * 4);
  constexpr int CH = CH_FIT >= BM ? BM : (CH_FIT / 16) * 16;   // C rows staged per round
  static_assert(CH >= 16, "epilogue staging");
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_U16];
  __shared__ int klut[KM == 0 ? 1024 : 1];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int L = xcd_remap(blockIdx.x, p.nwg);
  const int tile_m = L / p.tiles_n, tile_n = L % p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  auto A_at = [&](int buf, int plane) -> uint16_t* { return lds + ((buf * NP + plane) * (BM + BN)) * BK; };
  auto B_at = [&](int buf, int plane) -> uint16_t* { return lds + ((buf * NP + plane) * (BM + BN) + BM) * BK; };

  // ---------------- A-load state
  constexpr int S_KPT = (BM * BK) / NT;               // scalar: k elements per thread per step
  int64_t rowoff[VEC ? A_ROWS_PT : 1];
  int ih0[VEC ? A_ROWS_PT : 1], iw0[VEC ? A_ROWS_PT : 1];
  int64_t rbase[VEC ? A_ROWS_PT : 1];                 // element offset of tap (0,0), may be < 0
  unsigned hmask[VEC ? A_ROWS_PT : 1], wmask[VEC ? A_ROWS_PT : 1];   // in-bounds kh / kw bits

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
    for (int i = 0; i < A_ROWS_PT; ++i) {
      decode_row(m0 + (tid >> 3) + RPASS * i, rowoff[i], ih0[i], iw0[i]);
      rbase[i] = rowoff[i] + (int64_t)ih0[i] * p.xsh + (int64_t)iw0[i] * p.xsw;
      unsigned hm = 0, wmk = 0;
      for (int t = 0; t < p.KH; ++t) hm |= (unsigned)((unsigned)(ih0[i] + t) < (unsigned)p.Hi) << t;
      for (int t = 0; t < p.KW; ++t) wmk |= (unsigned)((unsigned)(iw0[i] + t) < (unsigned)p.Wi) << t;
      hmask[i] = hm;
      wmask[i] = wmk;
    }
  } else {
    decode_row(m0 + (tid % BM), rowoff[0], ih0[0], iw0[0]);
    // k -> packed (dh, dw, ci) table for this layer (k_pad <= 1024 checked on host)
    for (int k = tid; k < p.k_pad; k += NT) {
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

  // KM 1: incremental (kh, kw, ci) of this thread's chunk and its element offset
  int c_ci = (tid & 7) * 4, c_kh = 0, c_kw = 0;
  int64_t c_off = 0;
  auto c_advance = [&]() {   // carry c_ci >= Ci into kw / kh
    while (c_ci >= p.Ci && c_kh < p.KH) {
      c_ci -= p.Ci;
      c_off += p.xsw - p.Ci;
      if (++c_kw == p.KW) { c_kw = 0; ++c_kh; c_off += p.xsh - (int64_t)p.KW * p.xsw; }
    }
  };
  if constexpr (KM == 1) {
    c_off = c_ci;
    c_advance();
  }
  // KM 2: wave-uniform (chunk, kh, kw) of the next K-step to load
  int u_kh = 0, u_kw = 0, u_ci = 0;                   // u_ci = chunk*32
  int64_t u_off = 0;                                  // kh*xsh + kw*xsw + chunk*32
  const int cthr = (tid & 7) * 4;

  f4 areg[VEC ? A_ROWS_PT : 1];
  float sreg[VEC ? 1 : S_KPT];
  unsigned amask = 0;                                // in-bounds bits of areg / sreg
  f4 as4 = {1.f, 1.f, 1.f, 1.f}, ab4 = {0.f, 0.f, 0.f, 0.f};   // prologue affine of this K-step
  static_assert(A_ROWS_PT <= 32 && S_KPT <= 32, "amask");
  u4 breg[NP][B_PT];

  auto load_tile = [&](int kt) {
    if constexpr (VEC) {
      int kh, kw;
      int64_t off;
      bool kval;
      if constexpr (KM == 2) {
        kh = u_kh; kw = u_kw; off = u_off + cthr;
        kval = true;
        if constexpr (PRO) {
          as4 = *reinterpret_cast<const f4*>(p.in_scale + u_ci + cthr);
          ab4 = *reinterpret_cast<const f4*>(p.in_bias + u_ci + cthr);
        }
        // next K-step: kw, then kh, then the next 32-channel chunk
        u_off += p.xsw;
        if (++u_kw == p.KW) {
          u_kw = 0; u_off += p.xsh - (int64_t)p.KW * p.xsw;
          if (++u_kh == p.KH) { u_kh = 0; u_ci += BK; u_off += BK - (int64_t)p.KH * p.xsh; }
        }
      } else {
        kh = c_kh; kw = c_kw; off = c_off;
        kval = c_kh < p.KH;
        if constexpr (PRO) {
          const int cs = kval ? c_ci : 0;
          as4 = *reinterpret_cast<const f4*>(p.in_scale + cs);
          ab4 = *reinterpret_cast<const f4*>(p.in_bias + cs);
        }
        c_ci += BK;
        c_off += BK;
        c_advance();
      }
      // Branch-free gather: out-of-bounds taps read 16 zero bytes (PRO: their affine result is
      // zeroed in store_tile through amask). Nothing here consumes a loaded value, so the
      // loads stay in flight across compute().
      amask = 0;
#pragma unroll
      for (int i = 0; i < A_ROWS_PT; ++i) {
        const bool ok = kval && ((hmask[i] >> kh) & (wmask[i] >> kw) & 1u);
        const float* src = ok ? p.x + (rbase[i] + off) : p.zero;
        areg[i] = *reinterpret_cast<const f4*>(src);
        if constexpr (PRO) amask |= (unsigned)ok << i;
      }
    } else {
      const int kk0 = tid / BM;
      constexpr int KSTEP = NT / BM;
      amask = 0;
#pragma unroll
      for (int j = 0; j < S_KPT; ++j) {
        const int k = kt * BK + kk0 + KSTEP * j;
        const int e = klut[k];
        const int dh = e >> 24, dw = (e >> 16) & 0xFF, ci = e & 0xFFFF;
        const int ih = ih0[0] + dh, iw = iw0[0] + dw;
        const bool ok = e >= 0 && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi;
        sreg[j] = *(ok ? p.x + rowoff[0] + ih * p.xsh + iw * p.xsw + ci * p.xsc : p.x);
        amask |= (unsigned)ok << j;
      }
    }
    // B: packed planes [co_pad][k_pad] bf16
#pragma unroll
    for (int j = 0; j < B_PT; ++j) {
      const int c = tid + NT * j;
      if (B_CHUNKS % NT == 0 || c < B_CHUNKS) {
        const int row = c >> 2, ch = c & 3;
        const int64_t off = (int64_t)(n0 + row) * p.k_pad + kt * BK + ch * 8;
        breg[0][j] = *reinterpret_cast<const u4*>(p.whi + off);
        if constexpr (NP > 1) breg[1][j] = *reinterpret_cast<const u4*>(p.wlo + off);
        if constexpr (NP > 2) breg[NP - 1][j] = *reinterpret_cast<const u4*>(p.wlo2 + off);
      }
    }
  };

  // The staging writes of the next tile are split into pieces (one A row each, then B) that
  // compute() interleaves with its MFMA rows, so the split/convert VALU work and the LDS
  // writes issue under the MFMAs instead of after them.
  constexpr int NPIECE = VEC ? A_ROWS_PT + 1 : 1;
  auto store_piece = [&](int buf, int piece) {
    if constexpr (VEC) {
      const int c4 = tid & 7;
      if (piece < A_ROWS_PT) {
        const int i = piece;
        const int row = (tid >> 3) + RPASS * i;
        const int slot = (c4 >> 1) ^ swzF(row);
        const int off = row * BK + slot * 8 + (c4 & 1) * 4;
        bf16x4 pl[NP];
        f4 v = areg[i];
        if constexpr (PRO) {
          v = v * as4 + ab4;
          if (!((amask >> i) & 1u)) v = f4{0.f, 0.f, 0.f, 0.f};   // padding stays 0 (no prologue)
        }
        split_planes<NP>(v, pl);
#pragma unroll
        for (int q = 0; q < NP; ++q) *reinterpret_cast<bf16x4*>(A_at(buf, q) + off) = pl[q];
        return;
      }
    } else {
      const int row = tid % BM, kk0 = tid / BM;
      constexpr int KSTEP = NT / BM;
#pragma unroll
      for (int j = 0; j < S_KPT; ++j) {
        const int kk = kk0 + KSTEP * j;
        const int slot = (kk >> 3) ^ swzF(row);
        const int off = row * BK + slot * 8 + (kk & 7);
        float r = ((amask >> j) & 1u) ? sreg[j] : 0.f;
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
      const int c = tid + NT * j;
      if (B_CHUNKS % NT == 0 || c < B_CHUNKS) {
        const int row = c >> 2, ch = c & 3;
        const int off = row * BK + (ch ^ swzF(row)) * 8;
#pragma unroll
        for (int q = 0; q < NP; ++q) *reinterpret_cast<u4*>(B_at(buf, q) + off) = breg[q][j];
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int pc = 0; pc < NPIECE; ++pc) store_piece(buf, pc);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;

  auto compute = [&](int buf, int nbuf, bool stage) {
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
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int s = NP - 1; s >= 0; --s)
#pragma unroll
          for (int qa = s; qa >= 0; --qa)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[qa][i], bfr[s - qa][j], acc[i][j], 0, 0, 0);
      }
      // pieces go behind the second half of the MFMA rows: the global loads they consume
      // were issued at the top of this K-step and need that long to land
      constexpr int H0 = TM / 2, NR = TM - H0;
      if (stage && i >= H0) {
#pragma unroll
        for (int pc = (i - H0) * NPIECE / NR; pc < (i - H0 + 1) * NPIECE / NR; ++pc) store_piece(nbuf, pc);
      }
    }
  };

  // ---------------- main loop
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < p.nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < p.nk;
    if (more) load_tile(kt + 1);
    compute(cur, cur ^ 1, more);
    __syncthreads();
  }

  // ---------------- epilogue
  FrameMax ymax;                                      // per-frame running max|y| (p.y_amax)
  if (p.vec_out) {
    // Stage the raw accumulator tile through LDS (CH rows per round), then every thread owns
    // 16-B column chunks of whole rows: coalesced float4 residual loads and output stores.
    float* ct = reinterpret_cast<float*>(lds);
    constexpr int CPR = BN / 4;                     // float4 chunks per tile row
    constexpr int RPP = NT / CPR;                   // rows per pass
    const int cc = tid % CPR;
    const int col = n0 + cc * 4;
    f4 sc4 = {1.f, 1.f, 1.f, 1.f}, bi4 = {0.f, 0.f, 0.f, 0.f}, sl4 = {0.f, 0.f, 0.f, 0.f};
    if (col < p.Co) {
      if (p.scale) sc4 = *reinterpret_cast<const f4*>(p.scale + col);
      if (p.bias) bi4 = *reinterpret_cast<const f4*>(p.bias + col);
      if (p.slope) sl4 = *reinterpret_cast<const f4*>(p.slope + col);
    }
    for (int h0 = 0; h0 < BM; h0 += CH) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * WTM + i * 16 + fg * 4 + r - h0;
          if (row >= 0 && row < CH)
#pragma unroll
            for (int j = 0; j < TN; ++j) ct[row * CS + wn * WTN + j * 16 + fr] = acc[i][j][r];
        }
      __syncthreads();
      if (col < p.Co) {
        const int rows = BM - h0 < CH ? BM - h0 : CH;
        // EB rows per batch: all residual loads of a batch are issued before the first store
        // (y and r are distinct buffers, but the compiler cannot know that and would otherwise
        // serialise load -> store -> load on every row)
        constexpr int EB = 4;
        for (int rb = tid / CPR; rb < rows; rb += RPP * EB) {
          int64_t yo[EB];
          f4 res[EB];
          bool ok[EB];
          int fn[EB];
#pragma unroll
          for (int e = 0; e < EB; ++e) {
            const int rr = rb + RPP * e;
            const int m = m0 + h0 + rr;
            ok[e] = rr < rows && m < p.M;
            res[e] = f4{0.f, 0.f, 0.f, 0.f};
            yo[e] = 0;
            fn[e] = 0;
            if (ok[e]) {
              const int n = m / p.HoWo;
              fn[e] = n;
              const int rem = m - n * p.HoWo;
              const int oh = rem / p.Wo;
              const int ow = rem - oh * p.Wo;
              yo[e] = (int64_t)n * p.ysn + (int64_t)oh * p.ysh + (int64_t)ow * p.ysw + col;
              if (p.res_mode != PRPE_RES_NONE)
                res[e] = *reinterpret_cast<const f4*>(p.r + (int64_t)n * p.rsn + (int64_t)oh * p.rsh +
                                                      (int64_t)ow * p.rsw + col);
            }
          }
#pragma unroll
          for (int e = 0; e < EB; ++e) {
            if (!ok[e]) continue;
            f4 v = *reinterpret_cast<const f4*>(ct + (rb + RPP * e) * CS + cc * 4);
            v = v * sc4 + bi4;
            if (p.res_mode == PRPE_RES_PRE_ACT) v += res[e];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = apply_act(v[q], p.act, sl4[q]);
            if (p.res_mode == PRPE_RES_POST_ACT) v += res[e];
            *reinterpret_cast<f4*>(p.y + yo[e]) = v;
            if (p.y_amax) ymax.add(p.y_amax, fn[e], amax4(v));
          }
        }
      }
      if (h0 + CH < BM) __syncthreads();
    }
    if (p.y_amax) frame_amax_final(p.y_amax, ymax);
    return;
  }
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
        if (p.y_amax) ymax.add(p.y_amax, n, fabsf(v));
      }
    }
  }
  if (p.y_amax) frame_amax_final(p.y_amax, ymax);
}

// Direct fp32 conv for Co <= 4 (ViT adapter 128->3, YOLO adapter 64->3, head 80->1): a 16-wide
// MFMA tile would waste >= 75 % of its columns and the layer is bound by reading its input.
// Lanes run across input channels: a pixel is handled by LPP = pow2 >= Ci/4 lanes, each lane
// owning 4 channels (one coalesced float4 per tap) and holding its slice of the weights for
// all taps in registers (KHW*4*CO floats, rebuilt exactly as p0+p1+p2). Per pixel the LPP
// partial dot products are combined with a shuffle tree; grid-stride over pixels.
template <int CO, int KHW>
__global__ __launch_bounds__(256) void conv_smallco_kernel(ConvK p, int lpp_log2) {
  const int LPP = 1 << lpp_log2;
  const int lane = threadIdx.x & 63;
  const int c4 = lane & (LPP - 1);
  const int slot = lane >> lpp_log2;
  const int ppw = 64 >> lpp_log2;
  const bool cval = c4 * 4 < p.Ci;
  float w[KHW][4][CO];
#pragma unroll
  for (int t = 0; t < KHW; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int c = 0; c < CO; ++c) {
        float v = 0.f;
        if (cval) {
          const int64_t o = (int64_t)c * p.k_pad + t * p.Ci + c4 * 4 + e;
          v = (float)__builtin_bit_cast(__bf16, p.whi[o]) + (float)__builtin_bit_cast(__bf16, p.wlo[o]) +
              (float)__builtin_bit_cast(__bf16, p.wlo2[o]);
        }
        w[t][e][c] = v;
      }
  FrameMax ymax;
  const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int nw = (int)((gridDim.x * blockDim.x) >> 6);
  for (int base = gw * ppw; base < p.M; base += nw * ppw) {
    const int m = base + slot;
    float acc[CO];
#pragma unroll
    for (int c = 0; c < CO; ++c) acc[c] = 0.f;
    int n = 0, oh = 0, ow = 0;
    if (m < p.M) {
      n = m / p.HoWo;
      const int rem = m - n * p.HoWo;
      oh = rem / p.Wo;
      ow = rem - oh * p.Wo;
      const float* xb = p.x + (int64_t)n * p.xsn + c4 * 4;
#pragma unroll
      for (int t = 0; t < KHW; ++t) {
        const int kh = KHW == 1 ? 0 : t / 3, kw = KHW == 1 ? 0 : t % 3;
        const int ih = oh * p.stride - p.pad + kh, iw = ow * p.stride - p.pad + kw;
        if (cval && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi) {
          const f4 v = *reinterpret_cast<const f4*>(xb + (int64_t)ih * p.xsh + (int64_t)iw * p.xsw);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int c = 0; c < CO; ++c) acc[c] = fmaf(v[e], w[t][e][c], acc[c]);
        }
      }
    }
    for (int o = LPP >> 1; o > 0; o >>= 1)
#pragma unroll
      for (int c = 0; c < CO; ++c) acc[c] += __shfl_xor(acc[c], o, 64);
    if (c4 == 0 && m < p.M) {
      const int64_t yo = (int64_t)n * p.ysn + (int64_t)oh * p.ysh + (int64_t)ow * p.ysw;
      const int64_t ro = (int64_t)n * p.rsn + (int64_t)oh * p.rsh + (int64_t)ow * p.rsw;
#pragma unroll
      for (int c = 0; c < CO; ++c) {
        if (c >= p.Co) break;
        float v = acc[c] * (p.scale ? p.scale[c] : 1.f) + (p.bias ? p.bias[c] : 0.f);
        if (p.res_mode == PRPE_RES_PRE_ACT) v += p.r[ro + c * p.rsc];
        v = apply_act(v, p.act, p.slope ? p.slope[c] : 0.f);
        if (p.res_mode == PRPE_RES_POST_ACT) v += p.r[ro + c * p.rsc];
        p.y[yo + c * p.ysc] = v;
        if (p.y_amax) ymax.add(p.y_amax, n, fabsf(v));
      }
    }
  }
  if (p.y_amax) frame_amax_final(p.y_amax, ymax);
}

template <int BM, int BN, int WM, int WN, int KM, bool PRO>
int launch_km(const ConvK& kp, int prec, dim3 grid, hipStream_t st) {
  constexpr int NT = 64 * WM * WN;
  if (prec == 0) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, KM, 0, PRO>), grid, dim3(NT), 0, st, kp);
  else if (prec == 1) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, KM, 1, PRO>), grid, dim3(NT), 0, st, kp);
  else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, KM, 2, PRO>), grid, dim3(NT), 0, st, kp);
  return launch_status();
}

template <int BM, int BN, int WM, int WN>
int launch_cfg(const ConvK& kp0, int km, int prec, hipStream_t st) {
  ConvK kp = kp0;
  const int tiles_m = (kp.M + BM - 1) / BM;
  kp.tiles_n = (kp.Co + BN - 1) / BN;
  kp.nwg = tiles_m * kp.tiles_n;
  dim3 grid(kp.nwg);
  const bool pro = kp.in_scale != nullptr;
  if (km == 2) return pro ? launch_km<BM, BN, WM, WN, 2, true>(kp, prec, grid, st)
                          : launch_km<BM, BN, WM, WN, 2, false>(kp, prec, grid, st);
  if (km == 1) return pro ? launch_km<BM, BN, WM, WN, 1, true>(kp, prec, grid, st)
                          : launch_km<BM, BN, WM, WN, 1, false>(kp, prec, grid, st);
  if constexpr ((64 * WM * WN) % BM == 0) return launch_km<BM, BN, WM, WN, 0, false>(kp, prec, grid, st);
  return PRPE_EINVAL;
}

}  // namespace

// Validate a descriptor and fill the kernel arguments (shared by prpe_conv2d and
// prpe_conv2d_workspace_bytes). Returns 0 or PRPE_EINVAL; km = the K walk (0 scalar, 1 vector,
// 2 chunk-major).
static int conv_setup(const prpe_conv_desc* d, ConvK& kp, int& km) {
  if (!d || !view_ok(&d->x) || !view_ok(&d->y) || !d->w_hi) return PRPE_EINVAL;
  if (d->precision < 0 || d->precision > 4) return PRPE_EINVAL;
  if ((d->precision == 0 || d->precision == 2) && !d->w_lo) return PRPE_EINVAL;
  if (d->precision == 2 && !d->w_lo2) return PRPE_EINVAL;
  if (d->precision == 3 && (!d->w_h16 || !d->w_l16 || !d->scale16 || !d->x_amax || d->in_scale))
    return PRPE_EINVAL;
  // precision 4: one fp16 plane (w_h16) and the input's per-frame max bound; a prologue affine is
  // allowed (its output is bounded in-kernel); no dual input, no planes format
  if (d->precision == 4 && (!d->w_h16 || !d->scale16 || !d->x_amax || d->x2.ptr || d->x_planes || d->y_planes))
    return PRPE_EINVAL;
  if (d->kh <= 0 || d->kw <= 0 || d->stride <= 0 || d->pad < 0) return PRPE_EINVAL;
  const prpe_view& x = d->x; const prpe_view& y = d->y;
  if (x.n != y.n) return PRPE_EINVAL;
  const int Ho = (x.h + 2 * d->pad - d->kh) / d->stride + 1;
  const int Wo = (x.w + 2 * d->pad - d->kw) / d->stride + 1;
  if (Ho != y.h || Wo != y.w) return PRPE_EINVAL;
  // dual input (x2): 1x1, unpadded, both inputs channel-chunked, K = Ci + C2 in that order
  const bool dual = d->x2.ptr != nullptr;
  if (dual) {
    const prpe_view& v = d->x2;
    if (!view_ok(&v) || d->kh != 1 || d->kw != 1 || d->pad != 0 || v.n != y.n || v.h != Ho || v.w != Wo ||
        v.sc != 1 || v.c % 32 || x.c % 32 || v.sw % 4 || v.sh % 4 || v.sn % 4 || (uintptr_t)v.ptr % 16 ||
        d->in_scale || d->precision == 1 || (d->precision == 3 && !d->x2_amax))
      return PRPE_EINVAL;
    if (d->tile != 0 && d->tile < 20) return PRPE_EINVAL;
  }
  const int K = d->kh * d->kw * x.c + (dual ? d->x2.c : 0);
  if (d->k_pad % BK || d->k_pad < K || d->co_pad % 128 || d->co_pad < y.c) return PRPE_EINVAL;
  if (d->res_mode != PRPE_RES_NONE && !d->res.ptr) return PRPE_EINVAL;
  if (d->in_scale && !d->in_bias) return PRPE_EINVAL;
  if (d->act == PRPE_ACT_PRELU && !d->slope) return PRPE_EINVAL;
  if (d->k_order != 0 && d->k_order != 1) return PRPE_EINVAL;
  const int64_t M64 = (int64_t)x.n * Ho * Wo;
  if (M64 >= (1LL << 31)) return PRPE_EINVAL;
  // vector path: contiguous channels, Ci % 4 == 0, 16-B aligned rows
  const bool vec = x.sc == 1 && (x.c % 4) == 0 && (x.sw % 4) == 0 && (x.sh % 4) == 0 &&
                   (x.sn % 4) == 0 && ((uintptr_t)x.ptr % 16) == 0;
  // chunk-major K needs the vector path and whole 32-channel chunks
  if (d->k_order == 1 && (!vec || x.c % 32 != 0)) return PRPE_EINVAL;
  km = d->k_order == 1 ? 2 : (vec ? 1 : 0);
  if (km == 0 && d->k_pad > 1024) return PRPE_EINVAL;
  // the input-side affine is implemented on the vector paths only (IR-50 pre-BN, Ci >= 64);
  // the vector paths keep one validity bit per kh and per kw
  if (km == 0 && d->in_scale) return PRPE_EINVAL;
  if (km != 0 && (d->kh > 32 || d->kw > 32)) return PRPE_EINVAL;

  kp = ConvK{};
  kp.x = x.ptr; kp.xsn = x.sn; kp.xsh = x.sh; kp.xsw = x.sw; kp.xsc = x.sc;
  kp.Hi = x.h; kp.Wi = x.w; kp.Ci = x.c;
  kp.y = y.ptr; kp.ysn = y.sn; kp.ysh = y.sh; kp.ysw = y.sw; kp.ysc = y.sc;
  kp.Ho = Ho; kp.Wo = Wo; kp.Co = y.c;
  kp.r = d->res.ptr; kp.rsn = d->res.sn; kp.rsh = d->res.sh; kp.rsw = d->res.sw; kp.rsc = d->res.sc;
  kp.KH = d->kh; kp.KW = d->kw; kp.stride = d->stride; kp.pad = d->pad;
  kp.K = K; kp.k_pad = d->k_pad; kp.nk = (K + BK - 1) / BK;
  if (dual) {
    kp.x2 = d->x2.ptr; kp.x2sn = d->x2.sn; kp.x2sh = d->x2.sh; kp.x2sw = d->x2.sw;
    kp.nk1 = x.c / BK; kp.x2_amax = d->x2_amax;
  }
  kp.whi = d->w_hi; kp.wlo = d->w_lo; kp.wlo2 = d->w_lo2;
  kp.scale = d->scale; kp.bias = d->bias; kp.slope = d->slope;
  kp.in_scale = d->in_scale; kp.in_bias = d->in_bias;
  kp.act = d->act; kp.res_mode = d->res_mode;
  kp.M = (int)M64; kp.HoWo = Ho * Wo;
  auto a16 = [](const prpe_view& v) {
    return v.sc == 1 && v.c % 4 == 0 && v.sw % 4 == 0 && v.sh % 4 == 0 && v.sn % 4 == 0 &&
           ((uintptr_t)v.ptr % 16) == 0;
  };
  kp.vec_out = a16(y) && (d->res_mode == PRPE_RES_NONE || a16(d->res)) &&
               (!d->scale || (uintptr_t)d->scale % 16 == 0) && (!d->bias || (uintptr_t)d->bias % 16 == 0) &&
               (!d->slope || (uintptr_t)d->slope % 16 == 0);
  kp.wh16 = d->w_h16; kp.wl16 = d->w_l16; kp.x_amax = d->x_amax; kp.y_amax = d->y_amax;
  // planes format (see prpe.h): the wave-row kernel reads / writes it, two bf16 planes only
  kp.x_planes = d->x_planes; kp.y_planes = d->y_planes;
  if (d->x_planes && (d->precision != 0 || x.sc != 1 || x.c % 32 || d->in_scale || dual)) return PRPE_EINVAL;
  if (d->y_planes && (y.sc != 1 || y.c % 8 || y.sw % 8 || y.sh % 8 || y.sn % 8 || (uintptr_t)y.ptr % 32 ||
                      d->precision == 1))
    return PRPE_EINVAL;
  if (d->precision >= 3) kp.scale = d->scale16;
  // epilogue 1x1 GEMM (haloed-tile 3x3 kernel only)
  if (d->w2 && d->tile != 0 && (d->tile < 30 || d->tile >= 40)) return PRPE_EINVAL;
  if (d->w2) {
    const prpe_view& v2 = d->y2;
    if (!view_ok(&v2) || v2.n != y.n || v2.h != Ho || v2.w != Wo || v2.c > 32 || v2.sc != 1 || y.c > 128 ||
        d->y_planes || d->res_mode != PRPE_RES_NONE || d->y_amax || (uintptr_t)d->w2 % 16 || y.c % 4)
      return PRPE_EINVAL;
    kp.w2 = d->w2; kp.y2 = v2.ptr; kp.y2sn = v2.sn; kp.y2sh = v2.sh; kp.y2sw = v2.sw; kp.n2 = v2.c;
    if (d->w3) {
      if (d->n2 <= 0 || d->n2 > 64 || d->n2 % 4 || (uintptr_t)d->w3 % 16 || d->act2 < 0 || d->act2 > PRPE_ACT_SIGMOID ||
          d->act2 == PRPE_ACT_PRELU)
        return PRPE_EINVAL;
      kp.w3 = d->w3; kp.s2 = d->scale2; kp.b2 = d->bias2; kp.act2 = d->act2; kp.nmid = d->n2;
    }
  } else if (d->w3) {
    return PRPE_EINVAL;
  }
  kp.ylin = y.sh == (int64_t)Wo * y.sw && y.sn == (int64_t)Ho * y.sh;
  kp.rlin = d->res_mode == PRPE_RES_NONE ||
            (d->res.sh == (int64_t)Wo * d->res.sw && d->res.sn == (int64_t)Ho * d->res.sh);
  return 0;
}

// per-device address of the zero page (one host query per device, then cached)
static const float* zero_page() {
  static const float* zero_by_dev[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!zero_by_dev[dev]) {
    void* zp = nullptr;
    if (hipGetSymbolAddress(&zp, HIP_SYMBOL(g_zero8)) != hipSuccess || !zp) return nullptr;
    zero_by_dev[dev] = static_cast<const float*>(zp);
  }
  return zero_by_dev[dev];
}

// full-window linears with few M x N tiles (the IR-50 output layer): split along K
// (conv_splitk.hip) automatically; tile 50 forces it
static bool conv_use_splitk(const prpe_conv_desc* d, const ConvK& kp) {
  if (d->tile == 50) return true;
  return d->tile == 0 && kp.K >= 4096 && (int64_t)((kp.M + 63) / 64) * (kp.Co / 64) < 256 &&
         conv_splitk_eligible(kp, d->precision, d->k_order);
}

extern "C" int64_t prpe_conv2d_workspace_bytes(const prpe_conv_desc* d) {
  ConvK kp;
  int km = 0;
  if (conv_setup(d, kp, km) != 0) return PRPE_EINVAL;
  if (!conv_use_splitk(d, kp) || !conv_splitk_eligible(kp, d->precision, d->k_order)) return 0;
  return conv_splitk_workspace_bytes(kp);
}

extern "C" int prpe_conv2d(const prpe_conv_desc* d, void* stream) {
  ConvK kp;
  int km = 0;
  if (int rc = conv_setup(d, kp, km)) return rc;
  kp.zero = zero_page();
  if (!kp.zero) return PRPE_EINVAL;
  const prpe_view& x = d->x; const prpe_view& y = d->y;
  const bool dual = d->x2.ptr != nullptr;
  hipStream_t st = as_stream(stream);
  const int prec = d->precision;
  int tile = d->tile;
  // direct fp32 kernel for tiny Co (needs the 3 weight planes; exact fp32 products); 1x1 only:
  // for 3x3 Co=3 the MFMA path measured faster (7.5 ms vs 11.8 ms at bs=256)
  const int khw = d->kh * d->kw;
  // split-K: partial sums in the caller's workspace (prpe_conv2d_workspace_bytes)
  if (conv_use_splitk(d, kp)) {
    if (!conv_splitk_eligible(kp, prec, d->k_order)) return PRPE_EINVAL;
    const int64_t need = conv_splitk_workspace_bytes(kp);
    if (!d->workspace || d->workspace_bytes < need || (uintptr_t)d->workspace % 256) return PRPE_EINVAL;
    return conv_splitk_launch(kp, static_cast<float*>(d->workspace), st);
  }
  // epilogue 1x1 GEMM: the haloed-tile kernel's 128-column tile is the only implementation
  if (kp.w2) return conv_halo_eligible(kp, prec, km) ? conv_halo_launch(kp, prec, tile ? tile : 30, st) : PRPE_EINVAL;
  if (tile == 0 && y.c <= 4 && km == 1 && !d->in_scale && d->w_lo && d->w_lo2 && x.c <= 256 && khw == 1) {
    int lg = 0;
    while ((1 << lg) * 4 < x.c) ++lg;
    const int ppb = 4 * (64 >> lg);                      // pixels per block-iteration
    int blocks = (kp.M + ppb - 1) / ppb;
    if (blocks > 256 * 16) blocks = 256 * 16;
    if (y.c == 1) hipLaunchKernelGGL((conv_smallco_kernel<1, 1>), dim3(blocks), dim3(256), 0, st, kp, lg);
    else if (y.c <= 3) hipLaunchKernelGGL((conv_smallco_kernel<3, 1>), dim3(blocks), dim3(256), 0, st, kp, lg);
    else hipLaunchKernelGGL((conv_smallco_kernel<4, 1>), dim3(blocks), dim3(256), 0, st, kp, lg);
    return launch_status();
  }
  // direct global->LDS kernel (conv_glds.hip) for chunked inputs with Co > 32: tiles 10..12 only
  // (never the automatic choice since round 1: this file's 256x64 tile measures 27 % faster on
  // its shapes in isolation, profiles/r01_conv_bench_sweep_v4.txt, and -0.6..1.0 ms per
  // sequential forward; the round-1 environment switch back to it was removed in round 6)
  static const int wave_on = [] {
    const char* e = getenv("PRPE_CONV_WAVE");
    return e && e[0] == '0' ? 0 : 1;
  }();
  // haloed-tile 3x3 kernel (conv_halo.hip): the automatic choice for the 3x3 / s1 / p1 convs
  // where conv_halo_auto says it wins (profiles/r02_conv_bench_halo.txt, in-model per-layer
  // profile r02_layer_profile_halo.txt); tiles 30..35 force it, PRPE_CONV_HALO=0 turns it off
  static const int halo_on = [] {
    const char* e = getenv("PRPE_CONV_HALO");
    return e && e[0] == '0' ? 0 : 1;
  }();
  // 256-row GEMM kernel (conv_gemm.hip): the automatic choice for eligible 1x1 convs / linears
  // over at least 32K pixels whose input is in the planes format (in the model: ViT fc2 -16 %,
  // YOLO adapter 1x1 -9 %; with fp32 input it measured no better than the wave kernel there,
  // profiles/r02_layer_profile_gemm_ab.txt); tiles 40..42 force it, PRPE_CONV_GEMM=0 turns it off
  static const int gemm_on = [] {
    const char* e = getenv("PRPE_CONV_GEMM");
    return e && e[0] == '0' ? 0 : 1;
  }();
  if (tile >= 40 && tile < 50) return conv_gemm_eligible(kp, prec) ? conv_gemm_launch(kp, prec, tile, st) : PRPE_EINVAL;
  // precision 3 (the trunk's fp32 activations, split per frame) on the GEMM kernel: off by
  // default. PRPE_CONV_GEMM_P3=auto routes the deep 1x1s without a residual (K >= 1024), which
  // measured 10-13 % faster than the wave kernel's 256x128 tile while that tile was held to one
  // workgroup per CU by its 132-VGPR build (profiles/r05_layer_profile_p3gemm.txt); with the tile
  // back at 128 VGPRs the wave kernel is the faster one again (profiles/r05_p3gemm_recheck.txt).
  // =1 routes every eligible precision-3 conv (A/B runs).
  static const int gemm_p3 = [] {
    const char* e = getenv("PRPE_CONV_GEMM_P3");
    return e && e[0] == '1' ? 1 : e && e[0] == 'a' ? 2 : 0;
  }();
  const bool p3_gemm = prec == 3 && (gemm_p3 == 1 || (gemm_p3 == 2 && kp.K >= 1024 && kp.res_mode == PRPE_RES_NONE));
  // PRPE_GEMM_TILE=41..49 overrides the automatic GEMM tile (A/B runs)
  static const int gemm_tile = [] {
    const char* e = getenv("PRPE_GEMM_TILE");
    const int t = e ? atoi(e) : 40;
    return t >= 41 && t <= 49 ? t : 40;
  }();
  // the 256 x 256 tile (41) for the GEMMs that write the planes format through an activation
  // (ViT fc1: GELU, face-YOLO adapter.7: SiLU), the 256 x 128 one (40) for the rest: measured in
  // the model at bs = 256 (profiles/r05_layer_profile_gemm_tiles.txt): fc1 0.783 -> 0.725 ms,
  // adapter.7 6.71 -> 6.33 ms on 41, while fc2 / proj (residual epilogues) and qkv lose on it
  // (0.636 -> 0.729, 0.220 -> 0.264, 0.526 -> 0.542). PRPE_GEMM_WIDE=0 keeps 40 everywhere (A/B).
  // The wide tile runs persistent (47: each workgroup walks tiles, the next tile's first K-step
  // DMA'd under this tile's epilogue): fc1 8.77 -> 8.39 ms over the 12 layers, face-YOLO adapter.7
  // 6.29 -> 5.94 ms (profiles/r05_gemm_persist.txt); PRPE_GEMM_WIDE=1 keeps the plain 41.
  static const int gemm_wide = [] {
    const char* e = getenv("PRPE_GEMM_WIDE");
    return e && e[0] == '0' ? 0 : e && e[0] == '1' ? 1 : 2;
  }();
  if (tile == 0 && gemm_on && (kp.x_planes || p3_gemm) && kp.M >= (1 << 15) &&
      conv_gemm_eligible(kp, prec)) {
    const bool wide = gemm_wide && gemm_tile == 40 && kp.y_planes && kp.act != PRPE_ACT_NONE && kp.Co % 256 == 0;
    return conv_gemm_launch(kp, prec, wide ? (gemm_wide == 2 ? 47 : 41) : gemm_tile, st);
  }
  if (tile >= 30 && tile < 40)
    return conv_halo_eligible(kp, prec, km, tile) ? conv_halo_launch(kp, prec, tile, st) : PRPE_EINVAL;
  if (tile == 0 && halo_on && conv_halo_auto(kp, prec) && conv_halo_eligible(kp, prec, km))
    return conv_halo_launch(kp, prec, 30, st);
  // precision 3 (split fp16) and 4 (one fp16 plane) are implemented by the wave-row kernel only
  if (prec >= 3) {
    if (tile != 0 && tile < 20) return PRPE_EINVAL;
    return conv_wave_eligible(kp, prec, km) ? conv_wave_launch(kp, prec, tile ? tile : 20, st) : PRPE_EINVAL;
  }
  if (tile >= 20 || dual || d->x_planes || d->y_planes)
    return conv_wave_eligible(kp, prec, km) ? conv_wave_launch(kp, prec, tile ? tile : 20, st) : PRPE_EINVAL;
  if (tile >= 10) return conv_glds_eligible(kp, prec, km) ? conv_glds_launch(kp, prec, tile, st) : PRPE_EINVAL;
  // wave-row kernel everywhere it applies except two-plane Co <= 64, where the register-staged
  // 256x64 tile measured faster (profiles/r01_conv_bench_wave.txt, r01_conv_bench_sweep_v4.txt)
  if (tile == 0 && wave_on && y.c > 32 && (prec == 2 || y.c > 64) && conv_wave_eligible(kp, prec, km))
    return conv_wave_launch(kp, prec, 20, st);
  // measured (tools/conv_bench.py, profiles/r01_conv_bench_tiles.txt): the 3-plane mode wants the
  // 256x128 8-wave tile for wide Co (operand traffic per MFMA halves; +30%), 128x64 below;
  // the 2-plane mode is near-flat between 128x128 and 256x128 (256x128 +2% on 3x3) and
  // prefers 256x64 for Co <= 64
  if (tile == 0) {
    if (y.c > 64) tile = (prec == 2 || khw > 1) ? 5 : (x.c <= 128 ? 6 : 1);
    else if (y.c > 32) tile = prec == 2 ? 2 : 6;
    else tile = y.c > 16 ? 3 : 4;
  }
  switch (tile) {
    case 1: return launch_cfg<128, 128, 2, 2>(kp, km, prec, st);
    case 2: return launch_cfg<128, 64, 2, 2>(kp, km, prec, st);
    case 3: return launch_cfg<128, 32, 4, 1>(kp, km, prec, st);
    case 4: return launch_cfg<128, 16, 4, 1>(kp, km, prec, st);
    case 5: return launch_cfg<256, 128, 4, 2>(kp, km, prec, st);
    case 6: return launch_cfg<256, 64, 4, 2>(kp, km, prec, st);
    default: return PRPE_EINVAL;
  }
}
