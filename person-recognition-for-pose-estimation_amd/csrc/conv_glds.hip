// Implicit-GEMM convolution on CDNA4 MFMA with direct global->LDS staging
// (global_load_lds_dwordx4), for channel-contiguous inputs with Ci % 32 == 0 (every 1x1 conv,
// linear layer and chunk-major 3x3+ conv of the hot path except the 3/4-channel stems).
//
// Same GEMM view, split-bf16 arithmetic and epilogue as conv_igemm.hip (see there):
//   A[m,k] = x[n, oh*s-p+kh, ow*s-p+kw, ci] (fp32, gathered), B[k,co] = packed bf16 planes.
// What differs is the staging. conv_igemm loads A into registers, splits it into bf16 planes
// and writes those to LDS: ~135 VALU + 6 LDS writes per wave per K-step, issued in the MFMA
// shadow. Here the K-loop has no register staging at all:
//   * A (fp32, 128 B per tile row per K-step) and B (NP planes x 64 B per row) go straight
//     from global memory to LDS, 16 B per lane, in a STAGES-deep ring; a wave waits for its
//     own copies with a counted vmcnt and a raw s_barrier, so the copies of the next
//     STAGES-1 K-steps stay in flight across the barrier;
//   * each wave owns BM/NW full-width rows (waves tile M only), reads its A fragment rows as
//     fp32 from LDS and splits them into bf16 planes in registers (every A element is split
//     by exactly one wave), and reads the B planes as MFMA fragments.
// LDS images are lane-linear (a glds writes base + 16*lane), so the XOR swizzles that make the
// fragment reads conflict-free are applied to the per-lane SOURCE address (and undone on the
// read): A slot c of row r sits at physical slot c ^ ((r >> 1) & 7) in its 128-B row; B chunk j
// of row n at j ^ swzF(n) in its 64-B row. Padding taps read a zero page.
#include "conv.h"

namespace prpe_k {
namespace {

constexpr int BK = 32;

__device__ __forceinline__ int swzA(int r) { return (r >> 1) & 7; }

template <int BM, int BN, int NW, int NP, int STAGES>
__global__ __launch_bounds__(NW * 64, 2) void conv_glds_kernel(ConvK p) {
  constexpr int NT = NW * 64;
  constexpr int WTM = BM / NW;                 // tile rows per wave (waves tile M only)
  constexpr int TM = WTM / 16, TN = BN / 16;
  constexpr int A_BYTES = BM * 128;            // fp32 [BM][32]
  constexpr int B_BYTES = NP * BN * 64;        // bf16 [NP][BN][32]
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int IA = BM / (8 * NW);            // A wave-instructions per wave per stage
  constexpr int NB_TOT = NP * BN / 16;         // B wave-instructions per stage
  constexpr int IB = (NB_TOT + NW - 1) / NW;   // per wave (surplus slots repeat a copy: same bytes)
  constexpr int G = IA + IB;                   // glds per wave per stage (uniform over waves)
  constexpr int LDS_BYTES = STAGES * STAGE;
  constexpr int CS = BN + 4;                   // epilogue C tile pitch (floats)
  constexpr int CH_FIT = LDS_BYTES / (CS * 4);
  constexpr int CH = CH_FIT >= BM ? BM : (CH_FIT / 16) * 16;
  static_assert(TM >= 1 && TN >= 1 && IA >= 1 && BM % (8 * NW) == 0, "tile");
  static_assert(CH >= 16, "epilogue staging");
  static_assert(STAGES == 2 || STAGES == 3, "stages");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = xcd_remap(blockIdx.x, p.nwg);
  const int tile_m = L / p.tiles_n, tile_n = L % p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // ---- A copies: lane -> (row, 16-B slot) of each of this wave's IA instructions. The source
  // element offset folds in the swizzled channel group; invalid taps / rows read the zero page.
  int64_t rbase[IA];
  unsigned hmask[IA], wmask[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int row = (wave * IA + i) * 8 + (lane >> 3);
    const int m = m0 + row;
    const int c = (lane & 7) ^ swzA(row);
    unsigned hm = 0, wmk = 0;
    int64_t b = 0;
    if (m < p.M) {
      const int n = m / p.HoWo;
      const int rem = m - n * p.HoWo;
      const int oh = rem / p.Wo;
      const int ow = rem - oh * p.Wo;
      const int ih = oh * p.stride - p.pad, iw = ow * p.stride - p.pad;
      b = (int64_t)n * p.xsn + (int64_t)ih * p.xsh + (int64_t)iw * p.xsw + c * 4;
      for (int t = 0; t < p.KH; ++t) hm |= (unsigned)((unsigned)(ih + t) < (unsigned)p.Hi) << t;
      for (int t = 0; t < p.KW; ++t) wmk |= (unsigned)((unsigned)(iw + t) < (unsigned)p.Wi) << t;
    }
    rbase[i] = b;
    hmask[i] = hm;
    wmask[i] = wmk;
  }
  // ---- B copies: instruction j -> plane j / (BN/16), rows 16*(j % (BN/16)) .. +16
  const uint16_t* bsrc[IB];
  int bdst[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    int j = wave * IB + i;
    if (j >= NB_TOT) j -= NB_TOT;
    const int q = j / (BN / 16), rb = j % (BN / 16);
    const int nrow = rb * 16 + (lane >> 2);
    const int ch = (lane & 3) ^ swzF(nrow);
    const uint16_t* plane = q == 0 ? p.whi : (q == 1 ? p.wlo : p.wlo2);
    bsrc[i] = plane + (int64_t)(n0 + nrow) * p.k_pad + ch * 8;
    bdst[i] = A_BYTES + (q * BN + rb * 16) * 64;
  }

  // K-step walk of the copy side (wave-uniform): k = ((ci/32)*KH*KW + kh*KW + kw)*32 + ci%32
  int u_kh = 0, u_kw = 0;
  int64_t u_off = 0;                           // kh*xsh + kw*xsw + chunk*32
  auto issue = [&](int kt, int stage) {
    unsigned char* sb = lds + stage * STAGE;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const bool ok = (hmask[i] >> u_kh) & (wmask[i] >> u_kw) & 1u;
      const float* src = ok ? p.x + (rbase[i] + u_off) : p.zero;
      glds16(src, sb + (wave * IA + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) glds16(bsrc[i] + (int64_t)kt * BK, sb + bdst[i]);
    u_off += p.xsw;
    if (++u_kw == p.KW) {
      u_kw = 0; u_off += p.xsh - (int64_t)p.KW * p.xsw;
      if (++u_kh == p.KH) { u_kh = 0; u_off += BK - (int64_t)p.KH * p.xsh; }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;

  auto compute = [&](int stage) {
    const unsigned char* sb = lds + stage * STAGE;
    bf16x8 af[NP][TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wave * WTM + i * 16 + fr;
      const unsigned char* rp = sb + row * 128;
      const f4 v0 = *reinterpret_cast<const f4*>(rp + (((2 * fg) ^ swzA(row)) << 4));
      const f4 v1 = *reinterpret_cast<const f4*>(rp + (((2 * fg + 1) ^ swzA(row)) << 4));
      bf16x4 p0[NP], p1[NP];
      split_planes<NP>(v0, p0);
      split_planes<NP>(v1, p1);
#pragma unroll
      for (int q = 0; q < NP; ++q)
        af[q][i] = bf16x8{p0[q][0], p0[q][1], p0[q][2], p0[q][3], p1[q][0], p1[q][1], p1[q][2], p1[q][3]};
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nrow = j * 16 + fr;
      const unsigned char* bp = sb + A_BYTES + nrow * 64 + ((fg ^ swzF(nrow)) << 4);
      bf16x8 bfr[NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) bfr[q] = *reinterpret_cast<const bf16x8*>(bp + q * BN * 64);
      // partial products smallest first; terms with plane-index sum >= NP are dropped
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int s = NP - 1; s >= 0; --s)
#pragma unroll
          for (int qa = s; qa >= 0; --qa)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[qa][i], bfr[s - qa], acc[i][j], 0, 0, 0);
    }
  };

  // ---------------- main loop: STAGES-1 K-steps of copies in flight
  const int nk = p.nk;
  issue(0, 0);
  if constexpr (STAGES == 3) {
    if (nk > 1) issue(1, 1);
    int st = 0;
    for (int kt = 0; kt < nk; ++kt) {
      // this wave's copies of K-step kt are done once at most the next step's G are pending;
      // the barrier then publishes every wave's copies and retires all reads of step kt-1
      if (kt + 1 < nk) wait_barrier<G>();
      else wait_barrier<0>();
      if (kt + 2 < nk) issue(kt + 2, st == 0 ? 2 : st - 1);
      compute(st);
      st = st == 2 ? 0 : st + 1;
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) {
      wait_barrier<0>();
      if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);
      compute(kt & 1);
    }
  }
  __syncthreads();   // all fragment reads done before the ring is reused for the C tile

  // ---------------- epilogue (as conv_igemm.hip): C tile staged through LDS, whole-row
  // 16-B column chunks per thread, coalesced residual loads and output stores
  float* ct = reinterpret_cast<float*>(lds);
  FrameMax ymax;                               // per-frame running max|y| (p.y_amax)
  constexpr int CPR = BN / 4;
  constexpr int RPP = NT / CPR;
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
        const int row = wave * WTM + i * 16 + fg * 4 + r - h0;
        if (row >= 0 && row < CH)
#pragma unroll
          for (int j = 0; j < TN; ++j) ct[row * CS + j * 16 + fr] = acc[i][j][r];
      }
    __syncthreads();
    if (col < p.Co) {
      const int rows = BM - h0 < CH ? BM - h0 : CH;
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
}

template <int BM, int BN, int NW, int NP2_STAGES, int NP3_STAGES>
int launch(const ConvK& kp0, int prec, hipStream_t st) {
  ConvK kp = kp0;
  const int tiles_m = (kp.M + BM - 1) / BM;
  kp.tiles_n = (kp.Co + BN - 1) / BN;
  kp.nwg = tiles_m * kp.tiles_n;
  if (prec == 0)
    hipLaunchKernelGGL((conv_glds_kernel<BM, BN, NW, 2, NP2_STAGES>), dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
  else
    hipLaunchKernelGGL((conv_glds_kernel<BM, BN, NW, 3, NP3_STAGES>), dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
  return launch_status();
}

}  // namespace

bool conv_glds_eligible(const ConvK& kp, int prec, int km) {
  // chunk-major K walk (km 2, or any 1x1 on the vector path with whole 32-channel chunks),
  // no prologue, vectorised epilogue, precision 0 / 2, K in whole K-steps
  const bool chunked = km == 2 || (km == 1 && kp.KH * kp.KW == 1 && kp.Ci % 32 == 0);
  return chunked && kp.in_scale == nullptr && kp.vec_out && (prec == 0 || prec == 2) &&
         kp.K % BK == 0 && kp.k_pad == kp.K && kp.zero != nullptr;
}

int conv_glds_launch(const ConvK& kp, int prec, int tile, hipStream_t st) {
  if (tile == 0) tile = kp.Co > 64 ? 10 : 11;
  // LDS per stage (A 128 B/row + NP*64 B per B row): 256x128 48 / 56 KB, 256x64 40 / 44 KB,
  // 128x128 32 / 40 KB -> 3 stages where they fit in 160 KB, else 2
  switch (tile) {
    case 10: return launch<256, 128, 8, 3, 2>(kp, prec, st);
    case 11: return launch<256, 64, 8, 3, 3>(kp, prec, st);
    case 12: return launch<128, 128, 4, 3, 3>(kp, prec, st);
    default: return PRPE_EINVAL;
  }
}

}  // namespace prpe_k
