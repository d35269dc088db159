// 1x1 convolutions / linears (a plain GEMM over contiguous pixels: M = pixels, K = Ci,
// N = Co) on 256-row block tiles with BOTH operands staged in LDS by LDS-DMA.
//
// Why (tools/conv_bench.py ablations, profiles/r02_conv_ablation.txt): in the wave-row kernel a
// 128 x 128 block issues 8 vector-memory instructions per wave for every 48 MFMAs (A fragment
// loads + B ring DMA), and removing them makes the ViT fc2 GEMM 2x faster. A 256 x 256 tile
// halves the memory instructions per MFMA: per 32-deep K-step the block DMAs 32 KB of A (256
// rows x 32 channels, full 128-B lines) and 32 KB of B (2 planes x 256 columns x 64 B) -- 8
// pieces per wave -- for 96 MFMAs per wave; each A row is read from LDS by the 4 waves that
// share it instead of being fetched from L2 by one wave per column tile.
// Measured (profiles/r02_conv_bench_gemm.txt): that 256 x 256 two-stage tile (41) exposes the
// DMA latency (one block per CU, one step of lookahead) and loses to a 256 x 128 tile with a
// three-stage ring (40, the automatic one: 8 waves = 4 (M) x 2 (N), wave tile 64 x 64,
// 6 pieces per wave for 48 MFMAs, 144 KB LDS, two steps of lookahead).
//
// Per K-step: counted vmcnt + s_barrier (step kt landed, step kt+1 may be in flight), then the
// DMA of step kt + STAGES - 1 into the stage read at kt - 1 (pieces spread over this step's
// row blocks), fragments of step kt from LDS, MFMAs. Same K order, plane split and
// per-accumulator MFMA order as conv_wave.hip (bit-identical results, tested).
//
// LDS per stage: A [256 rows][8 slots x 16 B] (slot s of row r at s ^ swz_rows(r), conv.h) then B [2 planes]
// [BN cols][64 B] (conv_wave's swizzle). The epilogue slab reuses stage 0.
// swz_rows: a ds_read_b128 is serviced in four 16-lane groups (MI355X_MICROARCH.md, LDS), each
// holding rows fr = {0-3, 12-15} of one 16-B column slot L and rows {4-11} of slot L ^ 2. With the
// rows' 128-B pitch, even and odd rows fall in opposite halves of the 256-B bank row, so the slot
// function must give {f(r)} of one set and {f(r) ^ 2} of the other = all 8 slots per parity:
// f(r) = k & 5 with k = r >> 1 does (the earlier (r >> 1) & 7 was 2-way on every group: the
// 33 % of LDS-active cycles profiles/r02_pmc_fc2.txt shows as bank conflicts).
#include "conv.h"

namespace prpe_k {
namespace {

constexpr int GBK = 32;


// F16: precision 3 (fp16 planes of the per-frame-scaled activations, the weights' fp16 planes
// pre-scaled per output channel; the per-row inverse scale in the epilogue), as conv_wave.hip.
// BM = 128 (tile 43): 128 x 128 at 2 stages = 64 KB of LDS, two workgroups (16 waves) per CU
// PRIO (A/B, round 5; cdna_hip_programming.md T5): 1 = s_setprio(1) around each row block's MFMA
// cluster, 2 = the static form (the second-dispatched half, waves 4-7, at priority 1 for the whole
// K-loop), 0 = none
// EARLY (A/B, round 5): every DMA piece of the step issued right after the barrier (the
// minimum-2-phase recipe, cdna_hip_programming.md T3+T4) instead of one per row block.
// PERSIST (round 5, tiles 49 / 47): a workgroup walks tiles t, t + G, ... (G = the grid, a few per
// CU): right after a tile's last K-step its successor's first STAGES - 1 steps are DMA'd into the
// ring while this tile's epilogue runs out of the last stage (its slab fits one stage), so the
// ring refill and the workgroup launch no longer sit between two tiles' MFMAs. Same arithmetic
// (bit-identical).
template <int BN, int WM, int STAGES, bool APL, bool F16, int BM = 256, int PRIO = 0, bool EARLY = false,
          bool PERSIST = false>
__global__ __launch_bounds__(512, BM == 128 ? 4 : 1) void conv_gemm_kernel(ConvK p) {
  static_assert(!(APL && F16), "planes input is precision 0");
  using frag_t = typename std::conditional<F16, f16x8, bf16x8>::type;
  constexpr int NW = 8, NP = 2;
  constexpr int WN = NW / WM;                          // waves along N
  constexpr int WTN = BN / WN;                         // wave tile (BM / WM) x WTN
  constexpr int TM = BM / WM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * 128;                    // 32 KB
  constexpr int B_BYTES = NP * BN * 64;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int NA = A_BYTES / 1024, NBP = B_BYTES / 1024;
  constexpr int PW = (NA + NBP) / NW;                  // pieces per wave and K-step
  static_assert((NA + NBP) % NW == 0, "pieces");
  constexpr int CS = WTN + 4;                          // epilogue row pitch (floats)
  static_assert(NW * 16 * CS * 4 <= STAGES * STAGE, "epilogue slab");
  static_assert(!PERSIST || NW * 16 * CS * 4 <= STAGE, "persistent: the slab fits the last stage");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int wm = wave / WN, wn = wave % WN;
  int t = blockIdx.x;                                  // tile index (PERSIST: t, t + G, ...)
  int m0, n0;

  // ---- this wave's DMA pieces: j = wave * PW + i; j < NA: A rows 8j .. 8j+7, else B
  const float* src[PW];
  int dst[PW];
  auto setup = [&](int tt) {
    const int L = xcd_remap(tt, p.nwg);
    const int tile_m = L / p.tiles_n, tile_n = L % p.tiles_n;
    m0 = tile_m * BM;
    n0 = tile_n * BN;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int j = wave * PW + i;
      if (j < NA) {
        const int row = j * 8 + (lane >> 3);
        const int s = (lane & 7) ^ swz_rows(row);            // logical slot landing in this lane's slot
        const int m = m0 + row < p.M ? m0 + row : p.M - 1;   // tail rows re-read the last row
        src[i] = p.x + (int64_t)m * p.xsw + s * 4;
        dst[i] = j * 1024;
      } else {
        const int jb = j - NA;
        const int q = jb / (BN / 16), rb = jb % (BN / 16);
        const int nrow = rb * 16 + (lane >> 2);
        const int ch = (lane & 3) ^ swzF(nrow);
        const uint16_t* plane = F16 ? (q == 0 ? p.wh16 : p.wl16) : (q == 0 ? p.whi : p.wlo);
        src[i] = reinterpret_cast<const float*>(plane + (int64_t)(n0 + nrow) * p.k_pad + ch * 8);
        dst[i] = A_BYTES + (q * BN + rb * 16) * 64;
      }
    }
  };
  setup(t);
  // K-step advance of each piece's source: A 32 channels (floats), B 32 bf16 = 16 floats
  auto piece = [&](int i, int kt, int stage) {
    const int j = wave * PW + i;
    const float* s = src[i] + (int64_t)kt * (j < NA ? GBK : GBK / 2);
    glds16(s, lds + stage * STAGE + dst[i]);
  };

  bool pre = false;                                    // PERSIST: this tile's first steps already issued
  for (;;) {
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // precision 3: scale of each A row this lane splits (its frame's max|x| bound)
  float rsc[F16 ? TM : 1];
  if constexpr (F16) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * (BM / WM) + i * 16 + fr;
      rsc[i] = m < p.M ? ldexpf(1.f, 15 - f16_scale_exp(p.x_amax[m / p.HoWo])) : 1.f;
    }
  }

  const int nk = p.nk;
  if (!pre) {
#pragma unroll
    for (int i = 0; i < PW; ++i) piece(i, 0, 0);
    if constexpr (STAGES == 3) {
#pragma unroll
      for (int i = 0; i < PW; ++i) piece(i, nk > 1 ? 1 : 0, 1);
    }
  }

  if constexpr (PRIO == 2)
    if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // step kt landed (with 3 stages the PW pieces of step kt+1 may stay in flight)
    wait_barrier<(STAGES - 2) * PW>();
    // the step issued now (kt + STAGES - 1, clamped to the last: a harmless re-read into the
    // stage read at kt - 1, so the wait counts stay exact) goes into that stage
    const int ks = kt + STAGES - 1 < nk ? kt + STAGES - 1 : nk - 1;
    const int sn = st == 0 ? STAGES - 1 : st - 1;
    const bool more = STAGES == 3 || kt + 1 < nk;
    const unsigned char* sa = lds + st * STAGE;
    const unsigned char* sb = sa + A_BYTES;
    if constexpr (EARLY) {
      if (more) {
#pragma unroll
        for (int u = 0; u < PW; ++u) piece(u, ks, sn);
      }
    }
    // B fragments of the wave's 4 column blocks (both planes), held for the whole step
    frag_t bfr[TN][NP];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nrow = wn * WTN + j * 16 + fr;
      const unsigned char* bp = sb + nrow * 64 + ((fg ^ swzF(nrow)) << 4);
#pragma unroll
      for (int q = 0; q < NP; ++q) bfr[j][q] = *reinterpret_cast<const frag_t*>(bp + q * BN * 64);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (!EARLY && more) {                             // the DMA pieces spread over the row blocks
#pragma unroll
        for (int u = PW * i / TM; u < PW * (i + 1) / TM; ++u) piece(u, ks, sn);
      }
      const int row = wm * (BM / WM) + i * 16 + fr;
      const int sw = swz_rows(row);
      const unsigned char* ap = sa + row * 128;
      const f4 v0 = *reinterpret_cast<const f4*>(ap + (((2 * fg) ^ sw) << 4));
      const f4 v1 = *reinterpret_cast<const f4*>(ap + (((2 * fg + 1) ^ sw) << 4));
      frag_t af[NP];
      if constexpr (APL) {
        af[0] = __builtin_bit_cast(bf16x8, v0);
        af[1] = __builtin_bit_cast(bf16x8, v1);
      } else if constexpr (F16) {
        unsigned long long p0[2], p1[2];
        split_planes_f16(v0, rsc[i], p0);
        split_planes_f16(v1, rsc[i], p1);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
          af[q] = __builtin_bit_cast(f16x8, u64x2{p0[q], p1[q]});
        }
      } else {
        bf16x4 p0[NP], p1[NP];
        split_planes<NP>(v0, p0);
        split_planes<NP>(v1, p1);
#pragma unroll
        for (int q = 0; q < NP; ++q)
          af[q] = bf16x8{p0[q][0], p0[q][1], p0[q][2], p0[q][3], p1[q][0], p1[q][1], p1[q][2], p1[q][3]};
      }
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int s = NP - 1; s >= 0; --s)
#pragma unroll
          for (int qa = s; qa >= 0; --qa) acc[i][j] = mfma16(af[qa], bfr[j][s - qa], acc[i][j]);
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
    }
    st = st + 1 == STAGES ? 0 : st + 1;
  }
  wait_barrier<0>();
  if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);

  // ---------------- epilogue: per-wave 16-row x 64-column slices, 16-B row stores
  // (PERSIST: the slab is the last stage; the others take the next tile's first steps below)
  float* ct = reinterpret_cast<float*>(lds + (PERSIST ? (STAGES - 1) * STAGE : 0)) + wave * 16 * CS;
  constexpr int CPR = WTN / 4, RPP = 64 / CPR, EB = 16 / RPP;
  const int cc = lane % CPR, rr0 = lane / CPR;
  const int col = n0 + wn * WTN + cc * 4;
  const bool cval = col < p.Co;
  const int em0 = m0;
  f4 sc4 = {1.f, 1.f, 1.f, 1.f}, bi4 = {0.f, 0.f, 0.f, 0.f}, sl4 = {0.f, 0.f, 0.f, 0.f};
  if (cval) {
    if (p.scale) sc4 = *reinterpret_cast<const f4*>(p.scale + col);
    if (p.bias) bi4 = *reinterpret_cast<const f4*>(p.bias + col);
    if (p.slope) sl4 = *reinterpret_cast<const f4*>(p.slope + col);
  }
  if constexpr (PERSIST) {
    // the next tile's steps 0 and 1, issued after this tile's epilogue constants (one in-order
    // vmcnt: the compiler's waits for those loads then leave these pieces in flight)
    pre = t + (int)gridDim.x < p.nwg;
    if (pre) {
      setup(t + (int)gridDim.x);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < PW; ++i) piece(i, 0, 0);
      if constexpr (STAGES == 3) {
#pragma unroll
        for (int i = 0; i < PW; ++i) piece(i, nk > 1 ? 1 : 0, 1);
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  FrameMax ymax;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < TN; ++j) ct[(fg * 4 + r) * CS + j * 16 + fr] = acc[i][j][r];
    __builtin_amdgcn_wave_barrier();
    f4 res[EB];
    bool ok[EB];
    int mm[EB];
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int m = em0 + wm * (BM / WM) + i * 16 + rr0 + RPP * e;
      mm[e] = m;
      ok[e] = cval && m < p.M;
      res[e] = f4{0.f, 0.f, 0.f, 0.f};
      if (ok[e] && p.res_mode != PRPE_RES_NONE) res[e] = *reinterpret_cast<const f4*>(p.r + (int64_t)m * p.rsw + col);
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      f4 v = *reinterpret_cast<const f4*>(ct + (rr0 + RPP * e) * CS + cc * 4);
      if (!ok[e]) continue;
      if constexpr (F16) v = v * ldexpf(1.f, f16_scale_exp(p.x_amax[mm[e] / p.HoWo]) - 15);
      v = v * sc4 + bi4;
      if (p.res_mode == PRPE_RES_PRE_ACT) v += res[e];
      v = apply_act4(v, p.act, sl4);   // packed GELU / SiLU, bit-identical to apply_act
      if (p.res_mode == PRPE_RES_POST_ACT) v += res[e];
      const int64_t yo = (int64_t)mm[e] * p.ysw + col;
      if (p.y_planes) {
        bf16x4 pl[2];
        split_planes<2>(v, pl);
        uint16_t* y16 = reinterpret_cast<uint16_t*>(p.y) + 2 * (yo - col) + (col >> 3) * 16 + (col & 7);
        // non-temporal output stores: the ViT GEMMs -4 % each in the model (fc1 0.719 -> 0.697,
        // fc2 0.667 -> 0.630 ms), profiles/r05_gemm_nt_ab.txt; NT A loads lose (A is re-read per
        // column tile)
        __builtin_nontemporal_store(pl[0], reinterpret_cast<bf16x4*>(y16));
        __builtin_nontemporal_store(pl[1], reinterpret_cast<bf16x4*>(y16 + 8));
      } else {
        __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p.y + yo));
      }
      if (p.y_amax) ymax.add(p.y_amax, mm[e] / p.HoWo, amax4(v));
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (p.y_amax) frame_amax_final(p.y_amax, ymax);
  if constexpr (!PERSIST) break;
  t += gridDim.x;
  if (t >= p.nwg) break;
  }
}

}  // namespace

bool conv_gemm_eligible(const ConvK& kp, int prec) {
  // 1x1 / stride 1 / pad 0 over contiguous pixels (x, y, residual rows at one pixel stride),
  // whole 32-channel K-steps, Co a multiple of 128, precision 0 (fp32 or planes input) or 3
  // (fp32 input, fp16 planes + the input's per-frame max bound), vectorised epilogue, no
  // prologue / dual input
  const bool xlin = kp.xsh == (int64_t)kp.Wi * kp.xsw && kp.xsn == (int64_t)kp.Hi * kp.xsh && kp.xsc == 1;
  const bool p0 = prec == 0 && kp.whi && kp.wlo;
  const bool p3 = prec == 3 && kp.wh16 && kp.wl16 && kp.x_amax && !kp.x_planes;
  return (p0 || p3) && kp.KH == 1 && kp.KW == 1 && kp.stride == 1 && kp.pad == 0 && kp.Ci % GBK == 0 &&
         kp.K == kp.Ci && kp.k_pad == kp.K && kp.Co % 128 == 0 && kp.vec_out && kp.ylin && kp.rlin && xlin &&
         !kp.in_scale && !kp.x2 && kp.xsw % 4 == 0;
}

// PERSIST: the grid is PRPE_GEMM_PERSIST (default 4) workgroups per CU (one runs at a time per CU:
// the rest balance the tail when other streams' kernels hold CUs), each walking nwg / grid tiles
int gemm_persist_grid(int64_t nwg) {
  // 4 workgroups per CU (round 5's sweep of 2 / 4 / 8 / 16 was flat, profiles/r05_gemm_persist.txt)
  constexpr int per_cu = 4;
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  // a multiple of 8 (t + G stays on t's XCD), and at least 8: a device (or partition) with fewer
  // than two CUs would otherwise round the grid down to 0 workgroups
  int64_t g = (int64_t)per_cu * cus / 8 * 8;
  if (g < 8) g = 8;
  return (int)(nwg < g ? nwg : g);
}

template <int BN, int WM, int STAGES, int BM = 256, int PRIO = 0, bool EARLY = false, bool PERSIST = false>
int launch_gemm(const ConvK& kp0, int prec, hipStream_t st) {
  if (kp0.Co % BN) return PRPE_EINVAL;
  ConvK kp = kp0;
  kp.tiles_n = kp.Co / BN;
  const int64_t nwg = (int64_t)((kp.M + BM - 1) / BM) * kp.tiles_n;
  if (nwg >= (1LL << 31)) return PRPE_EINVAL;
  kp.nwg = (int)nwg;
  const dim3 g(PERSIST ? gemm_persist_grid(nwg) : kp.nwg), b(512);
  if (prec == 3)
    hipLaunchKernelGGL((conv_gemm_kernel<BN, WM, STAGES, false, true, BM, PRIO, EARLY, PERSIST>), g, b, 0, st, kp);
  else if (kp.x_planes)
    hipLaunchKernelGGL((conv_gemm_kernel<BN, WM, STAGES, true, false, BM, PRIO, EARLY, PERSIST>), g, b, 0, st, kp);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<BN, WM, STAGES, false, false, BM, PRIO, EARLY, PERSIST>), g, b, 0, st, kp);
  return launch_status();
}

// tile 40 = auto (256 x 128, 3 stages), 41 = 256 x 256 (2 stages), 42 = 256 x 128 (2 stages),
// 43 = 128 x 128 (2 stages, two workgroups per CU); 44 / 45 = tile 40 with PRIO 1 / 2, 46 = tile
// 41 with PRIO 1, 48 = tile 40 with PRIO 1 and EARLY (A/B), 47 / 49 = tiles 41 / 40 persistent
int conv_gemm_launch(const ConvK& kp, int prec, int tile, hipStream_t st) {
  switch (tile) {
    case 41: return launch_gemm<256, 2, 2>(kp, prec, st);
    case 42: return launch_gemm<128, 4, 2>(kp, prec, st);
    case 43: return launch_gemm<128, 4, 2, 128>(kp, prec, st);
    case 44: return launch_gemm<128, 4, 3, 256, 1>(kp, prec, st);
    case 45: return launch_gemm<128, 4, 3, 256, 2>(kp, prec, st);
    case 46: return launch_gemm<256, 2, 2, 256, 1>(kp, prec, st);
    case 47: return launch_gemm<256, 2, 2, 256, 0, false, true>(kp, prec, st);
    case 48: return launch_gemm<128, 4, 3, 256, 1, true>(kp, prec, st);
    case 49: return launch_gemm<128, 4, 3, 256, 0, false, true>(kp, prec, st);
    default: return launch_gemm<128, 4, 3>(kp, prec, st);
  }
}

}  // namespace prpe_k
