// Implicit-GEMM convolution on CDNA4 MFMA, "wave-row" variant: every wave owns whole output
// rows of the block tile (waves tile M only, each wave WTM x BN), the activation operand goes
// straight from global memory into the wave's MFMA fragment registers, and only the weight
// planes -- the operand every wave of the block shares -- are staged in LDS.
//
// Same GEMM view, K order, split-bf16 arithmetic and MFMA order as conv_igemm.hip / conv_glds.hip
// (the accumulation order per output element is identical, so the three kernels agree bit for
// bit):
//   A[m,k] = PRO(x[n, oh*s-p+kh, ow*s-p+kw, ci]) fp32, B[k,co] = packed bf16 planes [co][k].
//
// Why: in the LDS-staged kernels a wave issues 6 LDS-DMA pieces (~60 issue cycles each beside
// MFMAs), 20 fragment reads and the plane split for 48 MFMAs per K-step, and measured ~40 % of
// the MFMA rate. Here, at 64x128 per wave and two planes, one K-step is 96 MFMAs against
// 8 global loads (A, 32 B per lane per row block), 2 LDS-DMA pieces (B), 16 fragment reads and
// the split of 8 float4 -- the issue budget stays inside the MFMA shadow.
//
// A fragment of v_mfma_f32_16x16x32_bf16: lane (fr = lane & 15, fg = lane >> 4) holds row fr,
// k = 8 fg .. 8 fg + 7 -- i.e. channels 8 fg .. 8 fg + 7 of the K-step's 32-channel chunk at one
// tap: two 16-B loads. Rows whose tap falls into the padding read a 32-B zero page.
//
// Pipeline per K-step kt (B ring STAGES deep, A one step ahead in registers):
//   wait(my B pieces of step kt) + s_barrier     -- publishes every wave's pieces of step kt
//   load A(kt+1) -> raw registers                -- in flight across the MFMAs
//   LDS-DMA B(kt+STAGES-1) into the stage read at kt-1
//   MFMAs of step kt (B fragments from LDS, A planes in registers)
//   split raw -> A planes of step kt+1 (waits for A(kt+1), not for the younger B pieces)
// Loads past the last K-step are clamped to it (a harmless re-read), so the loop body is
// uniform and the compiler's vmcnt bookkeeping is exact.
//
// Epilogue: each wave stages its accumulator rows through a private 16-row LDS slice and
// writes whole-row 16-B vectors (scale/bias, act, residual), no block barrier.
#include "conv.h"
#include <stdlib.h>

namespace prpe_k {
namespace {

constexpr int BK = 32;

// F16 (precision 3): two fp16 planes instead of bf16 ones. The weights arrive pre-scaled per
// output channel (2^e[co], folded back through the epilogue scale); the activations are
// scaled by sa = 2^(15 - e) with max|x| < 2^e read from the producer's running maximum of
// the row's frame (x_amax[n], per-frame slots: a frame's rounding never depends on its
// batch-mates), so every scaled value is < 2^15 and the planes stay inside fp16's range: operand
// error ~2^-22, below fp32's own accumulation error for K >= 64 (Precision).
// DUAL: two 1x1 inputs summed in one GEMM, y = EPI(W[:, :K1] x + W[:, K1:] x2) (a ResNet
// bottleneck's conv3 and its downsample projection: the projection is never written to HBM
// and re-read as the residual). K-steps 0 .. nk1-1 read x, the rest read x2 (a view with the
// output's pixel grid, e.g. a stride-2 subsampling of the block input).
// APL: the input tensor is stored as interleaved bf16 planes (see prpe.h, "planes format"):
// the 32 bytes a lane loads for 8 channels already are the hi and lo fragments, no split.
// ONE (precision 4, with F16): ONE scaled fp16 plane per operand (RNE), one MFMA per product
// instead of three; the weights' hi plane alone (w_h16 = RNE(w 2^e[co])) is staged. Allows the
// prologue affine: the activation scale then comes from a bound of the prologue's output
// (prologue_bounds, conv.h). With a third of the MFMAs per K-step the per-step barrier would
// dominate, so one iteration covers TWO K-steps (KS = 2): the B stage holds the hi plane of
// K-steps 2s and 2s+1 where the two-plane forms hold two planes of one step (same 16 KB at
// BN = 128), and each accumulator takes step 2s then 2s+1 (the sequential order).
// launch bound: HIP's second argument is waves per SIMD. The 8-wave 2-plane tiles of 32-row
// waves without a prologue ask for 4 (two workgroups per CU, <= 128 VGPRs; they need 122-128):
// the precision-3 256x128 tile (the trunk's unfused convs) sat at exactly 128 until the round-4/5
// GELU rewrites grew the runtime-switched epilogue and it compiled to 132 -- one workgroup per CU,
// those convs 15-27 % slower. The larger tiles keep 2 (their 150-240 VGPRs would
// spill at 128). The precision-4 4-wave tile at two K-steps (KSF 1: AdaFace) likewise asks for
// 4 waves per SIMD (four workgroups per CU at 128 VGPRs; it had grown to 132).
template <int NW, int TM, int NP, bool PRO, bool ONE, int KSF>
constexpr int wave_wps() {
  return (NW == 8 && TM == 2 && NP == 2 && !PRO) || (NW == 4 && TM == 2 && ONE && KSF == 1 && !PRO) ? 4 : 2;
}
template <int NW, int TM, int TN, int NP, int STAGES, bool PRO, bool F16 = false, bool DUAL = false,
          bool APL = false, bool ONE = false, int KSF = 0, int XM = 0>
__global__ __launch_bounds__(NW * 64, (wave_wps<NW, TM, NP, PRO, ONE, KSF>())) void conv_wave_kernel(ConvK p) {
  static_assert(!APL || (NP == 2 && !F16 && !PRO && !DUAL), "planes input: two bf16 planes only");
  static_assert(!F16 || (NP == 2 && (!PRO || ONE)), "f16 planes: two planes, no prologue unless single-plane");
  static_assert(!ONE || (F16 && !DUAL && !APL), "single fp16 plane: precision 4");
  static_assert(!DUAL || !PRO, "dual input: no prologue");
  using frag_t = typename std::conditional<F16, f16x8, bf16x8>::type;
  // K-steps per iteration: 2 for ONE, except the 8-wave prologue tile (154 VGPRs at 2 steps: one
  // workgroup per CU instead of two, 56x56 IR-50 res_layer convs +12 %)
  // (KSF = 1 forces one K-step: 128 instead of 160 VGPRs on the 128 x 128 tile, 4 workgroups per CU)
  constexpr int KS = ONE && !(PRO && NW == 8) && KSF != 1 ? 2 : 1;
  constexpr int NSL = ONE ? KS : NP;                  // B stage slices: planes, or (ONE) K-steps
  constexpr int WTM = TM * 16, BM = NW * WTM, BN = TN * 16;
  constexpr int B_STAGE = NSL * BN * 64;              // bf16 / f16 [NSL][BN][32]
  constexpr int NB_TOT = NSL * BN / 16;               // 1-KiB LDS-DMA pieces per stage
  constexpr int IB = (NB_TOT + NW - 1) / NW;          // per wave (surplus slots repeat a piece)
  constexpr int CS = BN + 4;                          // epilogue row pitch (floats)
  constexpr int EPI = NW * 16 * CS * 4;
  constexpr int RING = STAGES * B_STAGE;
  // XM 1 (1x1 convs without padding, two fp32-derived planes): the A loads go out pixel-contiguous
  // -- load h (0, 1) of a row block: lane l reads row 8 h + (l >> 3), 16-B chunk l & 7 of the
  // K-step's 128 B, so each lane quad covers 64 contiguous bytes -- and a wave-private 2-KiB LDS
  // slot past the ring transposes them into the fragment layout (lane (fr, fg): row fr, channels
  // 8 fg .. +7) before the split, one row block after the other. Straight into fragment lanes,
  // every quad spans 4 pixels a row pitch apart: the texture-address unit was busy 0.68 of this
  // kernel's cycles over the model (profiles/r06_pmc_ta_table.txt). In the model (same box,
  // profiles/r06_layer_profile_x11_ab.txt) the trunk's 1x1 convs ran 2-10 % faster this way and
  // its 3x3 convs 2-6 % slower (their tap masks and more LDS traffic per MFMA), so the launcher
  // picks them for 1x1 convs (XM 1) and for unpadded convs of any size (XM 2: per-lane row
  // offsets, no tap masks -- the trunk's 3x3 convs read a zero-bordered copy of their input with
  // pad 0, engine.py, so they carry no masks either; with masks the 256 x 128 tile spilled).
  constexpr bool XC = XM != 0, XLIN = XM == 1;
  static_assert(!XC || (!PRO && !APL && NP == 2 && !ONE), "pixel-contiguous A: two-plane forms, no prologue");
  static_assert(XM != 2 || !DUAL, "dual GEMMs are 1x1 (XM 1)");
  constexpr int XC_OFF = RING;
  constexpr int MAIN = RING + (XC ? NW * 2048 : 0);
  constexpr int LDS_BYTES = MAIN > EPI ? MAIN : EPI;
  static_assert(STAGES == 2 || STAGES == 3, "stages");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];

  // wave index through readfirstlane: provably uniform, so the descriptors and LDS-DMA
  // destinations derived from it stay scalar (no waterfall loops around the buffer loads)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int L = xcd_remap(blockIdx.x, p.nwg);
  const int tile_m = L / p.tiles_n, tile_n = L % p.tiles_n;
  const int n0 = tile_n * BN;
  const int wrow0 = tile_m * BM + wave * WTM;

  // ---- A rows of this lane: wrow0 + 16 i + fr. The activation operand is read through buffer
  // descriptors based at the wave's first frame (shifted back by the padding, so every byte
  // offset is >= 0): rv[i] = the row's offset of tap (0,0) at channel 8 fg, the K-step's tap and
  // chunk offset is the wave-uniform soffset, and rows past M or taps in the padding read zeros
  // (an offset past the descriptor's range). No 64-bit address arithmetic per load.
  unsigned rv[TM];
  unsigned rv2[DUAL ? TM : 1];
  unsigned hmask[TM], wmask[TM];
  float sa[F16 ? TM : 1];                             // precision 3: per-row (= per-frame) scale
  // A wave's rows [wrow0, wrow0 + WTM) start in frame nf0 and, when a frame holds at least WTM
  // rows ("two"), reach at most into frame nf0 + 1 (rows >= nb): the frame of a row is one
  // compare, and the two frames' max|x| bounds are wave-uniform (scalar) loads.
  const int nf0 = wrow0 / p.HoWo;
  const int nb = (nf0 + 1) * p.HoWo;
  const bool two = p.HoWo >= WTM;
  float am0 = 0.f, am1 = 0.f;                         // max|x| of frames nf0, nf0 + 1 (F16)
  // PRO (precision 4 only): max|in_scale x + in_bias| <= max|x| pS + pB
  float pS = 1.f, pB = 0.f;
  if constexpr (F16 && PRO) prologue_bounds(p.in_scale, p.in_bias, p.Ci, pS, pB);
  auto bound = [&](float am) { return PRO ? fmaf(am, pS, pB) : am; };
  if constexpr (F16) {
    if (two) {
      if (wrow0 < p.M) am0 = bound(DUAL ? fmaxf(p.x_amax[nf0], p.x2_amax[nf0]) : p.x_amax[nf0]);
      if (nb < p.M) am1 = bound(DUAL ? fmaxf(p.x_amax[nf0 + 1], p.x2_amax[nf0 + 1]) : p.x_amax[nf0 + 1]);
    }
  }
  const __amdgpu_buffer_rsrc_t xr =
      buf_rsrc(p.x + ((int64_t)nf0 * p.xsn - (int64_t)p.pad * (p.xsh + p.xsw)), 0x7FFFFFF0);
  __amdgpu_buffer_rsrc_t x2r = xr;
  if constexpr (DUAL) x2r = buf_rsrc(p.x2 + (int64_t)nf0 * p.x2sn, 0x7FFFFFF0);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = wrow0 + i * 16 + fr;
    unsigned hm = 0, wmk = 0;
    unsigned v = BL_OOB, v2 = BL_OOB;
    if constexpr (F16) sa[i] = 1.f;
    if (m < p.M) {
      const int n = m / p.HoWo;
      if constexpr (F16) {
        // activation scale of this row's frame: max|x| < 2^e -> 2^(15 - e); a dual GEMM's two
        // inputs share one scale (their per-frame maxima combined)
        const float am = two ? (m >= nb ? am1 : am0)
                             : bound(DUAL ? fmaxf(p.x_amax[n], p.x2_amax[n]) : p.x_amax[n]);
        sa[i] = ldexpf(1.f, 15 - f16_scale_exp(am));
      }
      const int rem = m - n * p.HoWo;
      const int oh = rem / p.Wo;
      const int ow = rem - oh * p.Wo;
      const int ih = oh * p.stride - p.pad, iw = ow * p.stride - p.pad;
      v = (unsigned)(((int64_t)(n - nf0) * p.xsn + (int64_t)(ih + p.pad) * p.xsh + (int64_t)(iw + p.pad) * p.xsw +
                      fg * 8) * 4);
      if constexpr (DUAL)
        v2 = (unsigned)(((int64_t)(n - nf0) * p.x2sn + (int64_t)oh * p.x2sh + (int64_t)ow * p.x2sw + fg * 8) * 4);
      for (int t = 0; t < p.KH; ++t) hm |= (unsigned)((unsigned)(ih + t) < (unsigned)p.Hi) << t;
      for (int t = 0; t < p.KW; ++t) wmk |= (unsigned)((unsigned)(iw + t) < (unsigned)p.Wi) << t;
    }
    rv[i] = v;
    if constexpr (DUAL) rv2[i] = v2;
    hmask[i] = hm;
    wmask[i] = wmk;
  }
  // XC: the rows this lane loads are row 8 h + (lane >> 3) of row block i, chunk lane & 7. x is
  // dense and the conv 1x1 / stride 1 (the launcher's condition), so row m sits at m xsw floats:
  // one lane offset from a descriptor based at the wave's first row, the (i, h) row step in the
  // scalar offset, rows past M beyond the descriptor's range (zeros). x2 (a dual GEMM's strided
  // second input) keeps per-row offsets.
  __amdgpu_buffer_rsrc_t xlr = xr;
  unsigned xlv = 0;
  const int xsw4 = (int)(p.xsw * 4);
  if constexpr (XLIN) {
    const int64_t nrec = ((int64_t)(p.M - wrow0 - 1) * p.xsw + p.Ci) * 4;
    xlr = buf_rsrc(p.x + (int64_t)wrow0 * p.xsw, (int)(nrec < 0 ? 0 : nrec < 0x7FFFFFF0 ? nrec : 0x7FFFFFF0));
    xlv = (unsigned)(((lane >> 3) * (int)p.xsw + (lane & 7) * 4) * 4);
  }
  unsigned rv2c[XC && DUAL ? TM : 1][2];
  // XM 2: per-lane offsets of tap (0, 0) of those rows (the tap and chunk are the soffset)
  unsigned rvp[XM == 2 ? TM : 1][2];
  if constexpr (XM == 2) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = wrow0 + i * 16 + 8 * h + (lane >> 3);
        unsigned v = BL_OOB;
        if (m < p.M) {
          const int n = m / p.HoWo;
          const int rem = m - n * p.HoWo;
          const int oh = rem / p.Wo;
          const int ow = rem - oh * p.Wo;
          v = (unsigned)(((int64_t)(n - nf0) * p.xsn + (int64_t)oh * p.stride * p.xsh +
                          (int64_t)ow * p.stride * p.xsw + (lane & 7) * 4) * 4);
        }
        rvp[i][h] = v;
      }
  }
  if constexpr (XC && DUAL) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = wrow0 + i * 16 + 8 * h + (lane >> 3);
        unsigned v2 = BL_OOB;
        if (m < p.M) {
          const int n = m / p.HoWo;
          const int rem = m - n * p.HoWo;
          const int oh = rem / p.Wo;
          const int ow = rem - oh * p.Wo;
          v2 = (unsigned)(((int64_t)(n - nf0) * p.x2sn + (int64_t)oh * p.x2sh + (int64_t)ow * p.x2sw + (lane & 7) * 4) * 4);
        }
        rv2c[i][h] = v2;
      }
  }

  // ---- B pieces: piece j -> plane j / (BN/16), rows 16 (j % (BN/16)) .. +16; lane -> (row, slot),
  // through one descriptor per plane (the K-step's 64 B as soffset)
  const int wbytes = p.k_pad * 2 * (p.tiles_n * BN);
  const uint16_t* planes[3] = {F16 ? p.wh16 : p.whi, ONE ? p.wh16 : (F16 ? p.wl16 : p.wlo), p.wlo2};
  unsigned bvo[IB];
  int bdst[IB];
  int bq[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    int j = wave * IB + i;
    if (j >= NB_TOT) j -= NB_TOT;
    const int q = j / (BN / 16), rb = j % (BN / 16);
    const int nrow = rb * 16 + (lane >> 2);
    const int ch = (lane & 3) ^ swzF(nrow);
    bvo[i] = (unsigned)(((n0 + nrow) * p.k_pad + ch * 8) * 2);
    bdst[i] = (q * BN + rb * 16) * 64;
    bq[i] = q;                                          // wave-uniform
  }
  __amdgpu_buffer_rsrc_t wr[NSL];
#pragma unroll
  for (int q = 0; q < NSL; ++q) wr[q] = buf_rsrc(planes[q], wbytes);
  // kt: the iteration; ONE: slice q of its stage is K-step 2 kt + q of the hi plane
  auto issue_b = [&](int kt, int stage) {
    unsigned char* sb = lds + stage * B_STAGE;
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      __amdgpu_buffer_rsrc_t r = wr[0];
#pragma unroll
      for (int q = 1; q < NSL; ++q)
        if (bq[i] == q) r = wr[q];
      bl_lds16(r, sb + bdst[i], bvo[i], (ONE ? KS * kt + bq[i] : kt) * BK * 2);
    }
  };

  // ---- A walk (wave-uniform): k = ((ci/32)*KH*KW + kh*KW + kw)*32 + ci%32
  int u_kh = 0, u_kw = 0, u_ci = 0, u_step = 0;
  int u_off = 0;                                      // kh*xsh + kw*xsw + chunk*32 (elements)
  const int nk = p.nk;
  f4 raw[KS][TM][2];
  unsigned amask[KS];
  f4 as4[KS][2], ab4[KS][2];
  // the A operand of the walk's current K-step into sub-step slot ks, then advance the walk
  int u_cnt = 0;                                      // K-steps loaded so far (ONE: odd nk pads one)
  auto load_a = [&](int ks) {
    // ONE with odd nk: the last iteration's second step is a phantom (k >= K): zero A, so it adds
    // nothing whatever the B slice holds
    const bool phantom = ONE && u_cnt++ >= nk;
    if constexpr (PRO) {
      as4[ks][0] = *reinterpret_cast<const f4*>(p.in_scale + u_ci + fg * 8);
      as4[ks][1] = *reinterpret_cast<const f4*>(p.in_scale + u_ci + fg * 8 + 4);
      ab4[ks][0] = *reinterpret_cast<const f4*>(p.in_bias + u_ci + fg * 8);
      ab4[ks][1] = *reinterpret_cast<const f4*>(p.in_bias + u_ci + fg * 8 + 4);
    }
    amask[ks] = 0;
    const bool second = DUAL && u_step >= p.nk1;     // wave-uniform
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const bool ok = (hmask[i] >> u_kh) & (wmask[i] >> u_kw) & 1u;
      if constexpr (XC && DUAL) {
        if (second) {                                   // x2: 1x1, never padded
          const int so = (u_off - p.nk1 * BK) * 4;
          raw[ks][i][0] = bl_f4(x2r, rv2c[i][0], so);
          raw[ks][i][1] = bl_f4(x2r, rv2c[i][1], so);
        } else {
          raw[ks][i][0] = bl_f4(xlr, xlv, u_off * 4 + 16 * i * xsw4);
          raw[ks][i][1] = bl_f4(xlr, xlv, u_off * 4 + (16 * i + 8) * xsw4);
        }
      } else if constexpr (XLIN) {
        raw[ks][i][0] = bl_f4(xlr, xlv, u_off * 4 + 16 * i * xsw4);
        raw[ks][i][1] = bl_f4(xlr, xlv, u_off * 4 + (16 * i + 8) * xsw4);
      } else if constexpr (XM == 2) {
        raw[ks][i][0] = bl_f4(xr, rvp[i][0], u_off * 4);
        raw[ks][i][1] = bl_f4(xr, rvp[i][1], u_off * 4);
      } else if constexpr (DUAL) {
        if (second) {                                   // x2: 1x1, never padded
          const int so = (u_off - p.nk1 * BK) * 4;
          raw[ks][i][0] = bl_f4(x2r, rv2[i], so);
          raw[ks][i][1] = bl_f4(x2r, rv2[i] + 16, so);
        } else {
          raw[ks][i][0] = bl_f4(xr, rv[i], u_off * 4);
          raw[ks][i][1] = bl_f4(xr, rv[i] + 16, u_off * 4);
        }
      } else {
        const unsigned v = ok && !phantom ? rv[i] : BL_OOB;
        raw[ks][i][0] = bl_f4(xr, v, u_off * 4);
        raw[ks][i][1] = bl_f4(xr, v + 16, u_off * 4);
      }
      if constexpr (PRO) amask[ks] |= (unsigned)(ok && !phantom) << i;
    }
    // advance to the next K-step (kw, then kh, then the next chunk); stay on the last one
    if (++u_step < nk) {
      u_off += (int)p.xsw;
      if (++u_kw == p.KW) {
        u_kw = 0; u_off += (int)(p.xsh - (int64_t)p.KW * p.xsw);
        if (++u_kh == p.KH) { u_kh = 0; u_ci += BK; u_off += (int)(BK - (int64_t)p.KH * p.xsh); }
      }
    } else {
      u_step = nk - 1;
    }
  };

  frag_t af[NP][TM];                                  // planes, or (ONE) K sub-steps
  auto split_a = [&]() {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
     for (int ks = 0; ks < KS; ++ks) {
      f4 v0 = raw[ks][i][0], v1 = raw[ks][i][1];
      if constexpr (XC) {
        // transpose through this wave's slot (chunk slots XOR-swizzled by row: the b128 reads of
        // 8 lanes / 8 rows hit 8 distinct bank quads); same-wave LDS ops complete in order
        unsigned char* const scr = lds + XC_OFF + wave * 2048;
        const int q0 = lane >> 3, c = lane & 7;
        *reinterpret_cast<f4*>(scr + q0 * 128 + ((c ^ q0) << 4)) = v0;
        *reinterpret_cast<f4*>(scr + (8 + q0) * 128 + ((c ^ q0) << 4)) = v1;
        v0 = *reinterpret_cast<const f4*>(scr + fr * 128 + (((2 * fg) ^ (fr & 7)) << 4));
        v1 = *reinterpret_cast<const f4*>(scr + fr * 128 + (((2 * fg + 1) ^ (fr & 7)) << 4));
      }
      if constexpr (PRO) {
        if constexpr (ONE) {                          // (as conv_halo.hip's precision-4 prologue)
          v0 = affine4(v0, as4[ks][0], ab4[ks][0]);
          v1 = affine4(v1, as4[ks][1], ab4[ks][1]);
        } else {
          v0 = v0 * as4[ks][0] + ab4[ks][0];
          v1 = v1 * as4[ks][1] + ab4[ks][1];
        }
        if (!((amask[ks] >> i) & 1u)) { v0 = f4{0.f, 0.f, 0.f, 0.f}; v1 = v0; }   // padding stays 0
      }
      if constexpr (APL) {
        af[0][i] = __builtin_bit_cast(bf16x8, v0);
        af[1][i] = __builtin_bit_cast(bf16x8, v1);
      } else if constexpr (ONE) {
        af[ks][i] = cvt_f16_one(v0, v1, sa[i]);
      } else if constexpr (F16) {
        unsigned long long p0[2], p1[2];
        // XM 2 (launched only when a frame holds >= WTM rows: "two") takes the row's scale from the
        // two frames' wave-uniform scales instead of a register per row: the 256 x 128 tile sits
        // at its 128-VGPR cap and the per-lane offsets of XM 2 needed those registers
        float s_i = sa[i];
        if constexpr (XM == 2)
          s_i = wrow0 + i * 16 + fr >= nb ? ldexpf(1.f, 15 - f16_scale_exp(am1)) : ldexpf(1.f, 15 - f16_scale_exp(am0));
        split_planes_f16(v0, s_i, p0);
        split_planes_f16(v1, s_i, p1);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
          af[q][i] = __builtin_bit_cast(f16x8, u64x2{p0[q], p1[q]});
        }
      } else {
        bf16x4 p0[NP], p1[NP];
        split_planes<NP>(v0, p0);
        split_planes<NP>(v1, p1);
#pragma unroll
        for (int q = 0; q < NP; ++q)
          af[q][i] = bf16x8{p0[q][0], p0[q][1], p0[q][2], p0[q][3], p1[q][0], p1[q][1], p1[q][2], p1[q][3]};
      }
     }
     if constexpr (XC) __builtin_amdgcn_sched_barrier(0);   // one row block's transpose live at a time
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) {
    const unsigned char* sb = lds + stage * B_STAGE;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nrow = j * 16 + fr;
      const unsigned char* bp = sb + nrow * 64 + ((fg ^ swzF(nrow)) << 4);
      frag_t bfr[NSL];
#pragma unroll
      for (int q = 0; q < NSL; ++q) bfr[q] = *reinterpret_cast<const frag_t*>(bp + q * BN * 64);
      // partial products smallest first; terms with plane-index sum >= NP are dropped
      if constexpr (ONE) {                            // K-step KS kt, then KS kt + 1
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) acc[i][j] = mfma16(af[ks][i], bfr[ks], acc[i][j]);
        continue;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int s = NP - 1; s >= 0; --s)
#pragma unroll
          for (int qa = s; qa >= 0; --qa)
            acc[i][j] = mfma16(af[qa][i], bfr[s - qa], acc[i][j]);
    }
  };

  // ---------------- main loop (nit iterations of KS K-steps)
  const int nit = (nk + KS - 1) / KS;
  auto load_it = [&]() {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) load_a(ks);
  };
  load_it();
  issue_b(0, 0);
  if constexpr (STAGES == 3) issue_b(nit > 1 ? 1 : 0, 1);
  split_a();
  // planes input: the A fragments of step 0 ARE the load destinations (no split), so the
  // compiler's wait bookkeeping would carry their pending loads into the loop header and merge
  // them into a vmcnt(0) before every K-step's first MFMA (tools/loop_waits.py) -- i.e. every
  // step would wait for the A(kt+1) loads and B DMA it had just issued. Retiring the prologue
  // loads here with a wait the compiler can see costs one latency per block, and the loop keeps
  // its overlap (STAGES 2 waits for them at the loop top anyway).
  if constexpr (APL) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  int st = 0;
  for (int kt = 0; kt < nit; ++kt) {
    // B(kt) of this wave: at most the (STAGES-2)*IB pieces issued after it are still pending
    wait_barrier<(STAGES - 2) * IB>();
    load_it();
    {
      const int ks = kt + STAGES - 1 < nit ? kt + STAGES - 1 : nit - 1;
      const int sn = st == 0 ? STAGES - 1 : st - 1;   // the stage read at kt-1
      issue_b(ks, sn);
    }
    compute(st);
    split_a();
    st = st + 1 == STAGES ? 0 : st + 1;
  }
  wait_barrier<0>();   // every LDS-DMA landed and every fragment read retired: LDS is free

  // ---------------- epilogue: per-wave 16-row slices, whole-row 16-B vectors
  float* ct = reinterpret_cast<float*>(lds) + wave * 16 * CS;
  constexpr int CPR = BN / 4;                         // float4 chunks per row
  constexpr int RPP = 64 / CPR;                       // rows per pass
  constexpr int EB = 16 / RPP;                        // passes per 16-row slice
  const int cc = lane % CPR, rr0 = lane / CPR;
  const int col = n0 + cc * 4;
  const bool cval = col < p.Co;
  f4 sc4 = {1.f, 1.f, 1.f, 1.f}, bi4 = {0.f, 0.f, 0.f, 0.f}, sl4 = {0.f, 0.f, 0.f, 0.f};
  if (cval) {
    if (p.scale) sc4 = *reinterpret_cast<const f4*>(p.scale + col);
    if (p.bias) bi4 = *reinterpret_cast<const f4*>(p.bias + col);
    if (p.slope) sl4 = *reinterpret_cast<const f4*>(p.slope + col);
  }
  // per-frame max|y| (p.y_amax): with "two" a running maximum per frame (nf0, nf0 + 1) and
  // one wave reduction each at the end; else per-lane frame tracking (FrameMax)
  const bool track = F16 || p.y_amax;
  float ym0 = 0.f, ym1 = 0.f;
  FrameMax ymax;
  float inv0 = 1.f, inv1 = 1.f;                       // 2^(e - 15) of frames nf0, nf0 + 1: exact
  if constexpr (F16) {
    inv0 = ldexpf(1.f, f16_scale_exp(am0) - 15);
    inv1 = ldexpf(1.f, f16_scale_exp(am1) - 15);
  }
  auto frame_of = [&](int m) { return two ? nf0 + (m >= nb) : m / p.HoWo; };
  auto offs = [&](int m, int64_t& yo, int64_t& ro) {
    if (p.ylin && p.rlin) {
      yo = (int64_t)m * p.ysw + col;
      ro = (int64_t)m * p.rsw + col;
      return;
    }
    const int n = m / p.HoWo;
    const int rem = m - n * p.HoWo;
    const int oh = rem / p.Wo;
    const int ow = rem - oh * p.Wo;
    yo = (int64_t)n * p.ysn + (int64_t)oh * p.ysh + (int64_t)ow * p.ysw + col;
    ro = (int64_t)n * p.rsn + (int64_t)oh * p.rsh + (int64_t)ow * p.rsw + col;
  };
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < TN; ++j) ct[(fg * 4 + r) * CS + j * 16 + fr] = acc[i][j][r];
    int64_t yo[EB];
    f4 res[EB];
    bool ok[EB];
    int fn[EB];                                       // frame of the row (max|y| slots, F16 scale)
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int m = wrow0 + i * 16 + rr0 + RPP * e;
      ok[e] = cval && m < p.M;
      res[e] = f4{0.f, 0.f, 0.f, 0.f};
      yo[e] = 0;
      fn[e] = 0;
      if (ok[e]) {
        int64_t ro;
        offs(m, yo[e], ro);
        // residual convs (the trunk's conv3s): non-temporal residual loads and output stores (last
        // use / not re-read here: the A panel re-read per column tile keeps its L2 lines), +0.35 %
        // bench; for the other convs NT stores cost the YOLO net ~1 % (its next layer re-reads
        // the output from the caches), profiles/r05_nt_epilogue_ab.txt
        if (p.res_mode != PRPE_RES_NONE) res[e] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p.r + ro));
        if (track) fn[e] = frame_of(m);
      }
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      f4 v = *reinterpret_cast<const f4*>(ct + (rr0 + RPP * e) * CS + cc * 4);
      if (!ok[e]) continue;
      if constexpr (F16) {
        if (two) {
          v = v * (fn[e] == nf0 ? inv0 : inv1);
        } else {                                      // frames smaller than a wave tile
          const float am = bound(DUAL ? fmaxf(p.x_amax[fn[e]], p.x2_amax[fn[e]]) : p.x_amax[fn[e]]);
          v = v * ldexpf(1.f, f16_scale_exp(am) - 15);
        }
      }
      v = v * sc4 + bi4;
      if (p.res_mode == PRPE_RES_PRE_ACT) v += res[e];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = apply_act(v[q], p.act, sl4[q]);
      if (p.res_mode == PRPE_RES_POST_ACT) v += res[e];
      if (p.y_planes) {
        // planes format: channel group g = c / 8 of a pixel holds hi[8] then lo[8] (bf16)
        bf16x4 pl[2];
        split_planes<2>(v, pl);
        uint16_t* y16 = reinterpret_cast<uint16_t*>(p.y) + 2 * (yo[e] - col) + (col >> 3) * 16 + (col & 7);
        *reinterpret_cast<bf16x4*>(y16) = pl[0];
        *reinterpret_cast<bf16x4*>(y16 + 8) = pl[1];
      } else {
        if (p.res_mode != PRPE_RES_NONE) __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p.y + yo[e]));
        else *reinterpret_cast<f4*>(p.y + yo[e]) = v;
      }
      if (p.y_amax) {
        const float a = amax4(v);
        if (two) {
          ym0 = fmaxf(ym0, fn[e] == nf0 ? a : 0.f);
          ym1 = fmaxf(ym1, fn[e] == nf0 ? 0.f : a);
        } else {
          ymax.add(p.y_amax, fn[e], a);
        }
      }
    }
  }
  if (p.y_amax) {
    if (two) {
      if (wrow0 < p.M) amax_commit(p.y_amax + nf0, ym0);
      if (nb < p.M) amax_commit(p.y_amax + nf0 + 1, ym1);
    } else {
      frame_amax_final(p.y_amax, ymax);
    }
  }
}

template <int NW, int TM, int TN, int NP, int STAGES, bool F16 = false, bool ONE = false, int KSF = 0>
int launch(const ConvK& kp0, hipStream_t st) {
  constexpr int BM = NW * TM * 16, BN = TN * 16;
  ConvK kp = kp0;
  const int tiles_m = (kp.M + BM - 1) / BM;
  kp.tiles_n = (kp.Co + BN - 1) / BN;
  kp.nwg = tiles_m * kp.tiles_n;
  if constexpr (ONE) {
    if (kp.x2 || kp.x_planes) return PRPE_EINVAL;
    if (kp.in_scale)
      hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, true, true, false, false, true, KSF>), dim3(kp.nwg),
                         dim3(NW * 64), 0, st, kp);
    else
      hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, false, true, false, false, true, KSF>), dim3(kp.nwg),
                         dim3(NW * 64), 0, st, kp);
    return launch_status();
  }
  // the pixel-contiguous A loads (two planes only): XM 1 for 1x1 / stride-1 convs over a dense
  // x (linear row addressing), XM 2 for any other unpadded conv (per-lane row offsets)
  const bool x11 = NP == 2 && kp.KH == 1 && kp.KW == 1 && kp.pad == 0 && kp.stride == 1 &&
                   kp.xsh == (int64_t)kp.Wi * kp.xsw && kp.xsn == (int64_t)kp.Hi * kp.xsh && kp.xsw >= kp.Ci;
  const bool xp0 = NP == 2 && kp.pad == 0 && !x11 && kp.Ho * kp.Wo >= TM * 16;
  if (kp.x2) {
    // (not the dual precision-3 256 x 128 tile: its x2 row offsets stay per lane and spilled it)
    constexpr bool dual_x11 = !(NW == 8 && TM == 2 && TN == 8 && STAGES == 3);
    if constexpr (F16) {
      if (x11 && dual_x11)
        hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, false, true, true, false, false, 0, dual_x11 ? 1 : 0>),
                           dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
      else
        hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, false, true, true>), dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
    } else {
      hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, NP, STAGES, false, false, true>), dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
    }
    return launch_status();
  }
  if (kp.x_planes) {
    if constexpr (F16 || NP != 2) return PRPE_EINVAL;
    else hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, false, false, false, true>), dim3(kp.nwg),
                            dim3(NW * 64), 0, st, kp);
    return launch_status();
  }
  if constexpr (F16) {
    if (x11)
      hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, false, true, false, false, false, 0, 1>),
                         dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
    else if (xp0)
      hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, false, true, false, false, false, 0, 2>),
                         dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
    else
      hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, false, true>), dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
  } else if (kp.in_scale)
    hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, NP, STAGES, true>), dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
  else if constexpr (NP == 2) {
    if (x11)
      hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, false, false, false, false, false, 0, 1>),
                         dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
    else if (xp0)
      hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, false, false, false, false, false, 0, 2>),
                         dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
    else
      hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, 2, STAGES, false>), dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
  } else {
    hipLaunchKernelGGL((conv_wave_kernel<NW, TM, TN, NP, STAGES, false>), dim3(kp.nwg), dim3(NW * 64), 0, st, kp);
  }
  return launch_status();
}

}  // namespace

bool conv_wave_eligible(const ConvK& kp, int prec, int km) {
  // chunk-major K walk (km 2, or any 1x1 on the vector path with whole 32-channel chunks),
  // vectorised epilogue, precision 0 / 2 / 3, K in whole K-steps, B rows readable up to a
  // multiple of 128; precision 3 also needs its fp16 planes and the input's max bound and
  // has no prologue
  const bool chunked = km == 2 || (km == 1 && kp.KH * kp.KW == 1 && kp.Ci % 32 == 0);
  const bool p3 = prec == 3 && kp.wh16 && kp.wl16 && kp.x_amax && !kp.in_scale && (!kp.x2 || kp.x2_amax);
  const bool p4 = prec == 4 && kp.wh16 && kp.x_amax && !kp.x2 && (!kp.in_scale || kp.in_bias);
  const bool planes_ok = !kp.x_planes || (prec == 0 && !kp.in_scale && !kp.x2);
  // buffer descriptors: a wave's rows (at most 64, spanning at most 64 / HoWo + 2 frames) and its
  // taps must lie within 2^31 bytes of the wave's first frame, with non-negative strides
  const int64_t span_f = 64 / kp.HoWo + 2;
  const int64_t x_span = (span_f * kp.xsn + (int64_t)(kp.KH + kp.pad) * kp.xsh + (int64_t)(kp.KW + kp.pad) * kp.xsw +
                          kp.Ci) * 4;
  const int64_t x2_span = kp.x2 ? (span_f * kp.x2sn + (int64_t)kp.Ho * kp.x2sh + (int64_t)kp.Wo * kp.x2sw + 64) * 4 : 0;
  const bool addr_ok = kp.xsn >= 0 && kp.xsh >= 0 && kp.xsw >= 0 && x_span < 0x7FFFFFF0LL &&
                       (!kp.x2 || (kp.x2sn >= 0 && kp.x2sh >= 0 && kp.x2sw >= 0 && x2_span < 0x7FFFFFF0LL)) &&
                       (int64_t)kp.k_pad * 2 * kp.Co < (1LL << 30);
  return chunked && kp.vec_out && (prec == 0 || prec == 2 || p3 || p4) && kp.K % BK == 0 && kp.k_pad == kp.K &&
         kp.zero != nullptr && planes_ok && addr_ok;
}

// tile 20 = auto; 21.. force a configuration (tools/conv_bench.py sweeps them)
int conv_wave_launch(const ConvK& kp, int prec, int tile, hipStream_t st) {
  if (tile == 20) {
    // measured (tools/conv_bench.py, profiles/r01_conv_bench_wave.txt, r01_conv_bench_tiles_v3.txt,
    // r01_conv_bench_stages.txt): 32x128 waves in 4-wave 128x128 blocks with a 2-stage B ring
    // (32 KB ring + 33 KB epilogue slab: 4 blocks = 4 waves/SIMD instead of 3 with 3 stages;
    // the A operand's one-K-step register lookahead then meets its L2 latency: adapters' 3x3
    // -8..10 %, YOLO adapter 1x1 -12 %, ViT fc1 -4 % in isolation, +0.2..0.4 % on the
    // concurrent-heads bench), short-K or narrow precision-3 convs the 256x64 tile
    // PRPE_WAVE_WIDE=<tile> in the environment overrides the wide-shape choice (A/B runs)
    static const int wide = [] {
      const char* e = getenv("PRPE_WAVE_WIDE");
      return e ? atoi(e) : 28;
    }();
    // precision 3: Co <= 64 on the 256 x 64 tile (25); Co > 64 on the wide tile at any K: the
    // short-K residual GEMMs of the trunk (conv3 + residual, K = 64 / 128 / dual 128) run 16-19 %
    // faster on it than on the 256 x 64 tile at bs = 256 (profiles/r01_conv_bench_sweep_v4.txt;
    // bench +1.2 %). (The round-1/2 A/B switches of both choices were removed in round 6.)
    // precision 3, Co > 64: the 256 x 128 8-wave tile (wave 32 x 128, 3-stage ring) since round 4:
    // trunk convs 68.6 -> 66.1 ms at bs = 256 against the 128 x 128 2-stage tile, every unfused
    // trunk conv faster (profiles/r04_layer_profile_trunk_wide3_sweep.txt; round 2 had measured the
    // opposite, before the buffer-descriptor addressing of round 3)
    static const int wide3 = [] {
      const char* e = getenv("PRPE_WAVE_WIDE3");
      return e ? atoi(e) : 23;
    }();
    // PRPE_WAVE_P4=<26|27> overrides the precision-4 choice for Co > 64 (A/B runs)
    static const int wide4 = [] {
      const char* e = getenv("PRPE_WAVE_P4");
      return e && atoi(e) == 26 ? 26 : 27;
    }();
    static const int tile2 = [] {
      const char* e = getenv("PRPE_WAVE_P2");
      return e ? atoi(e) : 27;
    }();
    if (prec == 0) tile = wide;
    else if (prec == 3) tile = kp.Co > 64 ? wide3 : 25;
    else if (prec == 4) tile = kp.Co > 64 ? wide4 : 25;  // (the precision-3 overrides do not apply)
    else tile = kp.Co > 64 && kp.K > 128 ? tile2 : 24;
  }
  if (prec == 0) {
    switch (tile) {
      case 21: return launch<8, 4, 8, 2, 3>(kp, st);   // 512 x 128, wave 64 x 128
      case 22: return launch<8, 4, 4, 2, 3>(kp, st);   // 512 x 64,  wave 64 x 64
      case 23: return launch<8, 2, 8, 2, 3>(kp, st);   // 256 x 128, wave 32 x 128
      case 24: return launch<4, 4, 8, 2, 3>(kp, st);   // 256 x 128, wave 64 x 128, 4 waves
      case 25: return launch<8, 4, 8, 2, 2>(kp, st);   // 512 x 128, 2 stages
      case 26: return launch<4, 2, 8, 2, 3>(kp, st);   // 128 x 128, wave 32 x 128, 4 waves
      case 27: return launch<2, 4, 8, 2, 3>(kp, st);   // 128 x 128, wave 64 x 128, 2 waves
      case 28: return launch<4, 2, 8, 2, 2>(kp, st);   // 128 x 128, wave 32 x 128, 2 stages
      case 29: return launch<4, 4, 8, 2, 2>(kp, st);   // 256 x 128, wave 64 x 128, 2 stages
      default: return PRPE_EINVAL;
    }
  }
  if (prec == 3) {
    switch (tile) {
      case 21: return launch<8, 4, 8, 2, 3, true>(kp, st);
      case 22: return launch<8, 4, 4, 2, 3, true>(kp, st);
      case 23: return launch<8, 2, 8, 2, 3, true>(kp, st);
      case 24: return launch<4, 4, 8, 2, 3, true>(kp, st);
      case 25: return launch<8, 2, 4, 2, 3, true>(kp, st);   // 256 x 64, wave 32 x 64
      case 26: return launch<4, 2, 8, 2, 3, true>(kp, st);   // 128 x 128, wave 32 x 128, 4 waves
      case 27: return launch<4, 2, 8, 2, 2, true>(kp, st);   // 128 x 128, 2 stages
      default: return PRPE_EINVAL;
    }
  }
  if (prec == 4) {                                     // the precision-3 shapes, one fp16 plane
    // (no 256 x 128 / 64 x 128-wave tile: at two K-steps per iteration it spills)
    switch (tile) {
      case 24: return launch<4, 2, 4, 2, 3, true, true>(kp, st);   // 128 x 64, wave 32 x 64
      case 25: return launch<8, 2, 4, 2, 3, true, true>(kp, st);   // 256 x 64, wave 32 x 64
      case 26: return launch<4, 2, 8, 2, 3, true, true>(kp, st);   // 128 x 128, 3 stages
      case 27: return launch<4, 2, 8, 2, 2, true, true>(kp, st);   // 128 x 128, 2 stages
      case 28: return launch<4, 2, 8, 2, 2, true, true, 1>(kp, st);   // 27 at one K-step per iteration
      case 29: return launch<4, 1, 8, 2, 2, true, true>(kp, st);   // 64 x 128, wave 16 x 128
      default: return PRPE_EINVAL;
    }
  }
  switch (tile) {
    case 21: return launch<4, 2, 8, 3, 3>(kp, st);   // 128 x 128, wave 32 x 128, 4 waves
    case 22: return launch<8, 4, 4, 3, 3>(kp, st);   // 512 x 64,  wave 64 x 64
    case 23: return launch<8, 2, 8, 3, 3>(kp, st);   // 256 x 128, wave 32 x 128
    case 24: return launch<8, 2, 4, 3, 3>(kp, st);   // 256 x 64,  wave 32 x 64
    case 25: return launch<8, 2, 8, 3, 2>(kp, st);   // 256 x 128, 2 stages
    case 26: return launch<4, 2, 8, 3, 3>(kp, st);   // = 21 (128 x 128, 4 waves)
    case 27: return launch<4, 2, 8, 3, 2>(kp, st);   // 128 x 128, 4 waves, 2 stages
    default: return PRPE_EINVAL;
  }
}

}  // namespace prpe_k
