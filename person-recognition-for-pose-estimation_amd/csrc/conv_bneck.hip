// Fused ResNet-50 bottleneck with identity shortcut (torchvision Bottleneck.forward, v1.5; the
// reference's trunk, training/modify_models.py:413-446):
//   y = relu(bn3(conv3(relu(bn2(conv2_3x3(relu(bn1(conv1(x)))))))) + x)
// in ONE kernel per 8 x 16 output-pixel tile, precision 3 (two fp16 planes, three MFMA terms).
//
// Why: layer1's identity blocks run as three HBM-bound launches (conv1 reads the 256-channel
// block input, 6.7 GB at bs = 256, writes t1; conv2 reads t1 with its halo and writes t2; conv3
// reads t2 AND the block input again as the residual and writes y: ~27 GB per block, 7.0 ms,
// profiles/r03_layer_profile_bufaddr.txt). Here t1 and t2 live only in LDS, the block input is
// read once (plus the 3x3 halo, mostly L2) and y written once: ~14 GB.
//
// Phases of one workgroup (8 waves):
//   1. t1 = relu(bn1(W1 x)) on the tile's 10 x 18 haloed pixels (12 row blocks of 16), A straight
//      from global (buffer loads; pixels outside the image read zeros and their t1 is forced to
//      0 = conv2's zero padding), split into fp16 planes with the frame's scale (x_amax[n], as
//      the unfused conv1), W1 through an LDS-DMA ring. t1 is then written to LDS as fp16 planes
//      of t1 * s1 with ONE scale per tile, s1 = 2^(15 - e), max|t1 over the tile| < 2^e (a
//      block-wide max): t1's operand rounding depends only on this tile of this frame, so frames
//      stay independent of their batch-mates.
//   2. t2 = relu(bn2(conv2(t1))): conv_halo.hip's K-loop (9 taps x 2 chunks) on the LDS tile,
//      planes read without a split; t2 -> LDS as fp16 planes with the tile's scale s2.
//   3. y = relu(bn3(W3 t2) + x): W3 in two 128-column halves through LDS, residual read from
//      global, y written from the MFMA accumulator layout, per-frame max|y| raised (y_amax).
// Every MFMA is issued transposed (weights as the A operand, pixels as B), so a lane's
// accumulator holds 4 consecutive channels of one pixel: the epilogues write t1 / t2 planes with
// two 8-B LDS stores per 4 channels and read the residual / store y as 16-B buffer accesses.
// Epilogue arithmetic as conv_wave.hip (scale16 carries the weights' 2^-e, the activation
// scale is removed exactly); only t1 / t2 are rounded with per-tile instead of per-frame
// scales, so results agree with the unfused launches to the precision-3 operand error
// (tests/test_gpu_ops.py: vs fp64 and vs the unfused path).
//
// LDS (80 KB, two workgroups per CU): TT [2 chunks][192 px][128 B] (t1, then t2 in its first
// 32 KB), the swizzled planes layout of conv_halo.hip (slot s of pixel q at s ^ swz_halo(column), t2 at
// s ^ swz_rows(q): conv.h);
// the W1 / W2 ring [4 stages][2 planes][64 rows][64 B] right after it (three K-steps of
// lookahead; the block A operand of phase 1 is loaded two K-steps ahead into registers); phase
// 3's W3 half [2 K-steps][2 planes][128 rows][64 B] overlays TT's last 16 KB and ring stages 0-1.
#include "conv.h"

namespace prpe_k {

struct BneckK {
  const float* x; int64_t xsn, xsh, xsw; const float* x_amax;
  float* y; int64_t ysn, ysh, ysw; float* y_amax;
  int N, H, W;
  const uint16_t* wh[3]; const uint16_t* wl[3];
  int kp[3];
  const float* sc[3]; const float* bi[3];
  int tiles_w, tiles_h, nwg;
  int mid;                                               // 64 or 128 (BShape)
  int proj;                                              // x has mid channels (layer1.0, see BShape)
};

namespace {

constexpr int BK_ = 32;
constexpr int TC = 16;                                   // tile columns (one 16-pixel row block per wave)
constexpr int HW_ = TC + 2;                              // 18 haloed columns
constexpr int W3_PART = 32 * 1024;                       // one W3 part (below) in the overlay
constexpr int RING = 4;                                  // W1 / W2 ring stages (3 K-steps of lookahead)

// Block shape. MID = the inner width (64: layer1, 128: layer2), CIO = 4 MID output channels.
// Identity (layer1.1-2, layer2.1-3): x has CIO channels and is the residual; conv3 (K = MID)
// runs in parts of R3 output columns. Projection (PROJ, layer1.0): x has MID channels, conv3 and
// the downsample projection are one dual GEMM over [t2 | x] (the engine's pk_dual pack, K = 2 MID,
// W' = [s3 W3 | sd Wd]), run in four parts of 64 columns; no residual read.
// LDS: TT (t1, then t2 in its first (MID/32) CHB2 bytes), then the W1 / W2 ring; a W3 part
// overlays TT past t2 (and, at MID 64, ring stages 0-1). MID 64: 48 + 32 = 80 KB, two
// workgroups per CU; MID 128: 96 + 64 = 160 KB, one.
// TRT = output rows of the tile = waves of the workgroup (8: 8 x 16 pixels, 8 waves; 16 (MID 64
// only, round 5): 16 x 16 pixels, 16 waves, one workgroup per CU -- every weight byte staged
// into LDS serves twice the pixels, and the 3x3 halo is 1.27x the tile instead of 1.41x).
template <int MIDT, bool PROJ, int TRT = 8> struct BShape {
  static constexpr int MID = MIDT, CIO = 4 * MIDT;
  static constexpr int TR = TRT, NW = TRT;
  static constexpr int HP = (TR + 2) * HW_;               // 180 / 324 haloed pixels
  static constexpr int NRB1 = (HP + 15) / 16;             // 12 / 21 row blocks of haloed pixels
  static constexpr int CHB1 = NRB1 * 16 * 128;            // bytes of one 32-channel chunk of t1
  static constexpr int CHB2 = TR * TC * 128;              // ... of t2
  static constexpr int CIN = PROJ ? MID : CIO;           // x channels
  static constexpr int NK1 = CIN / BK_;                  // phase-1 K-steps
  // phase-1 A (x) lookahead in K-steps, in registers: 2 where four waves per SIMD cap VGPRs at
  // 128 (inner width 64), 4 at one 8-wave workgroup per CU (inner width 128, 16 K-steps)
  static constexpr int AD = MIDT > 64 ? 4 : 2;
  static constexpr int NKS3 = PROJ ? 2 * MID / BK_ : MID / BK_;   // phase-3 K-steps
  static constexpr int R3 = PROJ || MID > 64 ? 64 : 128; // output columns per phase-3 part
  static constexpr int NPART = CIO / R3;
  static constexpr int W3_STEP = 2 * R3 * 64;            // one K-step of a part (both planes)
  static constexpr int TT_BYTES = (MID / 32) * CHB1;
  static constexpr int STAGE = 2 * MID * 64;             // one K-step of W1 / W2 (both planes)
  // its LDS-DMA pieces per wave: whole 1-KiB pieces (16 weight rows x 64 B), or -- 16 waves on
  // an 8-KiB stage -- ONE half piece per wave (lanes 0-31, 8 rows): every wave issues the same
  // number of DMA instructions per K-step, so the counted waits below are the same for all
  static constexpr bool HALF = STAGE / 1024 < NW;
  static constexpr int PPW = HALF ? 1 : STAGE / 1024 / NW;
  static constexpr int PROWS = HALF ? 8 : 16;            // weight rows per piece
  static constexpr int PW3 = 32 / NW;                    // W3 pieces (1 KiB) per wave and part
  static constexpr int RING_OFF = TT_BYTES;
  static constexpr int W3_OFF = (MID / 32) * CHB2;       // after t2
  static constexpr int LDS_BYTES = TT_BYTES + RING * STAGE;
  static constexpr int WPC = LDS_BYTES <= 80 * 1024 ? 2 : 1;   // workgroups per CU
  // two W3 part buffers when the free LDS of phase 3 holds them (MID 128: TT past t2 + ring
  // stages 0-1): part h + 1 is then DMA'd under part h's MFMAs instead of after them
  static constexpr bool W3DB = W3_OFF + 2 * W3_PART <= RING_OFF + 2 * STAGE;
  static_assert(!PROJ || MID == 64, "projection block: layer1.0 only");
  static_assert(PPW >= 1 && STAGE == PPW * NW * PROWS * 64, "W ring pieces");
  static_assert(NKS3 * W3_STEP == W3_PART, "W3 part size");
  static_assert(NKS3 * 2 * (R3 / 16) == PW3 * NW && PW3 >= 1, "whole W3 pieces per wave and part");
  static_assert(TR == 8 || (TR == 16 && MID == 64), "16-row tile: inner width 64 only (LDS)");
  static_assert(W3_OFF + W3_PART <= RING_OFF + 2 * STAGE, "W3 part overlay below ring stage 2");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// the fp16 planes (4 x f16 each) of channels c0..c0+3 (c0 % 4 == 0, one 8-channel group) of
// pixel q into the planes layout: two 8-B LDS writes
// (sw: the pixel's slot swizzle -- swz_halo of its column for t1, swz_rows for t2)
__device__ __forceinline__ void put_planes4(unsigned char* base, int chb, int q, int sw, int c0,
                                            unsigned long long (&pl)[2]) {
  const int g = (c0 & 31) >> 3;
  unsigned char* pq = base + (c0 >> 5) * chb + q * 128 + (c0 & 7) * 2;
  *reinterpret_cast<unsigned long long*>(pq + (((2 * g) ^ sw) << 4)) = pl[0];
  *reinterpret_cast<unsigned long long*>(pq + (((2 * g + 1) ^ sw) << 4)) = pl[1];
}

// 16 B per lane out through a buffer descriptor (offsets past num_records are dropped)
__device__ __forceinline__ void bs_f4(__amdgpu_buffer_rsrc_t r, f4 v, unsigned voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, voff, soff, 0);
}

// gfx950 store-data hazard: a 128-bit buffer store reads its data VGPRs after
// it issues, and a VALU / MFMA write of them in the very next instruction replaces the data
// (round 4's reverted 8308d2f wrote garbage so). LLVM's hazard model exempts stores whose soffset
// is an SGPR, so nothing stops the scheduler from emitting that; this keeps v's registers live
// through an `s_nop 1` ordered after the store (a side-effecting asm stays behind the store), two
// wait states before any reuse. tools/barrier_hoist_check.py check 3 guards every kernel.
__device__ __forceinline__ void store_data_guard(f4 v) {
  asm volatile("s_nop 1" ::"v"(__builtin_bit_cast(v4u, v)));
}

// B fragments of column block j from a [2 planes][rows][64 B] stage (conv_wave's slot swizzle)
__device__ __forceinline__ void b_frags(const unsigned char* sb, int rows, int j, int fr, int fg, f16x8 (&b)[2]) {
  const int nrow = j * 16 + fr;
  const unsigned char* bp = sb + nrow * 64 + ((fg ^ swzF(nrow)) << 4);
  b[0] = *reinterpret_cast<const f16x8*>(bp);
  b[1] = *reinterpret_cast<const f16x8*>(bp + rows * 64);
}

// the three partial products of the split, smallest first (conv_wave.hip's order), computed
// transposed: the weight fragment is the MFMA's A operand and the activation fragment its B, so
// a lane's accumulator holds 4 consecutive CHANNELS of one pixel (16-B epilogue accesses)
__device__ __forceinline__ f32x4 mfma3t(const f16x8 (&w)[2], const f16x8 (&a)[2], f32x4 c) {
  c = mfma16(w[0], a[1], c);
  c = mfma16(w[1], a[0], c);
  c = mfma16(w[0], a[0], c);
  return c;
}

// launch bound: HIP's second argument is waves per SIMD, so WPC workgroups of NW waves per CU =
// WPC * NW / 4 (caps VGPRs at 128 for the 80-KB shapes; measured neutral, tools/run_r03ac.sh)
template <int MIDT, bool PROJ, int TRT>
__global__ __launch_bounds__(TRT * 64, (BShape<MIDT, PROJ, TRT>::WPC * TRT / 4)) void bneck_kernel(BneckK p) {
  using S = BShape<MIDT, PROJ, TRT>;
  constexpr int MID = S::MID, CIO = S::CIO, CIN = S::CIN, NK1 = S::NK1, R3 = S::R3, W3_STEP = S::W3_STEP;
  constexpr int STAGE = S::STAGE, PPW = S::PPW, RING_OFF = S::RING_OFF, W3_OFF = S::W3_OFF;
  constexpr int TR = S::TR, NW = S::NW, HP = S::HP, NRB1 = S::NRB1, CHB1 = S::CHB1, CHB2 = S::CHB2;
  constexpr int PROWS = S::PROWS, PW3 = S::PW3;
  constexpr int NJ1 = MID / 16;                              // 16-channel column blocks of t1 / t2
  __shared__ __attribute__((aligned(1024))) unsigned char lds[S::LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  int L = xcd_remap(blockIdx.x, p.nwg);
  const int tw = L % p.tiles_w;
  L /= p.tiles_w;
  const int th = L % p.tiles_h;
  const int n = L / p.tiles_h;
  const int oh0 = th * TR, ow0 = tw * TC;

  // ---- descriptors: this frame of x (phase 1 A and the residual), the six weight planes
  const float* xn = p.x + (int64_t)n * p.xsn;
  const int frame_bytes = (int)(((int64_t)(p.H - 1) * p.xsh + (int64_t)(p.W - 1) * p.xsw + CIN) * 4);
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(xn, frame_bytes);
  __amdgpu_buffer_rsrc_t wr[3][2];
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    const int rows = l == 2 ? CIO : MID;
    wr[l][0] = buf_rsrc(p.wh[l], rows * p.kp[l] * 2);
    wr[l][1] = buf_rsrc(p.wl[l], rows * p.kp[l] * 2);
  }
  // W1 / W2 ring pieces of this wave: piece j = wave PPW + i -> plane j / NPP (= the wave's
  // plane: the first half of the waves the hi plane, the second the lo), rows PROWS (j % NPP) ..
  // + PROWS (NPP = MID / PROWS pieces per plane). The plane's descriptors are selected once
  // (wave-uniform SGPRs: a per-piece select spilled them to scratch)
  constexpr int NPP = MID / PROWS;
  static_assert(NPP % PPW == 0 && PPW * NW == 2 * NPP, "W ring piece map");
  const bool bq = wave * PPW / NPP != 0;
  const __amdgpu_buffer_rsrc_t wq0 = bq ? wr[0][1] : wr[0][0], wq1 = bq ? wr[1][1] : wr[1][0];
  int bnrow[PPW], bch[PPW], bdst[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int j = wave * PPW + i;
    bnrow[i] = (j % NPP) * PROWS + ((lane >> 2) & (PROWS - 1));
    bch[i] = (lane & 3) ^ swzF(bnrow[i]);
    bdst[i] = RING_OFF + ((j / NPP) * MID + (j % NPP) * PROWS) * 64;
  }
  auto issue_w = [&](int l, int kt, int stage) {           // l = 0 (W1) or 1 (W2)
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const unsigned vo = (unsigned)((bnrow[i] * p.kp[l] + bch[i] * 8) * 2);
      if constexpr (S::HALF) {
        if (lane < 32) bl_lds16(l ? wq1 : wq0, lds + bdst[i] + stage * STAGE, vo, kt * BK_ * 2);
      } else {
        bl_lds16(l ? wq1 : wq0, lds + bdst[i] + stage * STAGE, vo, kt * BK_ * 2);
      }
    }
  };
  // the W stream: steps u < NK1 are W1's K-steps, the next 18 W2's; step u goes to stage u % RING
  constexpr int NK2 = (MID / 32) * 9, NU = NK1 + NK2;
  auto issue_wu = [&](int u) {
    if (u < NK1) issue_w(0, u, u % RING);
    else if (u < NU) issue_w(1, u - NK1, u % RING);
  };

  // =========================== phase 1: t1 on the haloed tile
  const float am = p.x_amax[n];
  const int ex = f16_scale_exp(am);
  const float sa = ldexpf(1.f, 15 - ex), inv0 = ldexpf(1.f, ex - 15);
  // row blocks wave and wave + 8 (the latter only for waves 0..3); lane fr's pixel of each
  const bool two = wave + NW < NRB1;                         // wave-uniform
  // The x loads go out pixel-contiguous: load h (0, 1) of lane l reads pixel 8 h + (l >> 3) of
  // the row block, 16-B chunk l & 7 of the K-step's 128 B (a lane quad = 64 contiguous bytes),
  // and a wave-private 2-KiB slot per row block in TT (free until t1's epilogue) transposes them
  // to the fragment layout (lane (fr, fg): pixel fr, channels fg*8 .. +7). Loaded straight into
  // fragment lanes, every quad spanned 4 pixels 1 KB apart: the texture-address unit was busy
  // 0.69 of the kernel's cycles after phase 3 went contiguous (profiles/r06_pmc_bneck_ta_ycoal.txt).
  static_assert(NRB1 * 2048 <= S::TT_BYTES, "x transpose slots in TT");
  unsigned av[2][2];
  bool pv[2];                                                // pixel fr of row block i is inside the image
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rb = wave + i * NW;
    auto inside = [&](int px, int& ih, int& iw) {
      const int hr = px / HW_, hc = px - hr * HW_;
      ih = oh0 - 1 + hr; iw = ow0 - 1 + hc;
      return px < HP && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W && rb < NRB1;
    };
    int ih, iw;
    pv[i] = inside(rb * 16 + fr, ih, iw);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool v = inside(rb * 16 + 8 * h + (lane >> 3), ih, iw);
      av[i][h] = v ? (unsigned)(((int64_t)ih * p.xsh + (int64_t)iw * p.xsw + (lane & 7) * 4) * 4) : BL_OOB;
    }
  }
  f32x4 acc1[2][NJ1];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ1; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // A straight from global into registers, two K-steps ahead (raw[step & 1])
  constexpr int AD = S::AD;
  f4 raw[AD][2][2];
  auto load_a = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i == 1 && !two) continue;
      raw[kt % AD][i][0] = bl_f4(xr, av[i][0], kt * BK_ * 4);
      raw[kt % AD][i][1] = bl_f4(xr, av[i][1], kt * BK_ * 4);
    }
  };
  f16x8 af[2][2];
  auto split = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i == 1 && !two) continue;
      // transpose through the row block's slot (chunk slots XOR-swizzled by pixel: the b128 reads
      // of 8 lanes / 8 pixels hit 8 distinct bank quads); same-wave LDS ops complete in order
      unsigned char* const scr = lds + (wave + i * NW) * 2048;
      const int q0 = lane >> 3, c = lane & 7;
      *reinterpret_cast<f4*>(scr + q0 * 128 + ((c ^ q0) << 4)) = raw[kt % AD][i][0];
      *reinterpret_cast<f4*>(scr + (8 + q0) * 128 + ((c ^ q0) << 4)) = raw[kt % AD][i][1];
      const f4 x0 = *reinterpret_cast<const f4*>(scr + fr * 128 + (((2 * fg) ^ (fr & 7)) << 4));
      const f4 x1 = *reinterpret_cast<const f4*>(scr + fr * 128 + (((2 * fg + 1) ^ (fr & 7)) << 4));
      unsigned long long p0[2], p1[2];
      split_planes_f16(x0, sa, p0);
      split_planes_f16(x1, sa, p1);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        af[i][q] = __builtin_bit_cast(f16x8, u64x2{p0[q], p1[q]});
      }
    }
  };
  // Per step kt: [wait + barrier] W(kt + RING - 1) issued, split of A(kt) (its registers are then
  // free), A(kt + AD) issued into them, MFMAs on A(kt). A(kt) was issued AD steps earlier: the
  // split waits for it at the start of its own step, not at the end of the one before (round 6:
  // the phase timeline, tools/bneck_trace.py, had phase 1 at 42 % of a tile, ~2.4 us per K-step
  // for ~0.3 us of MFMAs -- latency-bound on x with one step of cover). The wait leaves in flight
  // exactly the ops issued after this wave's pieces of W(kt): 2 W steps (PPW pieces each) and
  // na_step(kt) A steps (na = 4 / 2 loads each).
  static_assert(RING == 4 && NK1 >= AD, "phase-1 wait counts");
#pragma unroll
  for (int u = 0; u < RING - 1; ++u) issue_wu(u);
  // the counted waits below assume this issue order (W pieces, then the A loads); without the
  // fence the scheduler may hoist the A loads above the LDS-DMA (a build that only added A loads
  // did so, and W(0) was then not covered by the first wait: wrong results)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < AD; ++k) load_a(k);
  // A steps issued after W(kt): W(0..2) precede the AD prologue steps and steps 0..kt-1's loads;
  // W(kt >= 3) is followed by the loads of steps kt-3..kt-1 (step j loads A(j + AD) if < NK1)
  auto na_step = [&](int kt) {
    int m = kt < RING - 1 ? AD : 0;
    for (int j = kt < RING - 1 ? 0 : kt - (RING - 1); j < kt; ++j) m += j + AD < NK1;
    return m;
  };
#pragma unroll
  for (int kt = 0; kt < NK1; ++kt) {
    const int m = na_step(kt);
    if (two) {
      if (m == 2) wait_barrier<2 * PPW + 2 * 4>();
      else if (m == 3) wait_barrier<2 * PPW + 3 * 4>();
      else if (m == 4) wait_barrier<2 * PPW + 4 * 4>();
      else if (m == 5) wait_barrier<2 * PPW + 5 * 4>();
      else if (m == 6) wait_barrier<2 * PPW + 6 * 4>();
      else wait_barrier<2 * PPW>();                          // (m <= 1: a smaller count only waits longer)
    } else {
      if (m == 2) wait_barrier<2 * PPW + 2 * 2>();
      else if (m == 3) wait_barrier<2 * PPW + 3 * 2>();
      else if (m == 4) wait_barrier<2 * PPW + 4 * 2>();
      else if (m == 5) wait_barrier<2 * PPW + 5 * 2>();
      else if (m == 6) wait_barrier<2 * PPW + 6 * 2>();
      else wait_barrier<2 * PPW>();
    }
    issue_wu(kt + RING - 1);
    __builtin_amdgcn_sched_barrier(0);                       // W(kt + 3) before A(kt + AD): the counts
    split(kt);
    if (kt + AD < NK1) load_a(kt + AD);
    const unsigned char* sb = lds + RING_OFF + (kt % RING) * STAGE;
#pragma unroll
    for (int j = 0; j < NJ1; ++j) {
      f16x8 b[2];
      b_frags(sb, MID, j, fr, fg, b);
      acc1[0][j] = mfma3t(b, af[0], acc1[0][j]);
      if (two) acc1[1][j] = mfma3t(b, af[1], acc1[1][j]);
    }
  }
  // epilogue 1: bn1 + ReLU (zero outside the image: conv2's padding), tile max, planes -> TT.
  // Lane (fr, fg) holds channels j*16 + fg*4 .. +3 of pixel rb*16 + fr.
  float m1 = 0.f;
#pragma unroll
  for (int j = 0; j < NJ1; ++j) {
    const int c0 = j * 16 + fg * 4;
    const f4 s = *reinterpret_cast<const f4*>(p.sc[0] + c0), b = *reinterpret_cast<const f4*>(p.bi[0] + c0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = fmaf(acc1[i][j][r] * inv0, s[r], b[r]);
        v = v > 0.f && pv[i] && (i == 0 || two) ? v : 0.f;
        acc1[i][j][r] = v;
        m1 = fmaxf(m1, v);
      }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m1 = fmaxf(m1, __shfl_xor(m1, o, 64));
  // every wave's phase-1 reads of the ring done (their MFMAs consumed them). The W2 steps
  // W(NK1 .. NK1 + 2) issued in phase 1 stay in flight: a vmcnt(0) here made every tile wait for
  // their landing before its t1 epilogue (round 6, tools/bneck_trace.py)
  wait_barrier<(RING - 1) * PPW>();
  // tile max through per-wave slots in the ring stage of W1's last step (dead now; the next DMA
  // into it, W(NK1 + 3), is issued only after phase 2's first barrier): no zeroing, no atomics
  float* const wmax1 = reinterpret_cast<float*>(lds + RING_OFF + ((NK1 - 1) % RING) * STAGE);
  if (lane == 0) wmax1[wave] = m1;
  lds_barrier();                                             // (not __syncthreads: its fence drains vmcnt)
  m1 = wmax1[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) m1 = fmaxf(m1, wmax1[w]);
  const int e1 = f16_scale_exp(m1);
  const float s1 = ldexpf(1.f, 15 - e1), inv1 = ldexpf(1.f, e1 - 15);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (i == 1 && !two) continue;
#pragma unroll
    for (int j = 0; j < NJ1; ++j) {
      unsigned long long pl[2];
      split_planes_f16(acc1[i][j], s1, pl);
      {
        const int q1 = (wave + i * NW) * 16 + fr;
        put_planes4(lds, CHB1, q1, swz_halo(q1 % HW_), j * 16 + fg * 4, pl);
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        // t1 in LDS before the next barrier

  // =========================== phase 2: t2 = conv2(t1), the halo K-loop on the LDS tile
  int aoff[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int px = (wave + t / 3) * HW_ + fr + t % 3;
    aoff[t] = px * 128 + (((2 * fg) ^ swz_halo(px % HW_)) << 4);
  }
  f32x4 acc2[NJ1];
#pragma unroll
  for (int j = 0; j < NJ1; ++j) acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  static_assert(RING == 4, "phase-2 wait counts");
  int u = NK1;
#pragma unroll 1
  for (int c = 0; c < MID / 32; ++c) {
    const unsigned char* tc = lds + c * CHB1;
#pragma unroll
    for (int t = 0; t < 9; ++t, ++u) {
      // W stream step u (its first RING - 1 were issued during phase 1): in flight after this
      // wave's pieces of W(u) are those of W(u+1), W(u+2) -- fewer in the last two steps
      if (c == MID / 32 - 1 && t >= 7) wait_barrier<0>(); else wait_barrier<(RING - 2) * PPW>();
      issue_wu(u + RING - 1);
      f16x8 a[2];
      a[0] = *reinterpret_cast<const f16x8*>(tc + aoff[t]);
      a[1] = *reinterpret_cast<const f16x8*>(tc + (aoff[t] ^ 16));
      const unsigned char* sb = lds + RING_OFF + (u % RING) * STAGE;
#pragma unroll
      for (int j = 0; j < NJ1; ++j) {
        f16x8 b[2];
        b_frags(sb, MID, j, fr, fg, b);
        acc2[j] = mfma3t(b, a, acc2[j]);
      }
    }
  }
  // epilogue 2: bn2 + ReLU, tile max, planes -> TT (t1 is dead once every wave is past here).
  // Lane (fr, fg): output pixel (oh0 + wave, ow0 + fr), channels j*16 + fg*4 .. +3.
  const int oy = oh0 + wave, ox = ow0 + fr;
  const bool ov = oy < p.H && ox < p.W;
  float m2 = 0.f;
#pragma unroll
  for (int j = 0; j < NJ1; ++j) {
    const int c0 = j * 16 + fg * 4;
    const f4 s = *reinterpret_cast<const f4*>(p.sc[1] + c0), b = *reinterpret_cast<const f4*>(p.bi[1] + c0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = fmaf(acc2[j][r] * inv1, s[r], b[r]);
      v = v > 0.f && ov ? v : 0.f;
      acc2[j][r] = v;
      m2 = fmaxf(m2, v);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m2 = fmaxf(m2, __shfl_xor(m2, o, 64));
  wait_barrier<0>();                                         // all t1 / W2 reads done, TT and ring free
  float* const wmax2 = reinterpret_cast<float*>(lds + RING_OFF + 2 * STAGE);   // past the W3 overlay
  if (lane == 0) wmax2[wave] = m2;
  // PROJ: the downsample operand, x at this lane's output pixel (channels ks*32 + fg*8 .. +7),
  // loaded now (older than every W3 piece, so the counted waits below stay exact).
  // Identity: the residual of phase-3 part 0 (x at this lane's output pixel, channels j*16 +
  // fg*4 .. +3), loaded now for the same reason: issued at part 0's start it was a full HBM
  // latency behind the part's few MFMAs (round 6 phase timeline); part h + 1's is loaded by part
  // h's epilogue as each column block frees its registers
  constexpr int NXK = PROJ ? MID / BK_ : 1;
  constexpr int NJ3 = S::R3 / 16;
  f4 xc[NXK][2];
  f4 res[PROJ ? 1 : NJ3];
  // COAL: the residual loads and y stores go out pixel-contiguous (lane 4 q + c: pixel column q,
  // channels c*4 .. +3 of a 16-channel block, so a lane quad covers 64 contiguous bytes) and the
  // accumulator layout (lane = channels of pixel fr, quads spanning 4 pixels 1 KB apart) is
  // transposed through a wave-private 1-KiB LDS slot in ring stage 2 (wmax2's stage, dead in
  // phase 3). Round 6: TA_BUSY 0.76 of the kernel's cycles (profiles/r06_pmc_bneck_ta_base.txt) --
  // address processing of the quad-scattered 16-B accesses, not HBM, set the kernel's pace.
  constexpr bool COAL = NW * 1024 <= STAGE;
  constexpr int SCR_OFF = RING_OFF + 2 * STAGE;
  const int pxq = COAL ? (lane >> 2) : fr, chq = COAL ? (lane & 3) : fg;
  const int oxq = ow0 + pxq;
  const bool ovq = oy < p.H && oxq < p.W;
  const unsigned rvo = ovq ? (unsigned)(((int64_t)oy * p.xsh + (int64_t)oxq * p.xsw + chq * 4) * 4) : BL_OOB;
  if constexpr (PROJ) {
    const unsigned cvo = ov ? (unsigned)(((int64_t)oy * p.xsh + (int64_t)ox * p.xsw + fg * 8) * 4) : BL_OOB;
#pragma unroll
    for (int ks = 0; ks < NXK; ++ks) {
      xc[ks][0] = bl_f4(xr, cvo, ks * BK_ * 4);
      xc[ks][1] = bl_f4(xr, cvo + 16, ks * BK_ * 4);
    }
  } else {
#pragma unroll
    for (int j = 0; j < NJ3; ++j) res[j] = bl_f4(xr, rvo, j * 16 * 4);
  }
  // W3 part h (R3 output columns, all NKS3 K-steps, both planes) into the overlay (TT past t2 +
  // ring stages 0-1; buffer h & 1 when double-buffered): 32 pieces, 4 per wave
  constexpr bool W3DB = S::W3DB;
  auto issue_w3 = [&](int h) {
    unsigned char* const w3b = lds + W3_OFF + (W3DB ? (h & 1) * W3_PART : 0);
    constexpr int RB3 = R3 / 16;
#pragma unroll
    for (int i = 0; i < PW3; ++i) {
      const int idx = wave * PW3 + i;
      const int rb = idx % RB3, q = (idx / RB3) & 1, ks = idx / (2 * RB3);
      const int nrow = rb * 16 + (lane >> 2);
      const int ch = (lane & 3) ^ swzF(nrow);
      const unsigned vo = (unsigned)(((h * R3 + nrow) * p.kp[2] + ch * 8) * 2);
      bl_lds16(q ? wr[2][1] : wr[2][0], w3b + ks * W3_STEP + (q * R3 + rb * 16) * 64, vo, ks * BK_ * 2);
    }
  };
  // (fence: the x loads above and the W3 pieces stay in separate scheduling regions, so no
  // counted wait's window can depend on their relative order; tools/barrier_hoist_check.py)
  // conv3's scale / bias (CIO floats each) into ring stage 3 (free since the barrier above) by
  // LDS-DMA, older than every phase-3 access the counted waits below count: the epilogue reads
  // them from LDS. Loaded into registers there, they were the youngest vector-memory ops at each
  // use, so the compiler's wait for them (vmcnt(0), one in-order counter) also drained the part's
  // previous y stores: store -> load -> wait -> store, serialised per 16 columns.
  constexpr int SB3_OFF = RING_OFF + 3 * STAGE;
  static_assert(2 * CIO * 4 <= STAGE && 2 * (CIO / 256) <= NW, "SB3: one 1-KiB piece per wave");
  {
    constexpr int NSB = CIO / 256;                           // 1-KiB pieces per array
    if (wave < 2 * NSB) {
      const int arr = wave / NSB, pc = wave % NSB;
      bl_lds16(buf_rsrc(arr ? p.bi[2] : p.sc[2], CIO * 4), lds + SB3_OFF + (arr * CIO + pc * 256) * 4,
               (unsigned)(pc * 1024 + lane * 16), 0);
    }
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  issue_w3(0);
  // an LDS-only barrier: __syncthreads' fence is a vmcnt(0), which made the t2 epilogue wait for
  // W3 part 0 and part 0's residual; phase 3's first wait takes them instead, after this work
  lds_barrier();
  m2 = wmax2[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) m2 = fmaxf(m2, wmax2[w]);
  // PROJ: t2 and x feed one accumulator, so they share one scale (their maxima combined, as
  // prpe_conv2d's dual-input GEMM); the x bound is per frame, t2's per tile
  const int e2 = f16_scale_exp(PROJ ? fmaxf(m2, am) : m2);
  const float s2 = ldexpf(1.f, 15 - e2), inv2 = ldexpf(1.f, e2 - 15);
#pragma unroll
  for (int j = 0; j < NJ1; ++j) {
    unsigned long long pl[2];
    split_planes_f16(acc2[j], s2, pl);
    put_planes4(lds, CHB2, wave * 16 + fr, swz_rows(wave * 16 + fr), j * 16 + fg * 4, pl);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        // t2 in LDS before the next barrier
  f16x8 xb[NXK][2];
  if constexpr (PROJ) {
#pragma unroll
    for (int ks = 0; ks < NXK; ++ks) {
      unsigned long long p0[2], p1[2];
      split_planes_f16(xc[ks][0], s2, p0);
      split_planes_f16(xc[ks][1], s2, p1);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        xb[ks][q] = __builtin_bit_cast(f16x8, u64x2{p0[q], p1[q]});
      }
    }
  }

  // =========================== phase 3: y = relu(bn3(W3 t2) + x) in NPART parts of R3 columns
  // (PROJ: y = relu(W' [t2 | x] + b3 + bd)). Residual loads and y stores are 16-B buffer
  // accesses (an invalid pixel's offset is past the descriptor: zeros / dropped), issued
  // unconditionally so every wave counts the same vmcnt.
  constexpr int NPART = S::NPART, NKS3 = S::NKS3, NJ = NJ3;
  constexpr int NRES = PROJ ? 0 : NJ;                        // residual loads per part
  const int yframe_bytes = (int)(((int64_t)(p.H - 1) * p.ysh + (int64_t)(p.W - 1) * p.ysw + CIO) * 4);
  const __amdgpu_buffer_rsrc_t yr = buf_rsrc(p.y + (int64_t)n * p.ysn, yframe_bytes);
  const unsigned yvo = ovq ? (unsigned)(((int64_t)oy * p.ysh + (int64_t)oxq * p.ysw + chq * 4) * 4) : BL_OOB;
  const int q3 = wave * 16 + fr;
  const int a3 = q3 * 128 + (((2 * fg) ^ swz_rows(q3)) << 4);
  float ymax = 0.f;
#pragma unroll 1
  for (int h = 0; h < NPART; ++h) {
    if (h == 0) {
      wait_barrier<0>();                                     // t2 written; W3 part 0, SB3 and part 0's residual landed
    } else {
      // W3 part h was issued before part h-1's epilogue: its NJ stores and (identity) the NJ
      // residual loads of this part
      wait_barrier<NJ + NRES>();
    }
    if constexpr (W3DB) {
      // every wave is past part h-1's MFMAs: its buffer takes part h + 1 now
      if (h + 1 < NPART) issue_w3(h + 1);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);             // (the counted waits assume this issue order)
    }
    f32x4 acc3[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc3[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS3; ++ks) {
      f16x8 a[2];
      if (ks < MID / BK_) {
        a[0] = *reinterpret_cast<const f16x8*>(lds + ks * CHB2 + a3);
        a[1] = *reinterpret_cast<const f16x8*>(lds + ks * CHB2 + (a3 ^ 16));
      } else {
        a[0] = xb[ks - MID / BK_ < NXK ? ks - MID / BK_ : 0][0];
        a[1] = xb[ks - MID / BK_ < NXK ? ks - MID / BK_ : 0][1];
      }
      const unsigned char* sb = lds + W3_OFF + (W3DB ? (h & 1) * W3_PART : 0) + ks * W3_STEP;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        f16x8 b[2];
        b_frags(sb, R3, j, fr, fg, b);
        acc3[j] = mfma3t(b, a, acc3[j]);
      }
    }
    if (!W3DB && h + 1 < NPART) {
      // every wave is done reading W3 part h (its ds_reads fed the MFMAs above): overwrite it
      // with part h + 1 now, BEFORE this part's stores
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      issue_w3(h + 1);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);             // (the counted waits assume this issue order)
    }
    // (residual +) bn3 + ReLU: lane (fr, fg) = pixel (oy, ox), channels h*R3 + j*16 + fg*4 .. +3;
    // with COAL transposed to lane (pxq, chq) before the residual add
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c0 = h * R3 + j * 16 + fg * 4;
      const float* const sb3 = reinterpret_cast<const float*>(lds + SB3_OFF);
      const f4 s = *reinterpret_cast<const f4*>(sb3 + c0), b = *reinterpret_cast<const f4*>(sb3 + CIO + c0);
      f4 t;
#pragma unroll
      for (int r = 0; r < 4; ++r) t[r] = fmaf(acc3[j][r] * inv2, s[r], b[r]);
      if constexpr (COAL) {
        // (swizzled chunk slots: the 8 lanes of each b128 access phase hit 8 distinct bank quads)
        unsigned char* const scr = lds + SCR_OFF + wave * 1024;
        *reinterpret_cast<f4*>(scr + fr * 64 + (((fg ^ (fr >> 2)) & 3) << 4)) = t;
        t = *reinterpret_cast<const f4*>(scr + pxq * 64 + (((chq ^ (pxq >> 2)) & 3) << 4));
      }
      f4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float u = t[r];
        if constexpr (!PROJ) u += res[j][r];
        v[r] = u > 0.f ? u : 0.f;
        ymax = fmaxf(ymax, v[r]);
      }
      bs_f4(yr, v, yvo, (h * R3 + j * 16) * 4);
      store_data_guard(v);
      if constexpr (!PROJ) {
        if (h + 1 < NPART) res[j] = bl_f4(xr, rvo, ((h + 1) * R3 + j * 16) * 4);
      }
    }
    asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);             // (the counted waits assume this issue order)
  }
  if (!ovq) ymax = 0.f;                                      // (an invalid pixel's y is relu(bias))
  if (p.y_amax) amax_commit(p.y_amax + n, ymax);
}

}  // namespace

// tile rows: 8 (one workgroup of 8 waves per 8 x 16 tile, two per CU at inner width 64).
// PRPE_BNECK_TR=16 selects the 16 x 16-pixel, 16-wave tile for the inner-width-64 blocks (A/B
// runs, round 5): it halves the weight bytes staged per pixel and the halo (1.41x -> 1.27x) but
// measured slower -- layer1 identity block 5.21 -> 5.80 ms, projection 4.05 -> 4.38 ms at bs = 256
// (profiles/r05_bneck_ablate.txt): one 16-wave workgroup per CU stalls every wave at each
// barrier where two 8-wave workgroups cover each other's, and phase 1's 21 haloed row blocks
// leave 11 of 16 waves idle for half the phase
int bneck_rows(int mid) {
  static const int tr = [] {
    const char* e = getenv("PRPE_BNECK_TR");
    return e && e[0] == '1' && e[1] == '6' ? 16 : 8;
  }();
  return mid == 64 ? tr : 8;
}

template <int MIDT, bool PROJ, int TRT>
int bneck_launch_t(BneckK kp, hipStream_t st) {
  kp.tiles_w = (kp.W + TC - 1) / TC;
  kp.tiles_h = (kp.H + TRT - 1) / TRT;
  const int64_t nwg = (int64_t)kp.N * kp.tiles_w * kp.tiles_h;
  if (nwg <= 0 || nwg >= (1LL << 31)) return PRPE_EINVAL;
  kp.nwg = (int)nwg;
  hipLaunchKernelGGL((bneck_kernel<MIDT, PROJ, TRT>), dim3(kp.nwg), dim3(TRT * 64), 0, st, kp);
  return launch_status();
}

int bneck_launch(const BneckK& kp, int rows, hipStream_t st) {
  if (rows == 16 && kp.mid == 64)
    return kp.proj ? bneck_launch_t<64, true, 16>(kp, st) : bneck_launch_t<64, false, 16>(kp, st);
  if (rows != 8) return PRPE_EINVAL;
  if (kp.proj) return bneck_launch_t<64, true, 8>(kp, st);
  return kp.mid == 64 ? bneck_launch_t<64, false, 8>(kp, st) : bneck_launch_t<128, false, 8>(kp, st);
}

}  // namespace prpe_k

extern "C" int prpe_bottleneck(const prpe_bneck_desc* d, void* stream) {
  using namespace prpe_k;
  if (!d || !view_ok(&d->x) || !view_ok(&d->y) || !d->x_amax) return PRPE_EINVAL;
  const prpe_view& x = d->x; const prpe_view& y = d->y;
  if (views_overlap(x, y)) return PRPE_EINVAL;            // not in place (prpe.h)
  const int MID = d->mid, CIO = 4 * d->mid;
  const bool proj = x.c == MID;                          // projection block (layer1.0)
  if ((MID != 64 && MID != 128) || (proj && MID != 64) || (x.c != CIO && !proj) || y.c != CIO || x.n != y.n ||
      x.h != y.h || x.w != y.w)
    return PRPE_EINVAL;
  if (x.sc != 1 || y.sc != 1 || x.sw % 4 || x.sh % 4 || x.sn % 4 || (uintptr_t)x.ptr % 16 || x.sw < 0 || x.sh < 0 ||
      y.sw % 4 || y.sh % 4 || y.sn % 4 || (uintptr_t)y.ptr % 16 || y.sw < 0 || y.sh < 0)
    return PRPE_EINVAL;
  const int kneed[3] = {(int)x.c, 9 * MID, proj ? 2 * MID : MID};
  for (int l = 0; l < 3; ++l) {
    if (!d->w_h16[l] || !d->w_l16[l] || !d->scale16[l] || !d->bias[l] || d->k_pad[l] != kneed[l]) return PRPE_EINVAL;
    if ((uintptr_t)d->w_h16[l] % 16 || (uintptr_t)d->w_l16[l] % 16 || (uintptr_t)d->scale16[l] % 16 ||
        (uintptr_t)d->bias[l] % 16)
      return PRPE_EINVAL;
  }
  if (((int64_t)(x.h - 1) * x.sh + (int64_t)(x.w - 1) * x.sw + x.c) * 4 >= (1LL << 31) ||
      ((int64_t)(y.h - 1) * y.sh + (int64_t)(y.w - 1) * y.sw + CIO) * 4 >= (1LL << 31))
    return PRPE_EINVAL;
  BneckK kp{};
  kp.x = x.ptr; kp.xsn = x.sn; kp.xsh = x.sh; kp.xsw = x.sw; kp.x_amax = d->x_amax;
  kp.y = y.ptr; kp.ysn = y.sn; kp.ysh = y.sh; kp.ysw = y.sw; kp.y_amax = d->y_amax;
  kp.N = x.n; kp.H = x.h; kp.W = x.w;
  kp.proj = proj ? 1 : 0;
  kp.mid = MID;
  for (int l = 0; l < 3; ++l) {
    kp.wh[l] = d->w_h16[l]; kp.wl[l] = d->w_l16[l]; kp.kp[l] = d->k_pad[l];
    kp.sc[l] = d->scale16[l]; kp.bi[l] = d->bias[l];
  }
  return bneck_launch(kp, bneck_rows(MID), as_stream(stream));
}
