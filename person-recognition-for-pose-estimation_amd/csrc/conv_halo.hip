// 3x3 / stride 1 / pad 1 convolution on CDNA4 MFMA with the input tile staged ONCE per
// 32-channel chunk as a haloed spatial tile in LDS ("halo" kernel).
//
// Why (tools/conv_bench.py ablations of the wave-row kernel, profiles/r02_conv_ablation.txt):
// on the adapters' 3x3 256->128 convs the wave-row kernel spends ~25 % of its time on the A
// operand's fragment-shaped global loads (each input pixel is fetched once per tap: 9 times)
// and ~25 % on the B ring's LDS-DMA, i.e. on vector-memory instructions per MFMA, not on
// bytes. Here a block owns a TR x TC patch of output pixels of one frame (all of them in
// rows of 16 consecutive pixels) and, per 32-channel chunk, DMAs the (TR+2) x (TC+2) input
// patch into LDS in full 128-B pixel lines; the 9 taps of the chunk then read their A
// fragments from that tile (a tap is a shift of the patch). With 8 waves per block the B
// ring costs 2 DMA pieces per wave and K-step instead of 4, and the halo ~0.6.
//
// GEMM view, K order (chunk-major: k = (chunk * 9 + kh * 3 + kw) * 32 + ci % 32), split
// arithmetic and per-accumulator MFMA order are those of conv_wave.hip, so the result is
// bit-identical to it (tested).
//
// LDS (one array): halo double buffer [2][HQ * 8 px][8 x 16 B] (slot swizzle: logical 16-B
// slot s of pixel q lives at s ^ swz_halo(column of q) (conv.h): 16 consecutive pixels of a fragment read hit
// 16 distinct (half-row, slot) pairs -- conflict-free ds_read_b128), B ring [2][2 planes][128
// cols][64 B] (the wave kernel's swizzle). The epilogue slab reuses the halo buffers.
//
// Pipeline per K-step kt = (chunk c, tap t), one block barrier each:
//   vmcnt(0) + s_barrier          -- B(kt) and the halo of chunk c (issued earlier) landed
//   LDS-DMA B(kt+1) -> other stage, and this wave's share of the halo of chunk c+1 (spread
//   over the taps of chunk c) -> other halo buffer
//   A fragments of tap t from the halo of chunk c, B fragments from stage kt&1, MFMAs
#include "conv.h"

namespace prpe_k {
namespace {

constexpr int HBK = 32;


// 16-row slab GEMM of the epilogue: zc[jn] (16 x 16, jn < NTN) = slab[16][K] x W^T, W held as
// two bf16 planes (row stride ws, plane stride ps) in LDS; A split into two planes here; three
// products (precision 0). Lane layout as the main loop's 16x16x32 MFMA.
template <int NTN, int K>
__device__ __forceinline__ void slab_gemm(const float* ct, int cs, const uint16_t* w, int ws, int ps, int fr, int fg,
                                          f32x4 (&zc)[NTN]) {
#pragma unroll
  for (int jn = 0; jn < NTN; ++jn) zc[jn] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < K / 32; ++kk) {
    const float* ap = ct + fr * cs + kk * 32 + fg * 8;
    bf16x4 p0[2], p1[2];
    split_planes<2>(*reinterpret_cast<const f4*>(ap), p0);
    split_planes<2>(*reinterpret_cast<const f4*>(ap + 4), p1);
    bf16x8 za[2];
#pragma unroll
    for (int q = 0; q < 2; ++q)
      za[q] = bf16x8{p0[q][0], p0[q][1], p0[q][2], p0[q][3], p1[q][0], p1[q][1], p1[q][2], p1[q][3]};
#pragma unroll
    for (int jn = 0; jn < NTN; ++jn) {
      const uint16_t* bp = w + (jn * 16 + fr) * ws + kk * 32 + fg * 8;
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(bp);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(bp + ps);
      zc[jn] = mfma16(za[1], b0, zc[jn]);
      zc[jn] = mfma16(za[0], b1, zc[jn]);
      zc[jn] = mfma16(za[0], b0, zc[jn]);
    }
  }
}

// fp32 [rows][cols] (row-major, ld) -> two bf16 planes [R][ws] in LDS (zero outside rows x cols)
template <int R, int C>
__device__ __forceinline__ void stage_planes(const float* w, int rows, int cols, int ld, uint16_t* dst, int ws,
                                             int tid, int nthr) {
  for (int e = tid; e < R * C / 4; e += nthr) {
    const int r = e / (C / 4), c = (e - r * (C / 4)) * 4;
    f4 v = {0.f, 0.f, 0.f, 0.f};
    if (r < rows && c < cols) v = *reinterpret_cast<const f4*>(w + r * ld + c);
    bf16x4 pl[2];
    split_planes<2>(v, pl);
    *reinterpret_cast<bf16x4*>(dst + r * ws + c) = pl[0];
    *reinterpret_cast<bf16x4*>(dst + R * ws + r * ws + c) = pl[1];
  }
}

// TAPS 1: the epilogue's activated tile (all Co <= BN columns of 16 rows at a time, in the
// wave's LDS slice) is multiplied by w2 [n2][Co] (split-bf16 MFMAs, w2 split into LDS once per
// block) and z is written to y2 instead of y. TAPS 2: z1 = act2(s2 (y' w2^T) + b2) with w2
// [nmid <= 64][Co] first, back into the slice, then z = z1 w3^T (see prpe.h, w2 / w3).
// WN: waves along N (WN = 2: a 2 x 2 wave grid, wave tile 64 px x BN/2; the B fragments of a
// K-step are read by 2 waves instead of 4: -20 % LDS reads per MFMA at 4 waves).
// ONE (precision 4, with F16): one scaled fp16 plane per operand (RNE), one MFMA per product;
// the B ring stages the weights' hi plane only. At a third of the MFMAs per tap the fp32 A reads
// (two ds_read_b128 + the conversion per fragment, every tap) made the kernel LDS-bound, so the
// chunk's halo is converted ONCE, at its first tap, into an fp16 copy (64 B per pixel, 16-B slot
// g of pixel q at g ^ ((q >> 2) & 3): 16 consecutive pixels of one slot hit 16 distinct bank
// groups), and every tap reads one ds_read_b128 per fragment from it. One extra barrier per chunk.
template <int NW, int TR, int TC, int TN, bool F16, bool APL, int TAPS = 0, int WN = 1, bool ONE = false>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2))) void conv_halo_kernel(ConvK p, int tiles_w, int tiles_h) {
  static_assert(TC % 16 == 0 && (TR * TC / 16) % (NW / WN) == 0 && TN % WN == 0, "tile");
  static_assert(!(F16 && APL), "planes input is precision 0");
  static_assert(!ONE || (F16 && TAPS == 0), "single fp16 plane: precision 4, no epilogue GEMM");
  static_assert(WN == 1 || WN == 2, "waves along N");
  using frag_t = typename std::conditional<F16, f16x8, bf16x8>::type;
  constexpr int TM = TR * TC / 16 / (NW / WN);          // 16-pixel row blocks per wave
  constexpr int TNW = TN / WN;                          // 16-column tiles per wave
  constexpr int BN = TN * 16, NP = ONE ? 1 : 2;
  constexpr int HW_ = TC + 2, HP = (TR + 2) * HW_;      // halo pixels
  constexpr int HQ = (HP + 7) / 8;                      // 1-KiB DMA pieces per halo
  constexpr int HALO = HQ * 8 * 128;                    // bytes per halo buffer
  constexpr int B_STAGE = NP * BN * 64;
  constexpr int NB_TOT = NP * BN / 16;                  // 1-KiB pieces per B stage
  constexpr int IB = NB_TOT / NW;
  static_assert(NB_TOT % NW == 0, "B pieces per wave");
  constexpr int CS = BN / WN + 4;
  constexpr int EPI = NW * 16 * CS * 4;
  constexpr int H16 = ONE ? HQ * 8 * 64 : 0;            // fp16 copy of the current chunk's halo
  constexpr int MAIN = 2 * HALO + 2 * B_STAGE + H16;
  // w2 (and w3) bf16 planes after the slabs
  constexpr int W2R = TAPS == 2 ? 64 : 32;
  constexpr int W2B = TAPS ? 2 * W2R * (BN + 8) * 2 + (TAPS == 2 ? 2 * 32 * 72 * 2 : 0) : 0;
  constexpr int LDS_BYTES = MAIN > EPI + W2B ? MAIN : EPI + W2B;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];
  unsigned char* const halo0 = lds;
  unsigned char* const ring = lds + 2 * HALO;
  unsigned char* const h16 = lds + 2 * HALO + 2 * B_STAGE;

  // the wave index through readfirstlane: provably wave-uniform, so the buffer descriptors and
  // LDS-DMA destinations derived from it stay in SGPRs (no waterfall loops around the loads)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fg = lane >> 4;
  int L = xcd_remap(blockIdx.x, p.nwg);
  const int tile_n = L % p.tiles_n;
  L /= p.tiles_n;
  const int tw = L % tiles_w;
  L /= tiles_w;
  const int th = L % tiles_h;
  const int n = L / tiles_h;
  const int n0 = tile_n * BN;
  const int oh0 = th * TR, ow0 = tw * TC;

  // ---- LDS-DMA by buffer loads: every address is a wave-uniform descriptor + a per-lane byte
  // offset computed ONCE here + a wave-uniform step offset (soffset), so issuing a piece in the
  // K-loop costs no VALU (the 64-bit address arithmetic per piece and step was ~40 % of the
  // loop's VALU). Padding pixels get an offset past the descriptor's range: the hardware
  // returns zeros for them (no branch to a zero page).
  constexpr unsigned OOB = 0x80000000u;                // > num_records (host-checked < 2^31)
  const float* xn = p.x + (int64_t)n * p.xsn;
  const int frame_bytes = (int)(((int64_t)(p.Hi - 1) * p.xsh + (int64_t)(p.Wi - 1) * p.xsw + p.Ci) * 4);
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(xn, frame_bytes);
  // halo piece q = pixels 8q .. 8q+7 (lane -> pixel 8q + lane/8, physical slot lane%8); this
  // wave's pieces are q = wave + k NW, k < KQ
  constexpr int KQ = (HQ + NW - 1) / NW;
  unsigned hvo[KQ];
#pragma unroll
  for (int k = 0; k < KQ; ++k) {
    const int q = wave + k * NW;
    const int px = q * 8 + (lane >> 3);
    const int hr = px / HW_, hc = px - hr * HW_;
    const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
    const int sl = (lane & 7) ^ swz_halo(hc);         // logical slot stored at this lane's slot
    const bool ok = q < HQ && px < HP && (unsigned)ih < (unsigned)p.Hi && (unsigned)iw < (unsigned)p.Wi;
    hvo[k] = ok ? (unsigned)(((int64_t)ih * p.xsh + (int64_t)iw * p.xsw + sl * 4) * 4) : OOB;
  }
  auto issue_halo = [&](int k, int c, int buf) {
    // non-temporal: 6 % fewer L2 misses on the dominant launch at equal time
    bl_lds16_nt(xr, halo0 + buf * HALO + (wave + k * NW) * 1024, hvo[k], c * HBK * 4);
  };

  // ---- B pieces (as conv_wave.hip): piece j -> plane j / TN, rows 16 (j % TN) .. +16
  const int wbytes = p.k_pad * 2 * (p.tiles_n * BN);    // one plane [co_pad][k_pad] bf16 / f16
  const __amdgpu_buffer_rsrc_t wr0 = buf_rsrc(F16 ? p.wh16 : p.whi, wbytes);
  const __amdgpu_buffer_rsrc_t wr1 = buf_rsrc(F16 ? p.wl16 : p.wlo, wbytes);
  unsigned bvo[IB];
  int bdst[IB];
  bool bpl[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int j = wave * IB + i;
    const int q = j / (BN / 16), rb = j % (BN / 16);
    const int nrow = rb * 16 + (lane >> 2);
    const int ch = (lane & 3) ^ swzF(nrow);
    bvo[i] = (unsigned)(((n0 + nrow) * p.k_pad + ch * 8) * 2);
    bdst[i] = (q * BN + rb * 16) * 64;
    bpl[i] = q != 0;                                   // wave-uniform
  }
  auto issue_b = [&](int kt, int stage) {
    unsigned char* sb = ring + stage * B_STAGE;
#pragma unroll
    for (int i = 0; i < IB; ++i)
      bl_lds16(bpl[i] ? wr1 : wr0, sb + bdst[i], bvo[i], kt * HBK * 2);
  };

  // precision 3: one frame per block -> one activation scale. Precision 4 may carry the
  // input-side affine (pro): the scale then comes from the bound of its output, as in conv_wave.hip
  const bool pro = ONE && p.in_scale != nullptr;       // kernel-uniform
  float sa = 1.f, inv = 1.f;
  if constexpr (F16) {
    float am = p.x_amax[n];
    if (pro) {
      float pS, pB;
      prologue_bounds(p.in_scale, p.in_bias, p.Ci, pS, pB);
      am = fmaf(am, pS, pB);
    }
    const int e = f16_scale_exp(am);
    sa = ldexpf(1.f, 15 - e);
    inv = ldexpf(1.f, e - 15);
  }

  // A fragment rows of this lane: row block rb = wave * TM + i -> tile row rb / (TC/16),
  // pixels (rb % (TC/16)) * 16 + fr; halo pixel of tap (kh, kw) = base + kh * HW_ + kw. The
  // byte offset of the first 16-B slot (channels 8 fg .. +3) of every (row block, tap) is
  // computed once (the tap loop is unrolled); the second slot (+4 .. +7) is logical slot 2 fg + 1
  // = the first one's physical slot XOR 1, i.e. offset ^ 16
  int aoff[TM][9];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rb = wm * TM + i;
    const int hb0 = (rb / (TC / 16)) * HW_ + (rb % (TC / 16)) * 16 + fr;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int px = hb0 + (t / 3) * HW_ + t % 3;
      const int sw = swz_halo(px % HW_);
      aoff[i][t] = ONE ? px * 64 + ((fg ^ ((px >> 2) & 3)) << 4) : px * 128 + (((2 * fg) ^ sw) << 4);
    }
  }

  f32x4 acc[TM][TNW];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TNW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nc = p.Ci / HBK;
  const int nk = nc * 9;
  // prologue: the whole halo of chunk 0 and B(0)
#pragma unroll
  for (int k = 0; k < KQ; ++k)
    if (wave + k * NW < HQ) issue_halo(k, 0, 0);
  issue_b(0, 0);

#pragma unroll 1
  for (int c = 0; c < nc; ++c) {
    const unsigned char* hb = halo0 + (c & 1) * HALO;
    const int kt0 = c * 9;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int kt = kt0 + t;
      wait_barrier<0>();
      if (kt + 1 < nk) issue_b(kt + 1, (kt + 1) & 1);
      if (c + 1 < nc) {
        // this wave's halo share of chunk c+1, spread over the taps of chunk c
#pragma unroll
        for (int k = t; k < KQ; k += 9)
          if (wave + k * NW < HQ) issue_halo(k, c + 1, (c + 1) & 1);
      }
      if constexpr (ONE) {
        if (t == 0) {
          // the chunk's halo (landed: the barrier above) -> scaled fp16, RNE, once for all taps;
          // the fp16 copy of the previous chunk is free (every wave is past its last tap).
          // pro: s x + b first on the pixels inside the frame, the padding stays 0 (the reference
          // pads the affine's output). A thread's slot g = tid & 3 is the same at every e.
          f4 ps4[2], pb4[2];
          if (pro) {
            const int ch = c * HBK + (tid & 3) * 8;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              ps4[h] = *reinterpret_cast<const f4*>(p.in_scale + ch + 4 * h);
              pb4[h] = *reinterpret_cast<const f4*>(p.in_bias + ch + 4 * h);
            }
          }
          for (int e = tid; e < HP * 4; e += NW * 64) {
            const int q = e >> 2, g = e & 3;
            const int hr = q / HW_, hc = q - hr * HW_;
            const int sw = swz_halo(hc);
            f4 v0 = *reinterpret_cast<const f4*>(hb + q * 128 + (((2 * g) ^ sw) << 4));
            f4 v1 = *reinterpret_cast<const f4*>(hb + q * 128 + (((2 * g + 1) ^ sw) << 4));
            if (pro) {
              const bool in = (unsigned)(oh0 - 1 + hr) < (unsigned)p.Hi && (unsigned)(ow0 - 1 + hc) < (unsigned)p.Wi;
              v0 = in ? affine4(v0, ps4[0], pb4[0]) : f4{0.f, 0.f, 0.f, 0.f};
              v1 = in ? affine4(v1, ps4[1], pb4[1]) : f4{0.f, 0.f, 0.f, 0.f};
            }
            *reinterpret_cast<f16x8*>(h16 + q * 64 + ((g ^ ((q >> 2) & 3)) << 4)) = cvt_f16_one(v0, v1, sa);
          }
          __builtin_amdgcn_sched_barrier(0);
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // A fragments: 8 channels (two 16-B slots) of the tap-shifted pixel
      frag_t af[NP][TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (ONE) {
          af[0][i] = *reinterpret_cast<const f16x8*>(h16 + aoff[i][t]);
          continue;
        }
        const f4 v0 = *reinterpret_cast<const f4*>(hb + aoff[i][t]);
        const f4 v1 = *reinterpret_cast<const f4*>(hb + (aoff[i][t] ^ 16));
        if constexpr (APL) {
          af[0][i] = __builtin_bit_cast(bf16x8, v0);
          af[1][i] = __builtin_bit_cast(bf16x8, v1);
        } else if constexpr (ONE) {
          af[0][i] = cvt_f16_one(v0, v1, sa);
        } else if constexpr (F16) {
          unsigned long long p0[2], p1[2];
          split_planes_f16(v0, sa, p0);
          split_planes_f16(v1, sa, p1);
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
      const unsigned char* sb = ring + (kt & 1) * B_STAGE;
#pragma unroll
      for (int j = 0; j < TNW; ++j) {
        const int nrow = (wn * TNW + j) * 16 + fr;
        const unsigned char* bp = sb + nrow * 64 + ((fg ^ swzF(nrow)) << 4);
        frag_t bfr[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) bfr[q] = *reinterpret_cast<const frag_t*>(bp + q * BN * 64);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int s = NP - 1; s >= 0; --s)
#pragma unroll
            for (int qa = s; qa >= 0; --qa) acc[i][j] = mfma16(af[qa][i], bfr[s - qa], acc[i][j]);
      }
    }
  }
  wait_barrier<0>();   // every DMA landed and every fragment read retired: LDS is free

  // ---------------- epilogue: per-wave 16-row slices (one row block = 16 consecutive pixels)
  float* ct = reinterpret_cast<float*>(lds) + wave * 16 * CS;
  constexpr int CPR = BN / WN / 4;                     // this wave's columns: wn * BN / WN ..
  constexpr int RPP = 64 / CPR;
  constexpr int EB = 16 / RPP;
  const int cc = lane % CPR, rr0 = lane / CPR;
  const int col = n0 + wn * (BN / WN) + cc * 4;
  const bool cval = col < p.Co;
  f4 sc4 = {1.f, 1.f, 1.f, 1.f}, bi4 = {0.f, 0.f, 0.f, 0.f}, sl4 = {0.f, 0.f, 0.f, 0.f};
  if (cval) {
    if (p.scale) sc4 = *reinterpret_cast<const f4*>(p.scale + col);
    if (p.bias) bi4 = *reinterpret_cast<const f4*>(p.bias + col);
    if (p.slope) sl4 = *reinterpret_cast<const f4*>(p.slope + col);
  }
  float ym = 0.f;
  // TAPS: w2 (w3) split once into two bf16 planes (rows / columns beyond the real ones zero)
  constexpr int W2S = BN + 8, W3S = 72;                // padded rows: 16-B shift per row
  uint16_t* const w2s = reinterpret_cast<uint16_t*>(lds + EPI);
  uint16_t* const w3s = w2s + 2 * W2R * W2S;
  if constexpr (TAPS != 0) {
    stage_planes<W2R, BN>(p.w2, TAPS == 2 ? p.nmid : p.n2, p.Co, p.Co, w2s, W2S, tid, NW * 64);
    if constexpr (TAPS == 2) stage_planes<32, 64>(p.w3, p.n2, p.nmid, p.nmid, w3s, W3S, tid, NW * 64);
    __syncthreads();
  }
  // TAPS 2: this lane's middle columns jn * 16 + fr
  f32x4 s2 = {0.f, 0.f, 0.f, 0.f}, b2 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (TAPS == 2) {
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) {
      const int c = jn * 16 + fr;
      if (c < p.nmid) {
        s2[jn] = p.s2 ? p.s2[c] : 1.f;
        b2[jn] = p.b2 ? p.b2[c] : 0.f;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rb = wm * TM + i;
    const int oh = oh0 + rb / (TC / 16), owb = ow0 + (rb % (TC / 16)) * 16;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < TNW; ++j) ct[(fg * 4 + r) * CS + j * 16 + fr] = acc[i][j][r];
    int64_t yo[EB];
    f4 res[EB];
    bool ok[EB];
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int ow = owb + rr0 + RPP * e;
      ok[e] = cval && oh < p.Ho && ow < p.Wo;
      res[e] = f4{0.f, 0.f, 0.f, 0.f};
      yo[e] = 0;
      if (ok[e]) {
        yo[e] = (int64_t)n * p.ysn + (int64_t)oh * p.ysh + (int64_t)ow * p.ysw + col;
        if (p.res_mode != PRPE_RES_NONE)
          res[e] = *reinterpret_cast<const f4*>(p.r + (int64_t)n * p.rsn + (int64_t)oh * p.rsh + (int64_t)ow * p.rsw + col);
      }
    }
    // (ONE: two rows at a time; the fully unrolled form, with every activation's code inlined,
    // spilled ~340 VGPRs in this variant)
#pragma unroll(ONE ? 2 : EB)
    for (int e = 0; e < EB; ++e) {
      f4 v = *reinterpret_cast<const f4*>(ct + (rr0 + RPP * e) * CS + cc * 4);
      if (!ok[e]) continue;
      if constexpr (F16) v = v * inv;
      v = v * sc4 + bi4;
      if (p.res_mode == PRPE_RES_PRE_ACT) v += res[e];
      v = apply_act4(v, p.act, sl4);   // packed GELU / SiLU, bit-identical to apply_act
      if (p.res_mode == PRPE_RES_POST_ACT) v += res[e];
      if constexpr (TAPS != 0) {                       // keep the activated value for the tap GEMM
        *reinterpret_cast<f4*>(ct + (rr0 + RPP * e) * CS + cc * 4) = v;
        continue;
      }
      if (p.y_planes) {
        bf16x4 pl[2];
        split_planes<2>(v, pl);
        uint16_t* y16 = reinterpret_cast<uint16_t*>(p.y) + 2 * (yo[e] - col) + (col >> 3) * 16 + (col & 7);
        *reinterpret_cast<bf16x4*>(y16) = pl[0];
        *reinterpret_cast<bf16x4*>(y16 + 8) = pl[1];
      } else {
        *reinterpret_cast<f4*>(p.y + yo[e]) = v;
      }
      if (p.y_amax) ym = fmaxf(ym, amax4(v));
    }
    if constexpr (TAPS != 0) {
      // z [16 pixels][32] = y' [16][BN] w2^T on the matrix cores, the two-plane (3-product)
      // split as everywhere at precision 0: A = the activated slab rows, B = the w2 planes.
      // WN = 2: each wave of a pair holds half of the rows' columns = half of this GEMM's K;
      // the odd wave hands its partial sums to the even one through its slab (fixed order).
      __builtin_amdgcn_wave_barrier();
      constexpr int KH = BN / WN;                     // this wave's share of K
      const uint16_t* w2w = w2s + wn * KH;
      auto hand_over = [&](auto& part, auto nt) {     // wn 1 -> wn 0: part[jn] += partner's
        constexpr int NT_ = decltype(nt)::value;
        if (wn == 1) {
#pragma unroll
          for (int jn = 0; jn < NT_; ++jn)
#pragma unroll
            for (int r = 0; r < 4; ++r) ct[(fg * 4 + r) * CS + jn * 16 + fr] = part[jn][r];
        }
        __syncthreads();
        if (wn == 0) {
          const float* pc = ct + 16 * CS;             // the partner's slab (wave + 1)
#pragma unroll
          for (int jn = 0; jn < NT_; ++jn)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[jn][r] += pc[(fg * 4 + r) * CS + jn * 16 + fr];
        }
      };
      f32x4 zc[2];
      if constexpr (TAPS == 1) {
        slab_gemm<2, KH>(ct, CS, w2w, W2S, W2R * W2S, fr, fg, zc);
        if constexpr (WN == 2) hand_over(zc, std::integral_constant<int, 2>{});
      } else {
        f32x4 zm[4];
        slab_gemm<4, KH>(ct, CS, w2w, W2S, W2R * W2S, fr, fg, zm);
        if constexpr (WN == 2) hand_over(zm, std::integral_constant<int, 4>{});
        __builtin_amdgcn_wave_barrier();
        if (wn == 0) {
#pragma unroll
          for (int jn = 0; jn < 4; ++jn) {
            const f32x4 t = apply_act4(zm[jn] * s2[jn] + b2[jn], p.act2, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int r = 0; r < 4; ++r) ct[(fg * 4 + r) * CS + jn * 16 + fr] = t[r];
          }
          __builtin_amdgcn_wave_barrier();
          slab_gemm<2, 64>(ct, CS, w3s, W3S, 32 * W3S, fr, fg, zc);
        }
      }
      if (wn == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ow = owb + fg * 4 + r;
          if (oh < p.Ho && ow < p.Wo) {
            float* zo = p.y2 + (int64_t)n * p.y2sn + (int64_t)oh * p.y2sh + (int64_t)ow * p.y2sw;
#pragma unroll
            for (int jn = 0; jn < 2; ++jn)
              if (jn * 16 + fr < p.n2) zo[jn * 16 + fr] = zc[jn][r];
          }
        }
      }
      if constexpr (WN == 2) __syncthreads();       // the slabs are rewritten by the next row block
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (p.y_amax) amax_commit(p.y_amax + n, ym);
}

template <int NW, int TR, int TC, int TN, bool F16, bool APL, int TAPS = 0, int WN = 1, bool ONE = false>
int launch_halo(const ConvK& kp0, hipStream_t st) {
  ConvK kp = kp0;
  if (kp.w2 && kp.Co > TN * 16) return PRPE_EINVAL;     // the tap GEMM needs every column in one tile
  const int tiles_w = (kp.Wo + TC - 1) / TC, tiles_h = (kp.Ho + TR - 1) / TR;
  kp.tiles_n = (kp.Co + TN * 16 - 1) / (TN * 16);
  const int64_t nwg = (int64_t)(kp.M / kp.HoWo) * tiles_h * tiles_w * kp.tiles_n;
  if (nwg <= 0 || nwg >= (1LL << 31)) return PRPE_EINVAL;
  kp.nwg = (int)nwg;
  hipLaunchKernelGGL((conv_halo_kernel<NW, TR, TC, TN, F16, APL, TAPS, WN, ONE>), dim3(kp.nwg), dim3(NW * 64), 0, st,
                     kp, tiles_w, tiles_h);
  return launch_status();
}

template <int NW, int TR, int TC, int TN, int WN = 1>
int launch_halo_kind(const ConvK& kp, int prec, hipStream_t st) {
  if (prec == 3) return launch_halo<NW, TR, TC, TN, true, false, 0, WN>(kp, st);
  if constexpr ((TN * 16 / 16) % NW == 0)             // single-plane B ring: whole pieces per wave
    if (prec == 4) return launch_halo<NW, TR, TC, TN, true, false, 0, WN, true>(kp, st);
  if (prec == 4) return PRPE_EINVAL;
  return kp.x_planes ? launch_halo<NW, TR, TC, TN, false, true, 0, WN>(kp, st)
                     : launch_halo<NW, TR, TC, TN, false, false, 0, WN>(kp, st);
}

// epilogue tap GEMM: the 8 x 16-pixel, 128-column tile (NW = 4) or the 16 x 16 one (NW = 8)
template <int TAPS, int WN, int NW = 4>
int launch_halo_taps_t(const ConvK& kp, int prec, hipStream_t st) {
  constexpr int TR = NW == 4 ? 8 : 16;
  if (prec == 4) return PRPE_EINVAL;
  if (prec == 3) return launch_halo<NW, TR, 16, 8, true, false, TAPS, WN>(kp, st);
  return kp.x_planes ? launch_halo<NW, TR, 16, 8, false, true, TAPS, WN>(kp, st)
                     : launch_halo<NW, TR, 16, 8, false, false, TAPS, WN>(kp, st);
}
// PRPE_HALO_WN=2: the 2 x 2 wave grid (WN = 2) for the automatic and epilogue-GEMM tiles.
// Off by default: in the model at bs = 256 it measured ViT adapter.7 +0.6 %, face-YOLO .10
// +2.8 % (two block barriers per row block in the chain epilogue), AdaFace .7 -2.8 %, bench
// 1363 -> 1357 frames/s (profiles/r02_layer_profile_halo_wn.txt), although the micro-bench on
// random data had it 4-12 % faster (profiles/r02_conv_bench_halo_wn.txt).
int halo_wn() {
  static const int wn = [] {
    const char* e = getenv("PRPE_HALO_WN");
    return e && e[0] == '2' ? 2 : 1;
  }();
  return wn;
}
int launch_halo_taps(const ConvK& kp, int prec, hipStream_t st) {
  if (halo_wn() == 2) return kp.w3 ? launch_halo_taps_t<2, 2>(kp, prec, st) : launch_halo_taps_t<1, 2>(kp, prec, st);
  return kp.w3 ? launch_halo_taps_t<2, 1>(kp, prec, st) : launch_halo_taps_t<1, 1>(kp, prec, st);
}

}  // namespace

bool conv_halo_eligible(const ConvK& kp, int prec, int km, int tile) {
  // 3x3 / stride 1 / pad 1 over whole 32-channel chunks (chunk-major weights), vectorised
  // epilogue, precision 0 (fp32 or planes input) or 3 (fp16 planes + the input's max bound).
  // Precision 4's single-plane B ring needs whole LDS-DMA pieces per wave (launch_halo_kind:
  // TN % NW == 0), which the forced 16 x 16-pixel 64-column tile (35) does not have; the
  // automatic choice (30) never maps precision 4 there (34 / 36).
  const bool p3 = prec == 3 && kp.wh16 && kp.wl16 && kp.x_amax && !kp.x_planes;
  const bool p4 = prec == 4 && kp.wh16 && kp.x_amax && !kp.x_planes && (!kp.in_scale || kp.in_bias) && tile != 35 &&
                  !kp.w2;
  // buffer descriptors: one frame of x and one weight plane each < 2^31 bytes (32-bit offsets)
  const int64_t frame_bytes = ((int64_t)(kp.Hi - 1) * kp.xsh + (int64_t)(kp.Wi - 1) * kp.xsw + kp.Ci) * 4;
  const int64_t w_bytes = (int64_t)kp.k_pad * 2 * (((kp.Co + 127) / 128) * 128);
  return km == 2 && kp.KH == 3 && kp.KW == 3 && kp.stride == 1 && kp.pad == 1 && kp.Ci % HBK == 0 &&
         kp.vec_out && (prec == 0 || p3 || p4) && (!kp.in_scale || p4) && !kp.x2 && kp.k_pad == kp.K && kp.zero &&
         kp.Hi == kp.Ho && kp.Wi == kp.Wo && kp.xsh >= 0 && kp.xsw >= 0 && frame_bytes < (1LL << 31) &&
         w_bytes < (1LL << 31);
}

// Where the automatic choice takes it (measured in the model at bs = 256, r02_layer_profile_halo.txt):
// the tile must cover the image with <= 5 % padding waste (10x10 and 40x40 trunk maps ran 1.1-1.9x
// slower on 8 x 16 tiles), and an fp32-input precision-0 conv stays on the wave kernel (the
// AdaFace adapter's 128->64 ran 8 % slower); planes input and precision 3 win (adapters' 3x3
// 256->128 -3..-5 %, trunk layer1 3x3 -10 %).
// Precision 4 (one MFMA per product, so the wave kernel's per-tap A loads weigh three times as
// much) takes it from 14 x 14 up whatever the waste: the IR-50 body's 14x14 256->256 -38 %,
// 28x28 128->128 -21 %, 56x56 64->64 -30 % at bs = 256 (profiles/r04_conv_bench_ir50_halo.txt);
// 7 x 7 stays on the wave kernel (one 8 x 16 tile per frame, 2.6x waste: no gain).
// (PRPE_P4_HALO=0 in the environment restores the waste rule for precision 4: A/B runs)
bool conv_halo_auto(const ConvK& kp, int prec) {
  static const bool p4_halo = [] {
    const char* e = getenv("PRPE_P4_HALO");
    return !(e && e[0] == '0');
  }();
  if (prec == 4 && p4_halo && kp.Ho >= 14 && kp.Wo >= 14) return true;
  if (prec == 0 && !kp.x_planes) return false;
  const int tc = 16, tr = 8;
  const int64_t covered = (int64_t)((kp.Ho + tr - 1) / tr) * tr * ((kp.Wo + tc - 1) / tc) * tc;
  return covered * 20 <= (int64_t)kp.Ho * kp.Wo * 21;
}

// tile 30 = auto: 8 x 16 output pixels, 4 waves (two workgroups per CU), 128 output channels
// per workgroup, or 64 when Co <= 64 (tools/conv_bench.py, profiles/r02_conv_bench_halo.txt);
// 31..35 force a configuration
int conv_halo_launch(const ConvK& kp, int prec, int tile, hipStream_t st) {
  // PRPE_HALO_TILE=32 / 33 makes that tile the automatic choice for Co > 64 (A/B runs; for the
  // epilogue-GEMM convs 32 selects the 16 x 16-pixel 8-wave form)
  static const int env_tile = [] {
    const char* e = getenv("PRPE_HALO_TILE");
    const int t = e ? atoi(e) : 0;
    return t == 32 || t == 33 ? t : 0;
  }();
  if (tile == 30 && env_tile && kp.Co > 64 && (!kp.w2 || env_tile == 32)) tile = env_tile;
  if (kp.w2) {
    if (tile == 32) return kp.w3 ? launch_halo_taps_t<2, 1, 8>(kp, prec, st) : launch_halo_taps_t<1, 1, 8>(kp, prec, st);
    return tile == 30 || tile == 31 ? launch_halo_taps(kp, prec, st) : PRPE_EINVAL;
  }
  // precision 4 takes the 2 x 2 wave grid for Co > 64 (half the B fragment reads per wave; AdaFace
  // adapter.7 3.05 -> 2.78 ms in the model at bs = 256, profiles/r04_layer_profile_halo_p4_wn2.txt)
  if (tile == 30) tile = kp.Co <= 64 ? 34 : (halo_wn() == 2 || prec == 4 ? 36 : 31);
  switch (tile) {
    case 31: return launch_halo_kind<4, 8, 16, 8>(kp, prec, st);     // 8 x 16 px, 4 waves, 128 ch
    case 32: return launch_halo_kind<8, 16, 16, 8>(kp, prec, st);    // 16 x 16 px, 8 waves, 128 ch
    case 33: return launch_halo_kind<8, 8, 32, 8>(kp, prec, st);     // 8 x 32 px, 8 waves, 128 ch
    case 34: return launch_halo_kind<4, 8, 16, 4>(kp, prec, st);     // 8 x 16 px, 4 waves, 64 ch
    case 35: return launch_halo_kind<8, 16, 16, 4>(kp, prec, st);    // 16 x 16 px, 8 waves, 64 ch
    case 36: return launch_halo_kind<4, 8, 16, 8, 2>(kp, prec, st);  // 8 x 16 px, 2 x 2 waves (64 px x 64 ch), 128 ch
    case 37: return launch_halo_kind<8, 16, 16, 8, 2>(kp, prec, st); // 16 x 16 px, 4 x 2 waves (64 px x 64 ch), 128 ch
    default: return PRPE_EINVAL;
  }
}

}  // namespace prpe_k
