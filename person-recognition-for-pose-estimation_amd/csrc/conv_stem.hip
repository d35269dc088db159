// ResNet-50 stem + max-pool in ONE kernel (torchvision resnet50: conv1 7x7/2 pad 3 -> bn1 ->
// relu -> maxpool 3x3/2 pad 1; the reference trunk, training/modify_models.py:413-446):
//   y[n, py, px, c] = max_{dy, dx in -1..1} relu(bn1(conv1(x)))[n, 2py + dy, 2px + dx, c]
//
// Why: the stem writes a [B, 320, 320, 64] map (6.7 GB at bs = 256) that the max-pool reads
// back once to write a quarter of it; both launches are bound by those bytes and by the stem's
// in-kernel operand split (profiles/r03_layer_profile_*: stem 3.8 ms + pool 1.8 ms). Here the
// stem output lives only in LDS: HBM traffic = the input frames (once) + the pooled output.
//
// The conv is the same chunked implicit GEMM as prpe_conv2d's stem (Engine.stem): the frames
// as a zero-bordered NHWC4 buffer [N, H+6, W+8, 4], K-step kh reads the 128-B segment of row
// 2 oy + kh at column 2 ox (8 columns x 4 channels), weights W'[co][kh*32 + kw*4 + c] (zero for
// kw = 7, c = 3), precision 3 (two fp16 planes of the frame-scaled activations, the pack's
// per-channel-scaled fp16 weight planes, three MFMA terms smallest first) and the same epilogue
// arithmetic, so every stem value equals prpe_conv2d's bit for bit (tested).
//
// One workgroup = one frame x one strip of 40 pooled columns (81 stem columns), walking the
// frame's pooled rows top to bottom. Per pooled row py: 11 waves compute the two new stem rows
// 2py, 2py+1 (162 pixels, one 16-pixel block per wave, all 64 channels; MFMAs issued
// transposed -- weights as the A operand -- so a lane's accumulator holds 4 consecutive channels
// of one pixel), write them into a 3-row LDS ring (row 2py-1 is still there from the previous
// row), and pool. Stem outputs are >= 0 (ReLU), so zeros stand for the pool's -inf padding:
// max(v, 0) = v for every window, all of which hold at least one real output. The weights
// (7 K-steps x 2 planes x 64 rows x 64 B) are LDS-resident for the whole walk; the activations
// of the next pooled row are loaded (16-B buffer loads) while this row computes.
#include "conv.h"

namespace prpe_k {

struct StemK {
  const float* x; int64_t xsn, xsh;                      // NHWC4 frames (floats); pixel stride 4
  int xframe_bytes;
  const float* x_amax;
  const uint16_t* wh; const uint16_t* wl; int kp;
  const float* sc; const float* bi;
  float* y; int64_t ysn, ysh, ysw;
  float* y_amax;
  int N, Ws, Hp, Wp, strips, nwg;
};

namespace {

// 40 pooled columns: 81 stem columns x 2 rows = 162 pixels = 11 waves of 16 (3 / 3 / 3 / 2 per
// SIMD; 32 columns gave 9 waves, 3 / 2 / 2 / 2, and the 3-wave SIMD set the pace), and a 160-wide
// pooled map is 4 whole strips
constexpr int SP_PC = 40;                                // pooled columns per workgroup
constexpr int SP_SC = 2 * SP_PC + 1;                     // stem columns per workgroup (81)
constexpr int SP_PX = 2 * SP_SC;                         // stem pixels per pooled row (162)
constexpr int SP_NW = (SP_PX + 15) / 16;                 // waves: one 16-pixel block each (11)
constexpr int SP_CO = 64, SP_K = 7;                      // output channels, K-steps (tap rows)
constexpr int SP_WSTEP = 2 * SP_CO * 64;                 // one K-step of both weight planes (8 KB)
constexpr int SP_W_BYTES = SP_K * SP_WSTEP;              // 56 KB
constexpr int SP_ROW = SP_SC * SP_CO * 4;                // one stem row of the strip (20.25 KB)
constexpr int SP_LDS = SP_W_BYTES + 3 * SP_ROW;          // 117 KB: one workgroup per CU
static_assert(SP_PC * 16 <= SP_NW * 64, "pool phase: one thread per pooled column and 4 channels");
static_assert(SP_K * 8 > SP_NW, "weight pieces");

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// ring layout: stem pixel c's 4-channel group g (16 B) at float offset 4 (g ^ (c & 7)) of its
// 256-B line. The epilogue's ds_write_b128 is serviced in groups of 8 consecutive lanes = 8
// consecutive pixels at one g: unswizzled they all hit one bank set (8-way; 42 % of LDS-active
// cycles were conflicts); swizzled they cover 8 distinct 16-B slots. The pool's reads (16 lanes
// = all 16 groups of one pixel) stay one contiguous 256-B line.
__device__ __forceinline__ int rslot(int g, int c) { return (g ^ (c & 7)) * 4; }

__device__ __forceinline__ void lds_barrier() {         // LDS traffic retired + s_barrier, fenced
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__global__ __launch_bounds__(SP_NW * 64, 1) void stem_pool_kernel(StemK p) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[SP_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int L = xcd_remap(blockIdx.x, p.nwg);
  const int strip = L % p.strips, n = L / p.strips;
  const int px0 = strip * SP_PC;                         // first pooled column of the strip
  const int sc0 = 2 * px0 - 1;                           // stem column of ring column 0
  float* const ring = reinterpret_cast<float*>(lds + SP_W_BYTES);   // [3][SP_SC][64]

  // weights into LDS by LDS-DMA: piece j = K-step j / 8, plane (j / 4) & 1, rows 16 (j & 3) ..
  // (conv_wave's slot swizzle); every piece landed at the first barrier below (vmcnt(0))
  {
    const __amdgpu_buffer_rsrc_t w0 = buf_rsrc(p.wh, SP_CO * p.kp * 2), w1 = buf_rsrc(p.wl, SP_CO * p.kp * 2);
    for (int j = wave; j < SP_K * 8; j += SP_NW) {
      const int ks = j >> 3, q = (j >> 2) & 1, rb = j & 3;
      const int nrow = rb * 16 + (lane >> 2);
      const int ch = (lane & 3) ^ swzF(nrow);
      bl_lds16(q ? w1 : w0, lds + ks * SP_WSTEP + (q * SP_CO + rb * 16) * 64,
               (unsigned)((nrow * p.kp + ch * 8) * 2), ks * 32 * 2);
    }
  }
  // ring slot of stem row -1 (the pool's top padding) = 2: zeros
  for (int i = tid; i < SP_SC * SP_CO / 4; i += SP_NW * 64)
    reinterpret_cast<f4*>(ring + 2 * SP_SC * SP_CO)[i] = f4{0.f, 0.f, 0.f, 0.f};

  // this lane's stem pixel: ring column c of stem row 2py + r (q < SP_PX), stem column sc0 + c
  const int q = wave * 16 + fr;
  const int r = q / SP_SC, c = q - r * SP_SC;
  const int scol = sc0 + c;
  const bool pvalid = q < SP_PX && scol >= 0 && scol < p.Ws;
  const bool pstore = q < SP_PX;                         // padding columns store zeros
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(p.x + (int64_t)n * p.xsn, p.xframe_bytes);
  // input row of K-step kh for stem row 2py + r: 4py + 2r + kh (bordered buffer), column 2 scol
  const unsigned avo = pvalid ? (unsigned)(((int64_t)(2 * r) * p.xsh + (int64_t)(2 * scol) * 4 + fg * 8) * 4) : BL_OOB;
  const int rstep = (int)(4 * p.xsh * 4);                // bytes per pooled row (4 input rows)
  const int kstep = (int)(p.xsh * 4);                    // bytes per tap row

  const float am = p.x_amax[n];
  const int ex = f16_scale_exp(am);
  const float sa = ldexpf(1.f, 15 - ex), inv = ldexpf(1.f, ex - 15);
  float* const yn = p.y + (int64_t)n * p.ysn;
  // pool phase: thread -> pooled column j = tid / 16 of the strip, channels 4 (tid % 16) .. +3
  const int pj = tid >> 4, pc = (tid & 15) * 4;
  const bool pout = tid < SP_PC * 16 && px0 + pj < p.Wp;

  f4 raw[SP_K][2];
  auto load_rows = [&](int py) {
#pragma unroll
    for (int kh = 0; kh < SP_K; ++kh) {
      raw[kh][0] = bl_f4(xr, avo, py * rstep + kh * kstep);
      raw[kh][1] = bl_f4(xr, avo + 16, py * rstep + kh * kstep);
    }
  };
  load_rows(0);
  // weights landed (vmcnt(0): the DMA pieces and row 0's loads), slot 2 zeroed (lgkmcnt(0))
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  float ymax = 0.f;

#pragma unroll 1
  for (int py = 0; py < p.Hp; ++py) {
    // split this row's activations (frame scale), then load the next row's
    f16x8 af[SP_K][2];
#pragma unroll
    for (int kh = 0; kh < SP_K; ++kh) {
      unsigned long long p0[2], p1[2];
      split_planes_f16(raw[kh][0], sa, p0);
      split_planes_f16(raw[kh][1], sa, p1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        af[kh][h] = __builtin_bit_cast(f16x8, u64x2{p0[h], p1[h]});
      }
    }
    if (py + 1 < p.Hp) load_rows(py + 1);
    f32x4 acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < SP_K; ++kh) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int nrow = cb * 16 + fr;
        const unsigned char* bp = lds + kh * SP_WSTEP + nrow * 64 + ((fg ^ swzF(nrow)) << 4);
        f16x8 w[2];
        w[0] = *reinterpret_cast<const f16x8*>(bp);
        w[1] = *reinterpret_cast<const f16x8*>(bp + SP_CO * 64);
        // three terms, smallest first (prpe_conv2d's order): a_lo w_hi, a_hi w_lo, a_hi w_hi
        acc[cb] = mfma16(w[0], af[kh][1], acc[cb]);
        acc[cb] = mfma16(w[1], af[kh][0], acc[cb]);
        acc[cb] = mfma16(w[0], af[kh][0], acc[cb]);
      }
    }
    // every wave is done reading the ring (pool of row py - 1) before rows 2py, 2py + 1 replace
    // rows 2py - 3, 2py - 2
    lds_barrier();
    if (pstore) {
      float* const dst = ring + (((2 * py + r) % 3) * SP_SC + c) * SP_CO;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        // epilogue constants of channels cb*16 + 4 fg .. +3 (re-read per row from L1: held across
        // the walk they spilled the split fragments)
        const f4 scv = *reinterpret_cast<const f4*>(p.sc + cb * 16 + fg * 4);
        const f4 biv = *reinterpret_cast<const f4*>(p.bi + cb * 16 + fg * 4);
        f4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float t = fmaf(acc[cb][e] * inv, scv[e], biv[e]);
          v[e] = pvalid && t > 0.f ? t : 0.f;
          ymax = fmaxf(ymax, v[e]);
        }
        *reinterpret_cast<f4*>(dst + rslot(cb * 4 + fg, c)) = v;
      }
    }
    lds_barrier();
    // pool: rows 2py - 1 .. 2py + 1 (ring slots), ring columns 2 pj .. 2 pj + 2
    if (pout) {
      f4 m = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy) {
        const float* src = ring + (((2 * py + dy + 3) % 3) * SP_SC + 2 * pj) * SP_CO;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const f4 v = *reinterpret_cast<const f4*>(src + dx * SP_CO + rslot(pc >> 2, 2 * pj + dx));
#pragma unroll
          for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], v[e]);
        }
      }
      *reinterpret_cast<f4*>(yn + (int64_t)py * p.ysh + (int64_t)(px0 + pj) * p.ysw + pc) = m;
    }
  }
  if (p.y_amax) amax_commit(p.y_amax + n, ymax);
}

}  // namespace

int stem_pool_launch(const StemK& kp, hipStream_t st) {
  hipLaunchKernelGGL(stem_pool_kernel, dim3(kp.nwg), dim3(SP_NW * 64), 0, st, kp);
  return launch_status();
}

}  // namespace prpe_k

extern "C" int prpe_stem_maxpool(const prpe_stem_desc* d, void* stream) {
  using namespace prpe_k;
  if (!d || !d->x || !d->x_amax || !view_ok(&d->y)) return PRPE_EINVAL;
  const prpe_view& y = d->y;
  if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->h % 4 || d->w % 4) return PRPE_EINVAL;
  if (d->k_pad != SP_K * 32 || !d->w_h16 || !d->w_l16 || !d->scale16 || !d->bias) return PRPE_EINVAL;
  if ((uintptr_t)d->x % 16 || (uintptr_t)d->w_h16 % 16 || (uintptr_t)d->w_l16 % 16 || (uintptr_t)d->scale16 % 16 ||
      (uintptr_t)d->bias % 16 || (uintptr_t)y.ptr % 16)
    return PRPE_EINVAL;
  const int Hs = d->h / 2, Ws = d->w / 2, Hp = Hs / 2, Wp = Ws / 2;
  if (y.n != d->n || y.h != Hp || y.w != Wp || y.c != SP_CO || y.sc != 1 || y.sw % 4 || y.sh % 4 || y.sn % 4 ||
      y.sw < 0 || y.sh < 0)
    return PRPE_EINVAL;
  if (d->xsh < (int64_t)(d->w + 8) * 4 || d->xsn < (int64_t)(d->h + 6) * d->xsh || d->xsh % 4 || d->xsn % 4)
    return PRPE_EINVAL;
  const int64_t fb = (int64_t)(d->h + 6) * d->xsh * 4;
  if (fb >= (1LL << 31)) return PRPE_EINVAL;
  {                                                      // not in place (prpe.h)
    uintptr_t ylo, yhi;
    view_span(y, ylo, yhi);
    const uintptr_t xlo = (uintptr_t)d->x, xhi = xlo + (uintptr_t)((d->n - 1) * d->xsn * 4 + fb);
    if (spans_overlap(xlo, xhi, ylo, yhi)) return PRPE_EINVAL;
  }
  StemK kp{};
  kp.x = d->x; kp.xsn = d->xsn; kp.xsh = d->xsh; kp.xframe_bytes = (int)fb;
  kp.x_amax = d->x_amax;
  kp.wh = d->w_h16; kp.wl = d->w_l16; kp.kp = d->k_pad; kp.sc = d->scale16; kp.bi = d->bias;
  kp.y = y.ptr; kp.ysn = y.sn; kp.ysh = y.sh; kp.ysw = y.sw; kp.y_amax = d->y_amax;
  kp.N = d->n; kp.Ws = Ws; kp.Hp = Hp; kp.Wp = Wp;
  kp.strips = (Wp + SP_PC - 1) / SP_PC;
  const int64_t nwg = (int64_t)d->n * kp.strips;
  if (nwg >= (1LL << 31)) return PRPE_EINVAL;
  kp.nwg = (int)nwg;
  return stem_pool_launch(kp, as_stream(stream));
}
