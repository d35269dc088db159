// Memory-bound kernels of the hot path (HBM / L2 bound, VALU, wave64).
//   upconv3x3     : bilinear-upsample o conv3x3 rewrite, stage 2 (interp of per-tap GEMMs;
//                   fused rolling-row kernel, or separable through a workspace)
//   dwconv        : depthwise kxk conv + folded BN + act (+ residual)
//   maxpool       : kxk/s/p max pooling
//   upsample2x    : nearest x2
//   norm_sigmoid  : per-sample per-channel standardisation + sigmoid
//   layernorm     : row LayerNorm (+ReLU)
//   l2norm        : row L2 normalisation
//   dfl_decode    : YOLO head eval decode (DFL softmax-expectation, anchors, strides, sigmoid)
#include "common.h"
#include <stdlib.h>

namespace {

__device__ __forceinline__ int64_t voff(const prpe_view& v, int n, int h, int w, int c) {
  return (int64_t)n * v.sn + (int64_t)h * v.sh + (int64_t)w * v.sw + (int64_t)c * v.sc;
}

// x + (1 - l) a + l b with one fixed rounding sequence (fma((1 - l), a, l * b), then the add):
// every upconv form (fused, producer / consumer, separable) evaluates it identically whatever
// FP contraction the surrounding code would allow
__device__ __forceinline__ float lerp_add(float x, float l, float a, float b) {
  const float t = __builtin_fmaf(1.f - l, a, l * b);
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(t));
  return r;
}

// lerp_add on two channels as packed FP32 math (v_pk_mul_f32 l b, v_pk_fma_f32 (1 - l) a + l b,
// v_pk_add_f32; the scalar l / 1 - l broadcast by op_sel): per lane exactly lerp_add's three IEEE
// operations in the same order, so the packed and scalar forms are bit-identical. Contraction is
// off here so the add is not re-fused with the product (fadd(fma(m, a, l b), x) ->
// fma(m, a, fma(l, b, x)) is legal under contraction).
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v lerp_add2(f2v x, float l, f2v a, f2v b) {
#pragma clang fp contract(off)
  const float ml = 1.f - l;
  const f2v lb = l * b;
  return x + __builtin_elementwise_fma(f2v{ml, ml}, a, lb);
}

// PyTorch upsample_bilinear2d source index (aten/src/ATen/native/UpSample.h semantics):
// align_corners: src = dst * (in-1)/(out-1); else src = max(0, (dst+0.5)*in/out - 0.5).
__device__ __forceinline__ void bilin_src(int dst, int in, int out, int ac, int& i0, int& i1, float& l1) {
  float src;
  if (ac) {
    const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
    src = scale * (float)dst;
  } else {
    const float scale = (float)in / (float)out;
    src = scale * ((float)dst + 0.5f) - 0.5f;
    src = src < 0.f ? 0.f : src;
  }
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 < in - 1 ? i0 + 1 : i0;
  l1 = src - (float)i0;
}

// Launch geometry of the row kernels below: a 1-D grid of rows x chunks blocks, block b ->
// row = b / chunks (one output row (n, oy), decoded once per block on the scalar unit) and
// position (b % chunks) * 256 + threadIdx.x inside the row (pixel-major, channel group
// fastest). All chunks of a row are adjacent in dispatch order, so the blocks in flight cover
// a few consecutive rows (shared interpolation sources stay in L2). Per-thread index math is
// 32-bit.
__device__ __forceinline__ void row_pos(int chunks, int& row, int& j) {
  row = blockIdx.x / chunks;
  j = (blockIdx.x - row * chunks) * 256 + threadIdx.x;
}
struct UpK {
  prpe_view z, y;
  int Co, ac;
  const float* scale; const float* bias; const float* slope; int act;
  int per_row;    // Wo * (Co / VW)
  int chunks;     // ceil(per_row / 256)
  int y_planes;   // write y in the planes format (include/prpe.h, prpe_conv_desc)
  int xcd;        // fused kernel: XCD-contiguous block order
  float* y_amax;  // optional per-frame max|y| slots (a block covers one frame)
};

// Fused one-pass form (no workspace). One thread = VW channels of one output column, for a
// range of R consecutive output rows (block = 256 columns x one row range, the row range is
// block-uniform so the vertical source rows/weights live in SGPRs). The x-interpolated
// rows H_dy[r] = sum_dx valid * lerp_x(Z_{dy,dx}[r], sx(ox+dx-1)) are kept in two rolling
// registers per dy (rows y0 and y0+1 of the current source interval): moving down one output
// row advances the interval by at most one source row when upsampling, so each H row is built
// once per thread (6 L2 loads) instead of once per output row. HBM traffic is the output
// write plus the small z read. Same arithmetic, same order as the separable form.
// Addressing: the frame / source-row / tap-row part of every address is block-uniform
// (scalar base), the per-thread part is a loop-invariant 32-bit element offset (the host
// checks that one frame of z and of y spans < 2^31 elements), so the row loop holds one
// VGPR per load address and the x-interpolation positions are computed once per thread.
constexpr int UP_MAX_R = 256;   // longest row range of one fused-kernel block
struct UpX {        // per-thread x-interpolation of one dx: offsets of columns x0, x1
  int o0, o1;       // element offsets (x * sw + (dx * Co + c0) * sc) inside a z row
  float l1;         // weight of x1
};

template <int VW>
__device__ __forceinline__ void up_hrow(const float* __restrict__ zrow, const UpX (&ux)[3], unsigned xvalid,
                                       float (&h)[VW], int sc) {
#pragma unroll
  for (int v = 0; v < VW; ++v) h[v] = 0.f;
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    if (!((xvalid >> dx) & 1u)) continue;
    const float lx = ux[dx].l1;
    const float* a = zrow + ux[dx].o0;
    const float* b = zrow + ux[dx].o1;
    if constexpr (VW == 4) {
      const float4 A = *reinterpret_cast<const float4*>(a), B = *reinterpret_cast<const float4*>(b);
      h[0] = lerp_add(h[0], lx, A.x, B.x);
      h[1] = lerp_add(h[1], lx, A.y, B.y);
      h[2] = lerp_add(h[2], lx, A.z, B.z);
      h[3] = lerp_add(h[3], lx, A.w, B.w);
    } else {
      h[0] = lerp_add(h[0], lx, a[0], b[0]);
    }
  }
}

// ACT >= 0: the epilogue activation as a compile-time constant (one activation's code and
// registers per instantiation); -1 reads p.act
// ABL (diagnostic builds, PRPE_UPCONV_ABL): 1 = no z loads (H rows from registers), 2 = no y
// stores (kept live through a never-true condition), 3 = both
template <int VW, int ACT, int ABL = 0>
__global__ __launch_bounds__(256) void upconv_fused_kernel(UpK p, int R, int rblocks) {
  // XCD-aware order (p.xcd): consecutive chunks share their z source columns, so each XCD
  // takes a contiguous range of the logical blocks instead of every 8th one
  const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int chunk = bid % p.chunks;
  const int rb_n = bid / p.chunks;
  const int n = rb_n / rblocks, oy0 = (rb_n - n * rblocks) * R;
  const int j = chunk * 256 + threadIdx.x;
  const int Ho = p.y.h, Hi = p.z.h, Wo = p.y.w, Wi = p.z.w;
  const int oy1 = oy0 + R < Ho ? oy0 + R : Ho;
  // vertical source rows / weights of the block's output rows (+1 halo row each side), once
  // per block into LDS: the row loop reads them as wave-uniform scalars (readfirstlane)
  __shared__ int ty0[UP_MAX_R + 2];
  __shared__ float tly[UP_MAX_R + 2];
  for (int t = threadIdx.x; t < oy1 - oy0 + 2; t += 256) {
    const int yy = oy0 - 1 + t;
    int y0 = -1, y1; float ly = 0.f;
    if ((unsigned)yy < (unsigned)Ho) bilin_src(yy, Hi, Ho, p.ac, y0, y1, ly);
    ty0[t] = y0;
    tly[t] = ly;
  }
  __syncthreads();
  // lanes past the row stay for the block's max|y| reduction (amax_commit) but do no work
  const bool jl = j < p.per_row;
  if (!jl && !p.y_amax) return;
  const int cgroups = p.Co / VW;
  const int ox = j / cgroups, c0 = (j - ox * cgroups) * VW;
  const int zsw = (int)p.z.sw, zsc = (int)p.z.sc;

  UpX ux[3];
  unsigned xvalid = 0;
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int xx = ox + dx - 1;
    int x0 = 0, x1 = 0; float lx = 0.f;
    if ((unsigned)xx < (unsigned)Wo) {
      bilin_src(xx, Wi, Wo, p.ac, x0, x1, lx);
      xvalid |= 1u << dx;
    }
    const int co = (dx * p.Co + c0) * zsc;
    ux[dx].o0 = x0 * zsw + co;
    ux[dx].o1 = x1 * zsw + co;
    ux[dx].l1 = lx;
  }
  float sc[VW], bi[VW], sl[VW];
#pragma unroll
  for (int v = 0; v < VW; ++v) {
    sc[v] = p.scale ? p.scale[c0 + v] : 1.f;
    bi[v] = p.bias ? p.bias[c0 + v] : 0.f;
    sl[v] = p.slope ? p.slope[c0 + v] : 0.f;
  }
  const float* zn = p.z.ptr + (int64_t)n * p.z.sn;                       // block-uniform
  const int64_t tap_row = (int64_t)3 * p.Co * p.z.sc;                    // dy step in channels
  float* yn = p.y.ptr + (int64_t)n * p.y.sn;                             // block-uniform
  const int yo = ox * (int)p.y.sw + c0 * (int)p.y.sc;                    // per thread
  float hA[3][VW], hB[3][VW];
  int cur[3] = {-2, -2, -2};
  float ym = 0.f;
  for (int oy = oy0; oy < (jl ? oy1 : oy0); ++oy) {
    float acc[VW];
#pragma unroll
    for (int v = 0; v < VW; ++v) acc[v] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      // row yy = oy + dy - 1 is table entry oy - oy0 + dy (y0 = -1: outside the image)
      const int y0 = __builtin_amdgcn_readfirstlane(ty0[oy - oy0 + dy]);
      if (y0 < 0) continue;
      const float ly = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(
                                                     __builtin_bit_cast(int, tly[oy - oy0 + dy])));
      const int y1 = y0 < Hi - 1 ? y0 + 1 : y0;
      if (y0 != cur[dy]) {
        const float* zt = zn + dy * tap_row;
        if constexpr ((ABL & 1) != 0) {
#pragma unroll
          for (int v = 0; v < VW; ++v) {
            hA[dy][v] = hB[dy][v];
            hB[dy][v] = ux[v % 3].l1 * (float)(y1 + v);
          }
        } else {
          if (y0 == cur[dy] + 1) {
#pragma unroll
            for (int v = 0; v < VW; ++v) hA[dy][v] = hB[dy][v];
          } else {
            up_hrow<VW>(zt + (int64_t)y0 * p.z.sh, ux, xvalid, hA[dy], zsc);
          }
          up_hrow<VW>(zt + (int64_t)y1 * p.z.sh, ux, xvalid, hB[dy], zsc);
        }
        cur[dy] = y0;
      }
#pragma unroll
      for (int v = 0; v < VW; ++v) acc[v] = lerp_add(acc[v], ly, hA[dy][v], hB[dy][v]);
    }
    float out[VW];
    if constexpr (VW == 4) {
      f32x4 pre;
#pragma unroll
      for (int v = 0; v < 4; ++v) pre[v] = acc[v] * sc[v] + bi[v];
      const f32x4 o4 = apply_act4(pre, ACT >= 0 ? ACT : p.act, f32x4{sl[0], sl[1], sl[2], sl[3]});
#pragma unroll
      for (int v = 0; v < 4; ++v) out[v] = o4[v];
    } else {
#pragma unroll
      for (int v = 0; v < VW; ++v) out[v] = apply_act(acc[v] * sc[v] + bi[v], ACT >= 0 ? ACT : p.act, sl[v]);
    }
#pragma unroll
    for (int v = 0; v < VW; ++v) ym = fmaxf(ym, fabsf(out[v]));
    float* y = yn + (int64_t)oy * p.y.sh + yo;
    if constexpr ((ABL & 2) != 0) {
      if (out[0] + out[VW - 1] == 12345.678f) y[0] = out[0];
      continue;
    }
    // non-temporal stores: the output is not re-read here, and z's lines stay in L2
    // (-6 % on the adapters' shapes, tools/upconv_bench.py)
    if constexpr (VW == 4) {
      if (p.y_planes) {
        // channel group c0 / 8 of the pixel: hi[8] then lo[8] (bf16 RNE two-plane split)
        store_planes4<true>(reinterpret_cast<uint16_t*>(y - c0), c0, f32x4{out[0], out[1], out[2], out[3]});
        continue;
      }
      if (p.y.sc == 1) {
        __builtin_nontemporal_store(f32x4{out[0], out[1], out[2], out[3]}, reinterpret_cast<f32x4*>(y));
        continue;
      }
    }
#pragma unroll
    for (int v = 0; v < VW; ++v) y[(int64_t)v * p.y.sc] = out[v];
  }
  if (p.y_amax) amax_commit(p.y_amax + n, ym);
}

// LDS-DMA form (round 3; the automatic choice for VW = 4 whenever its geometry rules hold). Why:
// gfx950 has one vmcnt for a wave's loads AND stores, so in the fused kernel every H-row reload
// (6 dependent L2 loads per tap row, ~once per source interval) also waits for the output
// stores issued before it: loads and stores serialise (diagnostic builds: no loads 0.88 ms, no
// stores 0.84, full 1.56 at the face-YOLO shape, bs = 64). Here the z rows reach LDS by
// buffer-descriptor LDS-DMA, one source row ahead, issued right after the block barrier that
// brings the previous row into use: by the time a row is read, at least UPD_MIN stores (output
// rows x stores per row) were issued after its DMA, so `vmcnt(that many)` covers the DMA and
// never the recent stores. The H rows and the output follow the fused kernel's arithmetic
// exactly (same lerp_add sequence, same epilogue): bit-identical results.
// Block: frame n, output rows [oy0, oy1), 32 output columns x 32 channels (thread = 4 channels of
// one column; 8 threads = one pixel's 128-B line, so a wave stores 8 full lines), the source
// window of the block's columns (at most UPD_NSC source columns) x 9 taps x 32 channels per
// source row in a ring of UPD_RING rows (128-B segments, 8 lanes per segment).
constexpr int UPD_W = 32, UPD_C = 32, UPD_NSC = 8, UPD_RING = 4;
constexpr int UPD_SEG = UPD_NSC * 9;                  // 128-B segments per source row
constexpr int UPD_NI = (UPD_SEG + 7) / 8;             // 1-KiB DMA instructions per source row
constexpr int UPD_MIN = 4;                            // output rows between a row's DMA and its use

template <int ACT, bool PL>
__global__ __launch_bounds__(256) void upconv_dma_kernel(UpK p, int R, int rblocks, int ctiles, int cblocks) {
  __shared__ __attribute__((aligned(1024))) float ring[UPD_RING][UPD_NI * 256];
  __shared__ int ty0[UP_MAX_R + 2];
  __shared__ float tly[UP_MAX_R + 2];
  __shared__ int thi[UP_MAX_R];                        // hi_at(oy) per output row (below)
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  int t = bid;
  const int cb = t % cblocks;
  t /= cblocks;
  const int ct = t % ctiles;
  t /= ctiles;
  const int rbk = t % rblocks;
  const int n = t / rblocks;
  const int Ho = p.y.h, Hi = p.z.h, Wo = p.y.w, Wi = p.z.w;
  const int oy0 = rbk * R, oy1 = oy0 + R < Ho ? oy0 + R : Ho;
  const int ox0 = ct * UPD_W, c0 = cb * UPD_C;
  for (int e = threadIdx.x; e < oy1 - oy0 + 2; e += 256) {
    const int yy = oy0 - 1 + e;
    int y0 = -1, y1;
    float ly = 0.f;
    if ((unsigned)yy < (unsigned)Ho) bilin_src(yy, Hi, Ho, p.ac, y0, y1, ly);
    ty0[e] = y0;
    tly[e] = ly;
  }
  // source column window of the block (host-checked to span <= UPD_NSC columns)
  int xs_lo, xs_hi, tmp;
  float ltmp;
  bilin_src(ox0 > 0 ? ox0 - 1 : 0, Wi, Wo, p.ac, xs_lo, tmp, ltmp);
  bilin_src(ox0 + UPD_W < Wo ? ox0 + UPD_W : Wo - 1, Wi, Wo, p.ac, tmp, xs_hi, ltmp);
  const int nsc = xs_hi - xs_lo + 1;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // DMA: segment s = (source column j, tap) -> 128 B = channels c0 .. c0+31 of that tap map;
  // instruction i of a row moves segments 8i .. 8i+7 (lane -> segment 8i + lane/8, 16 B each)
  const float* zn = p.z.ptr + (int64_t)n * p.z.sn;
  const int zbytes = (int)(((int64_t)(Hi - 1) * p.z.sh + (int64_t)(Wi - 1) * p.z.sw + 9 * p.Co) * 4);
  const __amdgpu_buffer_rsrc_t zr = buf_rsrc(zn, zbytes);
  unsigned dvo[(UPD_NI + 3) / 4];
#pragma unroll
  for (int k = 0; k < (UPD_NI + 3) / 4; ++k) {
    const int i = wave + 4 * k;
    const int sg = i * 8 + (lane >> 3);
    const int j = sg / 9, tp = sg - j * 9;
    dvo[k] = (i < UPD_NI && j < nsc)
                 ? (unsigned)((((int64_t)(xs_lo + j) * p.z.sw + tp * p.Co + c0) + (lane & 7) * 4) * 4)
                 : BL_OOB;
  }
  auto issue_row = [&](int r) {
#pragma unroll
    for (int k = 0; k < (UPD_NI + 3) / 4; ++k) {
      const int i = wave + 4 * k;
      if (i < UPD_NI)
        bl_lds16(zr, reinterpret_cast<unsigned char*>(ring[r % UPD_RING]) + i * 1024, dvo[k],
                 (int)((int64_t)r * p.z.sh * 4));
    }
  };

  // this thread: output column ox, channels c0 + 4 cg .. +3
  const int col = tid >> 3, cg = tid & 7;
  const int ox = ox0 + col;
  const bool live = ox < Wo;                          // Co % 32 == 0 (host-checked)
  const bool wlive = __builtin_amdgcn_ballot_w64(live) != 0;   // wave-uniform
  int lo[3], l1[3];
  float lx[3];
  unsigned xvalid = 0;
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int xx = ox + dx - 1;
    int x0 = xs_lo, x1 = xs_lo;
    float l = 0.f;
    if (live && (unsigned)xx < (unsigned)Wo) {
      bilin_src(xx, Wi, Wo, p.ac, x0, x1, l);
      xvalid |= 1u << dx;
    }
    // float offset of (column, tap dy = 0, dx) in a ring row; the tap row dy adds 3 dy segments
    lo[dx] = ((x0 - xs_lo) * 9 + dx) * 32 + cg * 4;
    l1[dx] = ((x1 - xs_lo) * 9 + dx) * 32 + cg * 4;
    lx[dx] = l;
  }
  float sc[4], bi[4], sl[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int c = c0 + cg * 4 + v;
    sc[v] = p.scale ? p.scale[c] : 1.f;
    bi[v] = p.bias ? p.bias[c] : 0.f;
    sl[v] = p.slope ? p.slope[c] : 0.f;
  }
  // The ring reads are inline asm (all six of an H row, one lgkmcnt wait): as plain loads the
  // compiler put `s_waitcnt vmcnt(0)` before every one of them (an LDS read after an LDS-DMA it
  // cannot tell apart waits for the youngest DMA), i.e. each H-row rebuild drained every store
  // the wave had in flight -- the serialisation this kernel exists to avoid. The rows read here
  // are covered by the counted `vmcnt` + barrier at the event that brought them into use (see
  // above); a column outside the image reads an in-ring address (x0 = x1 = xs_lo) and skips its
  // lerp, as before.
  const unsigned ring_lds = (unsigned)(uintptr_t)(lds_ptr_t)&ring[0][0];
  auto hrow = [&](int r, int dy, f2v (&h)[2]) {
    const unsigned rr = ring_lds + (unsigned)(((r % UPD_RING) * UPD_NI * 256 + dy * 3 * 32) * 4);
    f32x4 A0, B0, A1, B1, A2, B2;
    asm volatile(
        "ds_read_b128 %0, %6\n\tds_read_b128 %1, %7\n\tds_read_b128 %2, %8\n\t"
        "ds_read_b128 %3, %9\n\tds_read_b128 %4, %10\n\tds_read_b128 %5, %11\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(A0), "=&v"(B0), "=&v"(A1), "=&v"(B1), "=&v"(A2), "=&v"(B2)
        : "v"(rr + lo[0] * 4), "v"(rr + l1[0] * 4), "v"(rr + lo[1] * 4), "v"(rr + l1[1] * 4), "v"(rr + lo[2] * 4),
          "v"(rr + l1[2] * 4));
    f2v h0 = {0.f, 0.f}, h1 = {0.f, 0.f};
    if (xvalid & 1u) { h0 = lerp_add2(h0, lx[0], A0.xy, B0.xy); h1 = lerp_add2(h1, lx[0], A0.zw, B0.zw); }
    if (xvalid & 2u) { h0 = lerp_add2(h0, lx[1], A1.xy, B1.xy); h1 = lerp_add2(h1, lx[1], A1.zw, B1.zw); }
    if (xvalid & 4u) { h0 = lerp_add2(h0, lx[2], A2.xy, B2.xy); h1 = lerp_add2(h1, lx[2], A2.zw, B2.zw); }
    h[0] = h0;
    h[1] = h1;
  };
  __syncthreads();                                    // the row tables
  // rows in use for output row oy: [y0 of row oy-1 (or oy), y1 of row oy+1]; hi_at = the top one
  auto hi_at = [&](int oy) {
    int h = -1;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int y0 = ty0[oy - oy0 + dy];
      if (y0 >= 0) h = y0 < Hi - 1 ? y0 + 1 : y0;
    }
    return h;
  };
  // ... tabulated once per block (one LDS read per output row in the loop instead of three and
  // the selects; the row loop is VALU-bound: ~160 VALU per thread and row, profiles/r04_pmc_upconv_conv.txt)
  for (int e = threadIdx.x; e < oy1 - oy0; e += 256) thi[e] = hi_at(oy0 + e);
  __syncthreads();
  int lo_row = Hi;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int y0 = ty0[dy];
    if (y0 >= 0 && y0 < lo_row) lo_row = y0;
  }
  int issued = __builtin_amdgcn_readfirstlane(hi_at(oy0));
  for (int r = __builtin_amdgcn_readfirstlane(lo_row); r <= issued; ++r) issue_row(r);
  if (issued + 1 < Hi) issue_row(++issued);           // one row ahead
  { __builtin_amdgcn_sched_barrier(0); asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory"); __builtin_amdgcn_sched_barrier(0); }
  int in_use = hi_at(oy0);

  const int yo = ox * (int)p.y.sw + (c0 + cg * 4) * (int)p.y.sc;
  float* yn = p.y.ptr + (int64_t)n * p.y.sn;
  // x-interpolated rows y0 (A) and y0 + 1 (B) of each dy in two register slots whose roles a
  // wave-uniform parity bit says (par 0: A = h0, B = h1): moving down one source row flips the
  // parity and refills the old A slot, so no register copies (the hA = hB rolling form made the
  // compiler move 8 registers per dy and row on every path)
  f2v h0[3][2], h1[3][2];
  int cur[3] = {-2, -2, -2};
  int par[3] = {0, 0, 0};
  float ym = 0.f;
  for (int oy = oy0; oy < oy1; ++oy) {
    const int need = __builtin_amdgcn_readfirstlane(thi[oy - oy0]);
    if (need > in_use) {
      // the row(s) coming into use were DMA'd at the previous such event, >= UPD_MIN output rows
      // (stores) ago: wait for everything older than those stores, then publish every wave's
      // pieces. A wave with no live column issues no stores: it waits for all of its DMA.
      if (!wlive) { __builtin_amdgcn_sched_barrier(0); asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory"); __builtin_amdgcn_sched_barrier(0); }
      else if constexpr (PL) { __builtin_amdgcn_sched_barrier(0); asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory"); __builtin_amdgcn_sched_barrier(0); }
      else { __builtin_amdgcn_sched_barrier(0); asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory"); __builtin_amdgcn_sched_barrier(0); }
      in_use = need;
      while (issued < need + 1 && issued + 1 < Hi) issue_row(++issued);   // one row ahead again
    }
    f2v acc[2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int y0 = __builtin_amdgcn_readfirstlane(ty0[oy - oy0 + dy]);
      if (y0 < 0) continue;
      const float ly = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(
                                                     __builtin_bit_cast(int, tly[oy - oy0 + dy])));
      const int y1 = y0 < Hi - 1 ? y0 + 1 : y0;
      if (y0 != cur[dy]) {
        if (y0 == cur[dy] + 1) {
          par[dy] ^= 1;                                // old B (row y0) is the new A
        } else if (par[dy]) {
          hrow(y0, dy, h1[dy]);
        } else {
          hrow(y0, dy, h0[dy]);
        }
        if (par[dy]) hrow(y1, dy, h0[dy]);             // B: the slot A does not use
        else hrow(y1, dy, h1[dy]);
        cur[dy] = y0;
      }
      if (par[dy]) {
#pragma unroll
        for (int q = 0; q < 2; ++q) acc[q] = lerp_add2(acc[q], ly, h1[dy][q], h0[dy][q]);
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q) acc[q] = lerp_add2(acc[q], ly, h0[dy][q], h1[dy][q]);
      }
    }
    if (!live) continue;
    f32x4 pre;
#pragma unroll
    for (int v = 0; v < 4; ++v) pre[v] = acc[v >> 1][v & 1] * sc[v] + bi[v];
    const f32x4 o4 = apply_act4(pre, ACT >= 0 ? ACT : p.act, f32x4{sl[0], sl[1], sl[2], sl[3]});
    const float out[4] = {o4[0], o4[1], o4[2], o4[3]};
    ym = fmaxf(ym, amax4(o4));
    float* y = yn + (int64_t)oy * p.y.sh + yo;
    if constexpr (PL)
      store_planes4<true>(reinterpret_cast<uint16_t*>(y - (c0 + cg * 4)), c0 + cg * 4,
                          f32x4{out[0], out[1], out[2], out[3]});
    else
      __builtin_nontemporal_store(f32x4{out[0], out[1], out[2], out[3]}, reinterpret_cast<f32x4*>(y));
  }
  if (p.y_amax) amax_commit(p.y_amax + n, ym);
}

// Unit-scale form (round 6): the Co <= 4 tap rewrites (Engine.conv3x3_smallco: ViTPose adapter.10
// 128 -> 3, face-YOLO adapter.16 64 -> 3) run prpe_upconv3x3 with the output grid = the input grid
// and align_corners, where every interpolation weight is 0 and every source index exact: the
// "upconv" is the plain 3x3 tap sum
//   y[n, oy, ox, c] = EPI( sum_dy sum_dx z[n, oy+dy-1, ox+dx-1, (3 dy + dx) Co + c] )
// over the taps inside the image. The rolling-row kernel took 0.86 ms for the ViT one (1.36 GB of z
// at bs = 256, 1.6 TB/s: one thread per channel); a thread per pixel gathering its nine Co-float
// slices took 1.01 ms (each dword load of a wave touched 64 cache lines at the 9 Co-float pixel
// pitch; profiles/r06_layer_profile_unit_gather.txt). Here one wave walks a 64-pixel column strip
// down a chunk of R output rows: each z row's segment (66 pixels x 9 Co floats, contiguous) is read
// with lane-contiguous dword loads (two cache lines per instruction), one row ahead in registers,
// staged through the wave's LDS slice, and every lane takes the 27 values its pixel needs (the
// three dy slices of the row feed three output rows in flight). Sums in the rolling-row kernel's
// order (per dy its dx taps, then the dy rows, each step an IEEE add), the same epilogue
// expression: the same bits for finite z (the general form adds 0 * (the next column), so a
// non-finite z one column outside a tap's support made its sum NaN; here it does not). A block
// (4 waves) is one frame: the per-frame max|y| slot.
constexpr int UPU_R = 32;                               // output rows per chunk
template <int CO>
__global__ __launch_bounds__(256) void upconv_unit_kernel(UpK p, int nstrip, int ngroups, int rchunks) {
  constexpr int ZP = 9 * CO;                            // floats per z pixel
  constexpr int SEG = 66 * ZP;                          // one row segment: pixels x0 - 1 .. x0 + 64
  constexpr int NL = (SEG + 63) / 64;                   // dword loads per lane and row
  __shared__ float seg_all[4][NL * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int t = blockIdx.x;
  const int sg = t % ngroups;
  t /= ngroups;
  const int rc = t % rchunks;
  const int n = t / rchunks;
  const int H = p.y.h, W = p.y.w;
  const int strip = sg * 4 + wave;
  float ym = 0.f;
  if (strip < nstrip) {
    float* seg = seg_all[wave];
    const int x0 = strip * 64, x = x0 + lane;
    const bool live = x < W;
    const int oy0 = rc * UPU_R, oy1 = oy0 + UPU_R < H ? oy0 + UPU_R : H;
    const int r0 = oy0 > 0 ? oy0 - 1 : 0, r1 = oy1 < H ? oy1 : H - 1;
    const float* zn = p.z.ptr + (int64_t)n * p.z.sn;
    // this lane's loads of a row: segment index j = lane + 64 k -> z pixel x0 - 1 + j / ZP
    int jo[NL];
    bool jv[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const int j = lane + 64 * k;
      const int px = x0 - 1 + j / ZP;
      jv[k] = j < SEG && px >= 0 && px < W;
      jo[k] = (x0 - 1) * ZP + j;                        // float offset inside the z row
    }
    float nxt[NL];
    auto load_row = [&](int r) {
      const float* zr = zn + (int64_t)r * p.z.sh;
#pragma unroll
      for (int k = 0; k < NL; ++k) nxt[k] = jv[k] ? zr[jo[k]] : 0.f;
    };
    float scv[CO], biv[CO], slv[CO];
#pragma unroll
    for (int c = 0; c < CO; ++c) {
      scv[c] = p.scale ? p.scale[c] : 1.f;
      biv[c] = p.bias ? p.bias[c] : 0.f;
      slv[c] = p.slope ? p.slope[c] : 0.f;
    }
    auto add = [](float a, float b) {
      float r;
      asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
      return r;
    };
    auto store = [&](int o, const float (&acc)[CO]) {
      if (!live) return;
      float* y = p.y.ptr + (int64_t)n * p.y.sn + (int64_t)o * p.y.sh + (int64_t)x * p.y.sw;
#pragma unroll
      for (int c = 0; c < CO; ++c) {
        const float out = apply_act(acc[c] * scv[c] + biv[c], p.act, slv[c]);
        ym = fmaxf(ym, fabsf(out));
        y[(int64_t)c * p.y.sc] = out;
      }
    };
    float accA[CO], accB[CO];                           // outputs r - 1 and r
#pragma unroll
    for (int c = 0; c < CO; ++c) accA[c] = accB[c] = 0.f;
    load_row(r0);
    for (int r = r0; r <= r1; ++r) {
      // the row into the wave's LDS slice (every lane's previous reads retired first), then the
      // next row's loads in flight while this one is summed
      __builtin_amdgcn_s_waitcnt(0xc07f);              // lgkmcnt(0): last row's ds_reads done
#pragma unroll
      for (int k = 0; k < NL; ++k) seg[lane + 64 * k] = nxt[k];
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      if (r < r1) load_row(r + 1);
      float h[3][CO];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
#pragma unroll
        for (int c = 0; c < CO; ++c) h[dy][c] = 0.f;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int xx = x + dx - 1;
          if ((unsigned)xx >= (unsigned)W) continue;
          const float* sp = seg + (lane + dx) * ZP + (dy * 3 + dx) * CO;
#pragma unroll
          for (int c = 0; c < CO; ++c) h[dy][c] = add(h[dy][c], sp[c]);
        }
      }
      // dy = 2 -> output r - 1 (complete), dy = 1 -> output r, dy = 0 -> output r + 1 (first term)
      if (r >= 1) {
#pragma unroll
        for (int c = 0; c < CO; ++c) accA[c] = add(accA[c], h[2][c]);
        if (r - 1 >= oy0) store(r - 1, accA);
      }
      float accC[CO];
#pragma unroll
      for (int c = 0; c < CO; ++c) {
        accB[c] = add(accB[c], h[1][c]);
        accC[c] = add(0.f, h[0][c]);
      }
#pragma unroll
      for (int c = 0; c < CO; ++c) {
        accA[c] = accB[c];
        accB[c] = accC[c];
      }
    }
    if (oy1 == H) store(H - 1, accA);                   // the last row has no dy = 2 term
  }
  if (p.y_amax) amax_commit(p.y_amax + n, ym);
}

// Separable form of the same sum (6 loads per output instead of 36):
//   H[n][dy][r][ox][c] = sum_dx valid(ox+dx-1) * lerp_x(Z_{dy,dx}[n, r, :, c], sx(ox+dx-1))
//   y[n][oy][ox][c]    = EPI( sum_dy valid(oy+dy-1) * lerp_y(H[n][dy][:, ox, c], sy(oy+dy-1)) )
// H is 3*Hi/Ho of the output's size and is re-read from L2 by every output row using it.
template <int VW>
__global__ __launch_bounds__(256) void upconv_h_kernel(UpK p, float* __restrict__ H) {
  int row, j;
  row_pos(p.chunks, row, j);
  if (j >= p.per_row) return;
  const int cgroups = p.Co / VW;
  const int ox = j / cgroups, cg = j - ox * cgroups;
  const int Wo = p.y.w, Hi = p.z.h, Wi = p.z.w;
  // row = (n*3 + dy)*Hi + r
  const int nd = row / Hi, r = row - nd * Hi;
  const int n = nd / 3, dy = nd - n * 3;
  const int c0 = cg * VW;
  float acc[VW];
#pragma unroll
  for (int v = 0; v < VW; ++v) acc[v] = 0.f;
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int xx = ox + dx - 1;
    if ((unsigned)xx >= (unsigned)Wo) continue;
    int x0, x1; float lx;
    bilin_src(xx, Wi, Wo, p.ac, x0, x1, lx);
    const float* z = p.z.ptr + (int64_t)n * p.z.sn + (int64_t)r * p.z.sh + (int64_t)((dy * 3 + dx) * p.Co + c0) * p.z.sc;
    const float* a = z + (int64_t)x0 * p.z.sw;
    const float* b = z + (int64_t)x1 * p.z.sw;
    if constexpr (VW == 4) {
      const float4 A = *reinterpret_cast<const float4*>(a), B = *reinterpret_cast<const float4*>(b);
      acc[0] = lerp_add(acc[0], lx, A.x, B.x);
      acc[1] = lerp_add(acc[1], lx, A.y, B.y);
      acc[2] = lerp_add(acc[2], lx, A.z, B.z);
      acc[3] = lerp_add(acc[3], lx, A.w, B.w);
    } else {
      acc[0] = lerp_add(acc[0], lx, a[0], b[0]);
    }
  }
  float* h = H + ((int64_t)row * Wo + ox) * p.Co + c0;
  if constexpr (VW == 4) *reinterpret_cast<float4*>(h) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  else h[0] = acc[0];
}

template <int VW>
__global__ __launch_bounds__(256) void upconv_out_kernel(UpK p, const float* __restrict__ H) {
  int row, j;
  row_pos(p.chunks, row, j);
  if (j >= p.per_row) return;
  const int cgroups = p.Co / VW;
  const int ox = j / cgroups, cg = j - ox * cgroups;
  const int Ho = p.y.h, Wo = p.y.w, Hi = p.z.h;
  const int n = row / Ho, oy = row - n * Ho;
  const int c0 = cg * VW;
  float acc[VW];
#pragma unroll
  for (int v = 0; v < VW; ++v) acc[v] = 0.f;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int yy = oy + dy - 1;
    if ((unsigned)yy >= (unsigned)Ho) continue;
    int y0, y1; float ly;
    bilin_src(yy, Hi, Ho, p.ac, y0, y1, ly);
    const float* hb = H + (((int64_t)n * 3 + dy) * Hi) * Wo * p.Co + (int64_t)ox * p.Co + c0;
    const float* a = hb + (int64_t)y0 * Wo * p.Co;
    const float* b = hb + (int64_t)y1 * Wo * p.Co;
    if constexpr (VW == 4) {
      const float4 A = *reinterpret_cast<const float4*>(a), B = *reinterpret_cast<const float4*>(b);
      acc[0] = lerp_add(acc[0], ly, A.x, B.x);
      acc[1] = lerp_add(acc[1], ly, A.y, B.y);
      acc[2] = lerp_add(acc[2], ly, A.z, B.z);
      acc[3] = lerp_add(acc[3], ly, A.w, B.w);
    } else {
      acc[0] = lerp_add(acc[0], ly, a[0], b[0]);
    }
  }
  float out[VW];
#pragma unroll
  for (int v = 0; v < VW; ++v) {
    const int co = c0 + v;
    const float s = p.scale ? p.scale[co] : 1.f;
    const float bb = p.bias ? p.bias[co] : 0.f;
    out[v] = apply_act(acc[v] * s + bb, p.act, p.slope ? p.slope[co] : 0.f);
  }
  float* y = p.y.ptr + voff(p.y, n, oy, ox, c0);
  if constexpr (VW == 4) {
    if (p.y.sc == 1) {
      *reinterpret_cast<float4*>(y) = make_float4(out[0], out[1], out[2], out[3]);
      return;
    }
  }
#pragma unroll
  for (int v = 0; v < VW; ++v) y[(int64_t)v * p.y.sc] = out[v];
}

// ------------------------------------------------------------------------- dwconv
struct DwK {
  prpe_view x, y, r;
  const float* w; int k, stride, pad;
  const float* scale; const float* bias; int act;
  int per_row, chunks;
};
__global__ __launch_bounds__(256) void dwconv_kernel(DwK p) {
  int row, j;
  row_pos(p.chunks, row, j);
  if (j >= p.per_row) return;
  const int C = p.y.c;
  const int ow = j / C, c = j - ow * C;
  const int n = row / p.y.h, oh = row - n * p.y.h;
  float acc = 0.f;
  const float* wc = p.w + (int64_t)c * p.k * p.k;
  for (int kh = 0; kh < p.k; ++kh) {
    const int ih = oh * p.stride - p.pad + kh;
    if ((unsigned)ih >= (unsigned)p.x.h) continue;
    for (int kw = 0; kw < p.k; ++kw) {
      const int iw = ow * p.stride - p.pad + kw;
      if ((unsigned)iw >= (unsigned)p.x.w) continue;
      acc += p.x.ptr[voff(p.x, n, ih, iw, c)] * wc[kh * p.k + kw];
    }
  }
  float v = acc * (p.scale ? p.scale[c] : 1.f) + (p.bias ? p.bias[c] : 0.f);
  v = apply_act(v, p.act, 0.f);
  if (p.r.ptr) v += p.r.ptr[voff(p.r, n, oh, ow, c)];
  p.y.ptr[voff(p.y, n, oh, ow, c)] = v;
}

// ------------------------------------------------------------------------- maxpool
struct PoolK { prpe_view x, y; int k, stride, pad; int per_row, chunks; };
typedef float f4v __attribute__((ext_vector_type(4)));
template <int VW>
__global__ __launch_bounds__(256) void maxpool_kernel(PoolK p) {
  int row, j;
  row_pos(p.chunks, row, j);
  if (j >= p.per_row) return;
  const int cg = p.y.c / VW;
  const int ow = j / cg, c = (j - ow * cg) * VW;
  const int n = row / p.y.h, oh = row - n * p.y.h;
  float m[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) m[e] = -INFINITY;
  for (int kh = 0; kh < p.k; ++kh) {
    const int ih = oh * p.stride - p.pad + kh;
    if ((unsigned)ih >= (unsigned)p.x.h) continue;
    for (int kw = 0; kw < p.k; ++kw) {
      const int iw = ow * p.stride - p.pad + kw;
      if ((unsigned)iw >= (unsigned)p.x.w) continue;
      const float* src = p.x.ptr + voff(p.x, n, ih, iw, c);
      float v[VW];
      if constexpr (VW == 4) {
        const f4v q = *reinterpret_cast<const f4v*>(src);
        v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
      } else {
        v[0] = src[0];
      }
#pragma unroll
      for (int e = 0; e < VW; ++e) m[e] = (v[e] > m[e] || v[e] != v[e]) ? v[e] : m[e];   // NaN propagates like torch
    }
  }
  float* dst = p.y.ptr + voff(p.y, n, oh, ow, c);
  if constexpr (VW == 4) *reinterpret_cast<f4v*>(dst) = f4v{m[0], m[1], m[2], m[3]};
  else dst[0] = m[0];
}

struct Up2K { prpe_view x, y; int per_row, chunks; };
__global__ __launch_bounds__(256) void upsample2x_kernel(Up2K p) {
  int row, j;
  row_pos(p.chunks, row, j);
  if (j >= p.per_row) return;
  const int C = p.y.c;
  const int ow = j / C, c = j - ow * C;
  const int n = row / p.y.h, oh = row - n * p.y.h;
  p.y.ptr[voff(p.y, n, oh, ow, c)] = p.x.ptr[voff(p.x, n, oh >> 1, ow >> 1, c)];
}

// ------------------------------------------------------------------------- norm_sigmoid
// one workgroup per sample; channels <= 4; double accumulation (two passes)
// One block of NS_T threads per sample; every pass covers all C <= 4 channels at once (a
// pixel's channels are adjacent in NHWC): sums, centred sums, then normalise + sigmoid. The
// pixel walk is incremental (no per-element division). Partial sums in fp64, as before.
constexpr int NS_T = 1024;
__global__ __launch_bounds__(NS_T) void norm_sigmoid_kernel(prpe_view x, prpe_view y) {
  constexpr int NWV = NS_T / 64;
  const int n = blockIdx.x;
  const int C = x.c, W = x.w, HW = x.h * x.w;
  __shared__ double red[NWV][8];
  __shared__ float stat[4][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* xn = x.ptr + (int64_t)n * x.sn;
  const int h0 = (int)threadIdx.x / W, w0 = (int)threadIdx.x - h0 * W;
  const int dh = NS_T / W, dw = NS_T - dh * W;                 // dw < W: at most one carry
  // pass 1: per-channel sums -> means
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  for (int i = threadIdx.x, h = h0, w = w0; i < HW; i += NS_T) {
    const float* px = xn + (int64_t)h * x.sh + (int64_t)w * x.sw;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < C) s[c] += px[(int64_t)c * x.sc];
    w += dw; h += dh;
    if (w >= W) { w -= W; ++h; }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const double t = warp_sum_d(s[c]);
    if (lane == 0) red[wave][c] = t;
  }
  __syncthreads();
  float mean[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    double t = 0.0;
    for (int v = 0; v < NWV; ++v) t += red[v][c];
    mean[c] = (float)(t / HW);
  }
  __syncthreads();
  // pass 2: std of the centred values (modify_models.py:84-85): unbiased, around their own mean
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  for (int i = threadIdx.x, h = h0, w = w0; i < HW; i += NS_T) {
    const float* px = xn + (int64_t)h * x.sh + (int64_t)w * x.sw;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < C) {
        const double d = (double)(px[(int64_t)c * x.sc] - mean[c]);
        s1[c] += d; s2[c] += d * d;
      }
    w += dw; h += dh;
    if (w >= W) { w -= W; ++h; }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const double t1 = warp_sum_d(s1[c]), t2 = warp_sum_d(s2[c]);
    if (lane == 0) { red[wave][c] = t1; red[wave][4 + c] = t2; }
  }
  __syncthreads();
  if (threadIdx.x < 4 && (int)threadIdx.x < C) {
    const int c = threadIdx.x;
    double S1 = 0.0, S2 = 0.0;
    for (int v = 0; v < NWV; ++v) { S1 += red[v][c]; S2 += red[v][4 + c]; }
    const double var = (S2 - S1 * S1 / HW) / (HW - 1);
    stat[c][0] = mean[c];
    stat[c][1] = (float)sqrt(var > 0.0 ? var : 0.0);
  }
  __syncthreads();
  // pass 3: normalise + sigmoid
  float* yn = y.ptr + (int64_t)n * y.sn;
  for (int i = threadIdx.x, h = h0, w = w0; i < HW; i += NS_T) {
    const float* px = xn + (int64_t)h * x.sh + (int64_t)w * x.sw;
    float* py = yn + (int64_t)h * y.sh + (int64_t)w * y.sw;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < C) {
        const float v = (px[(int64_t)c * x.sc] - stat[c][0]) / (stat[c][1] + 1e-6f);
        py[(int64_t)c * y.sc] = 1.f / (1.f + expf(-v));
      }
    w += dw; h += dh;
    if (w >= W) { w -= W; ++h; }
  }
}

// ------------------------------------------------------------------------- layernorm
// one wave per row
__global__ __launch_bounds__(256) void layernorm_kernel(const float* x, int64_t xs, float* y, int64_t ys,
                                                        int64_t rows, int C, const float* g, const float* b,
                                                        float eps, int relu) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const float* xr = x + row * xs;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[c];
  const float mean = warp_sum(s) / (float)C;
  float v = 0.f;
  for (int c = lane; c < C; c += 64) { const float d = xr[c] - mean; v += d * d; }
  const float var = warp_sum(v) / (float)C;
  const float rstd = 1.f / sqrtf(var + eps);
  float* yr = y + row * ys;
  for (int c = lane; c < C; c += 64) {
    float o = (xr[c] - mean) * rstd * g[c] + b[c];
    if (relu) o = o > 0.f ? o : 0.f;
    yr[c] = o;
  }
}

// register-resident variant: the row is read once (NV float4 per lane, C % 4 == 0,
// C <= 256*NV, 16-B aligned rows), statistics from registers, one write
template <int NV>
__global__ __launch_bounds__(256) void layernorm_reg_kernel(const float* __restrict__ x, int64_t xs,
                                                            float* __restrict__ y, int64_t ys, int64_t rows, int C,
                                                            const float* __restrict__ g,
                                                            const float* __restrict__ b, float eps, int relu) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const float* xr = x + row * xs;
  f4v v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    v[i] = c < C ? *reinterpret_cast<const f4v*>(xr + c) : f4v{0.f, 0.f, 0.f, 0.f};
    s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  }
  const float mean = warp_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < C) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float d = v[i][e] - mean; q += d * d; }
    }
  }
  const float var = warp_sum(q) / (float)C;
  const float rstd = 1.f / sqrtf(var + eps);
  float* yr = y + row * ys;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < C) {
      const f4v gg = *reinterpret_cast<const f4v*>(g + c), bb = *reinterpret_cast<const f4v*>(b + c);
      f4v o = (v[i] - mean) * rstd * gg + bb;
      if (relu & 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = o[e] > 0.f ? o[e] : 0.f;
      }
      if (relu & 2) store_planes4(reinterpret_cast<uint16_t*>(yr), c, o);
      else *reinterpret_cast<f4v*>(yr + c) = o;
    }
  }
}

// ------------------------------------------------------------------------- l2norm
// emb = x / max(||x||, eps): eps = 0 is IR-50's torch.div(x, norm) (net_adaface.py:334-335),
// eps = 1e-12 is F.normalize's clamp_min (face_recognition/module.py:137-138); norm = ||x||
__global__ __launch_bounds__(256) void l2norm_kernel(const float* x, float* emb, float* norm, int rows, int C,
                                                     float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const float* xr = x + (int64_t)row * C;
  double s = 0.0;
  for (int c = lane; c < C; c += 64) s += (double)xr[c] * xr[c];
  const float nrm = (float)sqrt(warp_sum_d(s));
  const float den = fmaxf(nrm, eps);
  for (int c = lane; c < C; c += 64) emb[(int64_t)row * C + c] = xr[c] / den;
  if (lane == 0) norm[row] = nrm;
}

// ------------------------------------------------------------------------- dfl decode
struct DflK {
  const float* head; float* out; int B, nc, A, nlev;
  int hw[8][2]; float stride[4]; int off[5];
};
__global__ __launch_bounds__(256) void dfl_decode_kernel(DflK p) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.B * p.A) return;
  const int b = t / p.A, a = t % p.A;
  int l = 0;
  while (l + 1 < p.nlev && a >= p.off[l + 1]) ++l;
  const int ia = a - p.off[l];
  const int w = p.hw[l][1];
  const float ax = (float)(ia % w) + 0.5f, ay = (float)(ia / w) + 0.5f;
  const float st = p.stride[l];
  const int no = 64 + p.nc;
  const float* h = p.head + ((int64_t)b * p.A + a) * no;
  float d[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    float m = -INFINITY;
    for (int i = 0; i < 16; ++i) m = fmaxf(m, h[s * 16 + i]);
    float e[16], sum = 0.f;
    for (int i = 0; i < 16; ++i) { e[i] = expf(h[s * 16 + i] - m); sum += e[i]; }
    float acc = 0.f;
    for (int i = 0; i < 16; ++i) acc += (e[i] / sum) * (float)i;
    d[s] = acc;
  }
  const float x1 = ax - d[0], y1 = ay - d[1], x2 = ax + d[2], y2 = ay + d[3];
  float* o = p.out + (int64_t)b * (4 + p.nc) * p.A + a;
  o[0] = ((x1 + x2) / 2.f) * st;
  o[(int64_t)p.A] = ((y1 + y2) / 2.f) * st;
  o[(int64_t)2 * p.A] = (x2 - x1) * st;
  o[(int64_t)3 * p.A] = (y2 - y1) * st;
  for (int c = 0; c < p.nc; ++c) o[(int64_t)(4 + c) * p.A] = 1.f / (1.f + expf(-h[64 + c]));
}

// ------------------------------------------------------------------------- copy_pad
// y[n,h,w,c] = c < x.c ? x[n,h,w,c] : 0  (layout change + channel zero-padding, e.g. NCHW
// frames -> NHWC4 so the 7x7 stem takes the vectorised implicit-GEMM path)
// (+ optional per-frame max|y| into y_amax[n]: the stem's precision-3 activation scale)
struct CopyK { prpe_view x, y; int rpb; float* y_amax; };
// One block = rpb consecutive rows of ONE frame (rpb divides y.h), threads striding over the
// rows' pixels; the frame's max|y| is reduced over the block and committed once (a per-wave
// commit made every wave of a frame race on the frame's slot: 6400 same-address atomics per
// 640x640 frame, 4.5x the copy's own time at bs = 256).
// Y4: y is 4 contiguous, 16-B aligned channels per pixel (the stem's NHWC4 buffer): one
// 16-B store per pixel instead of four 4-B ones
template <bool Y4>
__global__ __launch_bounds__(256) void copy_pad_kernel(CopyK p) {
  __shared__ float wmax[4];
  const int row0 = blockIdx.x * p.rpb;
  const int n = row0 / p.y.h, h0 = row0 - n * p.y.h;
  const int W = p.y.w;
  float m = 0.f;
  for (int i = threadIdx.x; i < p.rpb * W; i += 256) {
    const int r = i / W, w = i - r * W, h = h0 + r;
    float* y = p.y.ptr + voff(p.y, n, h, w, 0);
    if constexpr (Y4) {
      float v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        v[c] = c < p.x.c ? p.x.ptr[voff(p.x, n, h, w, c)] : 0.f;
        m = fmaxf(m, fabsf(v[c]));
      }
      *reinterpret_cast<float4*>(y) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      for (int c = 0; c < p.y.c; ++c) {
        const float v = c < p.x.c ? p.x.ptr[voff(p.x, n, h, w, c)] : 0.f;
        y[(int64_t)c * p.y.sc] = v;
        m = fmaxf(m, fabsf(v));
      }
    }
  }
  if (!p.y_amax) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    if (m > 0.f) atomicMax(reinterpret_cast<unsigned*>(p.y_amax + n), __float_as_uint(m));
  }
}

inline unsigned nblocks(int64_t total, int bs = 256) { return (unsigned)((total + bs - 1) / bs); }

// 1-D grid of rows * ceil(per_row / 256) blocks (see row_pos); false when it does not fit
inline bool rowgrid(int64_t rows, int64_t per_row, dim3& g, int& chunks) {
  if (rows <= 0 || per_row <= 0 || per_row >= (1LL << 30)) return false;
  const int64_t c = (per_row + 255) / 256, total = rows * c;
  if (total >= (1LL << 31)) return false;
  chunks = (int)c;
  g = dim3((unsigned)total);
  return true;
}

}  // namespace

extern "C" int64_t prpe_upconv3x3_workspace_bytes(const prpe_view* z, const prpe_view* y) {
  if (!z || !y) return 0;
  return (int64_t)sizeof(float) * 3 * y->n * z->h * y->w * y->c;
}

// host restatement of bilin_src (the same float arithmetic) for the DMA kernel's geometry rules
static void bilin_src_h(int dst, int in, int out, int ac, int& i0, int& i1) {
  float src;
  if (ac) {
    const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
    src = scale * (float)dst;
  } else {
    const float scale = (float)in / (float)out;
    src = scale * ((float)dst + 0.5f) - 0.5f;
    src = src < 0.f ? 0.f : src;
  }
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 < in - 1 ? i0 + 1 : i0;
}

static bool upd_geometry_ok(const prpe_view* z, const prpe_view* y, int ac) {
  const int Hi = z->h, Wi = z->w, Ho = y->h, Wo = y->w;
  if (Hi < 2 || Ho < 5 * Hi) return false;
  // source window of every 32-column tile (+1 column each side) <= UPD_NSC columns
  for (int ox0 = 0; ox0 < Wo; ox0 += UPD_W) {
    int lo, hi, t;
    bilin_src_h(ox0 > 0 ? ox0 - 1 : 0, Wi, Wo, ac, lo, t);
    bilin_src_h(ox0 + UPD_W < Wo ? ox0 + UPD_W : Wo - 1, Wi, Wo, ac, t, hi);
    if (hi - lo + 1 > UPD_NSC) return false;
  }
  // every source interval (output rows with the same y0) spans >= 5 output rows, except the first
  // and the last (the prologue waits for everything; no event follows the last)
  int prev = -1, run = 0, first = 1;
  for (int oy = 0; oy < Ho; ++oy) {
    int y0, y1;
    bilin_src_h(oy, Hi, Ho, ac, y0, y1);
    if (y0 != prev) {
      if (prev >= 0 && !first && run < 5) return false;
      if (prev >= 0) first = 0;
      prev = y0;
      run = 0;
    }
    ++run;
  }
  const int64_t zb = ((int64_t)(Hi - 1) * z->sh + (int64_t)(Wi - 1) * z->sw + z->c) * 4;
  return zb < (1LL << 31) && z->sh >= 0 && z->sw >= 0 && y->sh >= 0 && y->sw >= 0;
}

extern "C" int prpe_upconv3x3(const prpe_view* z, const prpe_view* y, int32_t align_corners,
                              const float* scale, const float* bias, const float* slope, int32_t act,
                              int32_t y_planes, float* y_amax, void* workspace, int64_t workspace_bytes,
                              void* stream) {
  if (!view_ok(z) || !view_ok(y) || z->n != y->n || z->c != 9 * y->c) return PRPE_EINVAL;
  if (y_amax && workspace) return PRPE_EINVAL;        // max|y| on the one-pass kernels only
  if (act == PRPE_ACT_PRELU && !slope) return PRPE_EINVAL;
  UpK p{};
  p.z = *z; p.y = *y; p.Co = y->c; p.ac = align_corners ? 1 : 0;
  p.scale = scale; p.bias = bias; p.slope = slope; p.act = act;
  p.y_planes = y_planes ? 1 : 0;
  p.y_amax = y_amax;
  const bool v4 = (y->c % 4 == 0) && z->sc == 1 && (z->sw % 4 == 0) && (z->sh % 4 == 0) &&
                  (z->sn % 4 == 0) && ((uintptr_t)z->ptr % 16 == 0) &&
                  (y->sc != 1 || ((y->sw % 4 == 0) && (y->sh % 4 == 0) && (y->sn % 4 == 0) &&
                                  ((uintptr_t)y->ptr % 16 == 0)));
  hipStream_t st = as_stream(stream);
  const int VWs = v4 ? 4 : 1;
  p.per_row = y->w * (y->c / VWs);
  dim3 g_out, g_h;
  if (!rowgrid((int64_t)y->n * y->h, p.per_row, g_out, p.chunks) ||
      !rowgrid((int64_t)y->n * 3 * z->h, p.per_row, g_h, p.chunks))
    return PRPE_EINVAL;
  const int64_t need = prpe_upconv3x3_workspace_bytes(z, y);
  if (y_planes && (!v4 || y->sc != 1 || y->c % 8 || y->sw % 8 || y->sh % 8 || y->sn % 8 ||
                   (uintptr_t)y->ptr % 32 || workspace))
    return PRPE_EINVAL;
  if (workspace && workspace_bytes >= need && ((uintptr_t)workspace % 16) == 0) {
    float* H = static_cast<float*>(workspace);
    if (v4) {
      hipLaunchKernelGGL(upconv_h_kernel<4>, g_h, dim3(256), 0, st, p, H);
      hipLaunchKernelGGL(upconv_out_kernel<4>, g_out, dim3(256), 0, st, p, (const float*)H);
    } else {
      hipLaunchKernelGGL(upconv_h_kernel<1>, g_h, dim3(256), 0, st, p, H);
      hipLaunchKernelGGL(upconv_out_kernel<1>, g_out, dim3(256), 0, st, p, (const float*)H);
    }
    return launch_status();
  }
  // unit scale (output grid = input grid, align_corners: every weight 0) with Co <= 4: the tap sum
  // (upconv_unit_kernel, same bits for finite z)
  if (align_corners && y->c <= 4 && z->h == y->h && z->w == y->w && !y_planes && z->sc == 1 &&
      z->sw == z->c && z->sh >= 0 && z->sn >= 0 && y->sh >= 0 && y->sw >= 0 && y->sc >= 0) {
    const int nstrip = (y->w + 63) / 64, ngroups = (nstrip + 3) / 4, rchunks = (y->h + UPU_R - 1) / UPU_R;
    const int64_t nb = (int64_t)y->n * rchunks * ngroups;
    if (nb >= (1LL << 31)) return PRPE_EINVAL;
    const dim3 g((unsigned)nb), b(256);
    switch (y->c) {
      case 1: hipLaunchKernelGGL(upconv_unit_kernel<1>, g, b, 0, st, p, nstrip, ngroups, rchunks); break;
      case 2: hipLaunchKernelGGL(upconv_unit_kernel<2>, g, b, 0, st, p, nstrip, ngroups, rchunks); break;
      case 3: hipLaunchKernelGGL(upconv_unit_kernel<3>, g, b, 0, st, p, nstrip, ngroups, rchunks); break;
      default: hipLaunchKernelGGL(upconv_unit_kernel<4>, g, b, 0, st, p, nstrip, ngroups, rchunks); break;
    }
    return launch_status();
  }
  // LDS-DMA path (upconv_dma_kernel): 4-channel vectors, Co % 32 == 0, channel-contiguous y,
  // every output column tile's source window <= UPD_NSC columns, every source interval >= 5
  // output rows (the kernel's vmcnt counting), one frame of z < 2^31 bytes. PRPE_UPCONV_DMA=0
  // keeps the fused kernel (A/B runs).
  static const int dma_env = [] {
    const char* e = getenv("PRPE_UPCONV_DMA");
    return e ? atoi(e) : 1;
  }();
  if (dma_env && v4 && y->c % UPD_C == 0 && y->sc == 1 && z->sc == 1 && y->h <= UP_MAX_R && upd_geometry_ok(z, y, p.ac)) {
    const int R = y->h, rblocks = 1;
    const int ctiles = (y->w + UPD_W - 1) / UPD_W, cblocks = y->c / UPD_C;
    const int64_t nb = (int64_t)y->n * rblocks * ctiles * cblocks;
    if (nb < (1LL << 31)) {
      const dim3 g((unsigned)nb);
#define PRPE_UPD(A)                                                                                               \
  if (y_planes) hipLaunchKernelGGL((upconv_dma_kernel<A, true>), g, dim3(256), 0, st, p, R, rblocks, ctiles, cblocks);  \
  else hipLaunchKernelGGL((upconv_dma_kernel<A, false>), g, dim3(256), 0, st, p, R, rblocks, ctiles, cblocks);
      if (act == PRPE_ACT_NONE) { PRPE_UPD(PRPE_ACT_NONE) }
      else if (act == PRPE_ACT_SILU) { PRPE_UPD(PRPE_ACT_SILU) }
      else if (act == PRPE_ACT_PRELU) { PRPE_UPD(PRPE_ACT_PRELU) }
      else if (act == PRPE_ACT_GELU) { PRPE_UPD(PRPE_ACT_GELU) }
      else { PRPE_UPD(-1) }
#undef PRPE_UPD
      return launch_status();
    }
  }
  // fused path: R output rows per thread; shrink R while the grid would not fill the chip
  // rows per thread: each thread's first rows rebuild both interpolation rows of every dy, so
  // long runs amortise that (measured, tools/upconv_bench.py bs=256: R 32 -> 256 = +4..10 %);
  // PRPE_UPCONV_R overrides it for A/B runs
  static const int r_env = [] {
    const char* e = getenv("PRPE_UPCONV_R");
    return e ? atoi(e) : 256;
  }();
  int R = r_env < UP_MAX_R ? (r_env > 0 ? r_env : 1) : UP_MAX_R;
  while (R > 4 && (int64_t)y->n * ((y->h + R - 1) / R) * p.chunks < 8192) R /= 2;
  const int rblocks = (y->h + R - 1) / R;
  const int64_t nb = (int64_t)y->n * rblocks * p.chunks;
  if (nb >= (1LL << 31)) return PRPE_EINVAL;
  // 32-bit per-thread offsets inside one frame (see the fused kernel)
  auto span = [](const prpe_view* v) {
    return (int64_t)(v->h - 1) * v->sh + (int64_t)(v->w - 1) * v->sw + (int64_t)(v->c - 1) * v->sc;
  };
  if (span(z) >= (1LL << 31) || span(y) >= (1LL << 31) || z->sw < 0 || z->sc < 0 || z->sh < 0 || y->sw < 0 ||
      y->sc < 0)
    return PRPE_EINVAL;
  p.xcd = 1;   // XCD-contiguous block order (round 2: -12..27 % per launch; its A/B switch removed in round 6)
  const dim3 g((unsigned)nb);
  static const int abl = [] {
    const char* e = getenv("PRPE_UPCONV_ABL");
    return e ? atoi(e) : 0;
  }();
#define PRPE_UP_ABL(A)                                                                                     \
  if (abl == 1) hipLaunchKernelGGL((upconv_fused_kernel<4, A, 1>), g, dim3(256), 0, st, p, R, rblocks);     \
  else if (abl == 2) hipLaunchKernelGGL((upconv_fused_kernel<4, A, 2>), g, dim3(256), 0, st, p, R, rblocks); \
  else hipLaunchKernelGGL((upconv_fused_kernel<4, A, 3>), g, dim3(256), 0, st, p, R, rblocks);
  if (abl && v4 && act == PRPE_ACT_SILU) {
    PRPE_UP_ABL(PRPE_ACT_SILU)
    return launch_status();
  }
  if (abl && v4 && act == PRPE_ACT_GELU) {
    PRPE_UP_ABL(PRPE_ACT_GELU)
    return launch_status();
  }
#undef PRPE_UP_ABL
  if (!v4) hipLaunchKernelGGL((upconv_fused_kernel<1, -1>), g, dim3(256), 0, st, p, R, rblocks);
  else if (act == PRPE_ACT_NONE) hipLaunchKernelGGL((upconv_fused_kernel<4, PRPE_ACT_NONE>), g, dim3(256), 0, st, p, R, rblocks);
  else if (act == PRPE_ACT_SILU) hipLaunchKernelGGL((upconv_fused_kernel<4, PRPE_ACT_SILU>), g, dim3(256), 0, st, p, R, rblocks);
  else if (act == PRPE_ACT_PRELU) hipLaunchKernelGGL((upconv_fused_kernel<4, PRPE_ACT_PRELU>), g, dim3(256), 0, st, p, R, rblocks);
  else if (act == PRPE_ACT_GELU) hipLaunchKernelGGL((upconv_fused_kernel<4, PRPE_ACT_GELU>), g, dim3(256), 0, st, p, R, rblocks);
  else hipLaunchKernelGGL((upconv_fused_kernel<4, -1>), g, dim3(256), 0, st, p, R, rblocks);
  return launch_status();
}

extern "C" int prpe_dwconv(const prpe_view* x, const prpe_view* y, const prpe_view* res, const float* w,
                           int32_t k, int32_t stride, int32_t pad, const float* scale, const float* bias,
                           int32_t act, void* stream) {
  if (!view_ok(x) || !view_ok(y) || !w || x->c != y->c || x->n != y->n || k <= 0 || stride <= 0) return PRPE_EINVAL;
  if ((x->h + 2 * pad - k) / stride + 1 != y->h || (x->w + 2 * pad - k) / stride + 1 != y->w) return PRPE_EINVAL;
  if (act == PRPE_ACT_PRELU) return PRPE_EINVAL;
  DwK p{};
  p.x = *x; p.y = *y;
  if (res && res->ptr) p.r = *res;
  p.w = w; p.k = k; p.stride = stride; p.pad = pad; p.scale = scale; p.bias = bias; p.act = act;
  p.per_row = y->w * y->c;
  dim3 g;
  if (!rowgrid((int64_t)y->n * y->h, (int64_t)y->w * y->c, g, p.chunks)) return PRPE_EINVAL;
  hipLaunchKernelGGL(dwconv_kernel, g, dim3(256), 0, as_stream(stream), p);
  return launch_status();
}

extern "C" int prpe_copy_pad(const prpe_view* x, const prpe_view* y, float* y_amax, void* stream) {
  if (!view_ok(x) || !view_ok(y) || x->n != y->n || x->h != y->h || x->w != y->w || y->c < x->c) return PRPE_EINVAL;
  // rows per block: a divisor of y.h (rows of one frame), about 2048 pixels per block
  int rpb = 1;
  for (int r = 2; r <= 64 && (int64_t)r * y->w <= 2048; ++r)
    if (y->h % r == 0) rpb = r;
  const int64_t blocks = (int64_t)y->n * y->h / rpb;
  if (blocks >= (1LL << 31) || (int64_t)rpb * y->w >= (1LL << 30)) return PRPE_EINVAL;
  CopyK p{*x, *y, rpb, y_amax};
  const bool y4 = y->c == 4 && y->sc == 1 && y->sw % 4 == 0 && y->sh % 4 == 0 && y->sn % 4 == 0 &&
                  (uintptr_t)y->ptr % 16 == 0;
  if (y4) hipLaunchKernelGGL(copy_pad_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), p);
  else hipLaunchKernelGGL(copy_pad_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), p);
  return launch_status();
}

extern "C" int prpe_maxpool(const prpe_view* x, const prpe_view* y, int32_t k, int32_t stride, int32_t pad,
                            void* stream) {
  if (!view_ok(x) || !view_ok(y) || x->c != y->c || x->n != y->n || k <= 0 || stride <= 0) return PRPE_EINVAL;
  if ((x->h + 2 * pad - k) / stride + 1 != y->h || (x->w + 2 * pad - k) / stride + 1 != y->w) return PRPE_EINVAL;
  auto a16 = [](const prpe_view* v) {
    return v->sc == 1 && v->c % 4 == 0 && v->sw % 4 == 0 && v->sh % 4 == 0 && v->sn % 4 == 0 &&
           ((uintptr_t)v->ptr % 16) == 0;
  };
  const bool v4 = a16(x) && a16(y);
  PoolK p{*x, *y, k, stride, pad, y->w * (y->c / (v4 ? 4 : 1)), 0};
  dim3 g;
  if (!rowgrid((int64_t)y->n * y->h, p.per_row, g, p.chunks)) return PRPE_EINVAL;
  if (v4) hipLaunchKernelGGL(maxpool_kernel<4>, g, dim3(256), 0, as_stream(stream), p);
  else hipLaunchKernelGGL(maxpool_kernel<1>, g, dim3(256), 0, as_stream(stream), p);
  return launch_status();
}

extern "C" int prpe_upsample_nearest2x(const prpe_view* x, const prpe_view* y, void* stream) {
  if (!view_ok(x) || !view_ok(y) || x->c != y->c || x->n != y->n || y->h != 2 * x->h || y->w != 2 * x->w)
    return PRPE_EINVAL;
  Up2K p{*x, *y, y->w * y->c, 0};
  dim3 g;
  if (!rowgrid((int64_t)y->n * y->h, (int64_t)y->w * y->c, g, p.chunks)) return PRPE_EINVAL;
  hipLaunchKernelGGL(upsample2x_kernel, g, dim3(256), 0, as_stream(stream), p);
  return launch_status();
}

extern "C" int prpe_norm_sigmoid(const prpe_view* x, const prpe_view* y, void* stream) {
  if (!view_ok(x) || !view_ok(y) || x->c > 4 || x->c != y->c || x->n != y->n || x->h != y->h || x->w != y->w ||
      x->h * x->w < 2)
    return PRPE_EINVAL;
  hipLaunchKernelGGL(norm_sigmoid_kernel, dim3(x->n), dim3(NS_T), 0, as_stream(stream), *x, *y);
  return launch_status();
}

extern "C" int prpe_layernorm(const float* x, int64_t xs, float* y, int64_t ys, int64_t rows, int32_t C,
                              const float* g, const float* b, float eps, int32_t flags, void* stream) {
  if (!x || !y || !g || !b || rows <= 0 || C <= 0) return PRPE_EINVAL;
  if (flags & ~3) return PRPE_EINVAL;
  const bool al = C % 4 == 0 && xs % 4 == 0 && ys % 4 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0 &&
                  (uintptr_t)g % 16 == 0 && (uintptr_t)b % 16 == 0;
  // planes output (flags bit 1): the register-resident kernels only, whole 8-channel groups
  if ((flags & 2) && (!al || C % 8 || C > 1024 || ys % 8 || (uintptr_t)y % 32)) return PRPE_EINVAL;
  const int relu = flags;
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t st = as_stream(stream);
  if (al && C <= 256) { hipLaunchKernelGGL(layernorm_reg_kernel<1>, grid, dim3(256), 0, st, x, xs, y, ys, rows, C, g, b, eps, relu); return launch_status(); }
  if (al && C <= 512) { hipLaunchKernelGGL(layernorm_reg_kernel<2>, grid, dim3(256), 0, st, x, xs, y, ys, rows, C, g, b, eps, relu); return launch_status(); }
  if (al && C <= 768) { hipLaunchKernelGGL(layernorm_reg_kernel<3>, grid, dim3(256), 0, st, x, xs, y, ys, rows, C, g, b, eps, relu); return launch_status(); }
  if (al && C <= 1024) { hipLaunchKernelGGL(layernorm_reg_kernel<4>, grid, dim3(256), 0, st, x, xs, y, ys, rows, C, g, b, eps, relu); return launch_status(); }
  hipLaunchKernelGGL(layernorm_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, as_stream(stream), x, xs, y,
                     ys, rows, C, g, b, eps, relu & 1);
  return launch_status();
}

extern "C" int prpe_l2norm(const float* x, float* emb, float* norm, int32_t rows, int32_t C, float eps,
                           void* stream) {
  if (!x || !emb || !norm || rows <= 0 || C <= 0 || !(eps >= 0.f)) return PRPE_EINVAL;
  hipLaunchKernelGGL(l2norm_kernel, dim3((rows + 3) / 4), dim3(256), 0, as_stream(stream), x, emb, norm, rows, C,
                     eps);
  return launch_status();
}

extern "C" int prpe_dfl_decode(const float* head, float* out, int32_t B, int32_t nc, int32_t nlev,
                               const int32_t* level_hw, const float* strides, void* stream) {
  if (!head || !out || B <= 0 || nc <= 0 || nlev <= 0 || nlev > 4 || !level_hw || !strides) return PRPE_EINVAL;
  DflK p{};
  p.head = head; p.out = out; p.B = B; p.nc = nc; p.nlev = nlev;
  int a = 0;
  for (int l = 0; l < nlev; ++l) {
    p.hw[l][0] = level_hw[2 * l]; p.hw[l][1] = level_hw[2 * l + 1];
    p.stride[l] = strides[l]; p.off[l] = a;
    a += level_hw[2 * l] * level_hw[2 * l + 1];
  }
  p.off[nlev] = a;
  p.A = a;
  hipLaunchKernelGGL(dfl_decode_kernel, dim3(nblocks((int64_t)B * a)), dim3(256), 0, as_stream(stream), p);
  return launch_status();
}
