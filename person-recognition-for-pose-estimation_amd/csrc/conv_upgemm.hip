// Upsample-fused 1x1 GEMM (round 5): the face-YOLO adapter's
//   .4  conv3x3(bilinear_upsample(x)) + BN + SiLU      (via the tap rewrite: z = W_taps x, low-res)
//   .7  conv1x1 512 -> 256 + BN + SiLU                 (training/modify_models.py:47-56)
// as ONE kernel: the A operand of the 1x1 GEMM -- the upconv output, 512 channels per pixel -- is
// computed per K-step from the low-resolution tap maps z in LDS and never reaches HBM (unfused:
// prpe_upconv3x3 writes 13.4 GB of planes at bs = 256 and the GEMM reads them back).
//
// Workgroup = one 16 x 16 output-pixel tile of one frame x all Co = 256 GEMM columns, 8 waves as
// 2 (pixels) x 4 (columns), wave tile 128 x 64 (8 row blocks = 8 output rows of the tile). Per
// 32-channel K-step kt:
//   top    wait for this step's LDS-DMA (z window, W planes), barrier
//   H      Hs[dy][r][ox] = sum_dx valid * lerp_x(z_{dy,dx}[r], sx(ox + dx - 1)), the x-interpolated
//          tap rows of the tile's source window (at most 5 source rows), into LDS; barrier
//   (issue the next step's z window and W planes by LDS-DMA: the z window is free now)
//   A      a[m] = act(bn(sum_dy valid * lerp_y(Hs[dy][r0], Hs[dy][r1]))) for the tile's 256 pixels,
//          split into the two bf16 planes and written in conv_gemm.hip's A image; barrier
//   MFMA   conv_gemm.hip's K-step (B fragments of the wave's 4 column blocks, A per row block,
//          3 MFMAs per product, the same K order and per-accumulator MFMA order)
// The arithmetic of H and A is prpe_upconv3x3's (pointwise.hip: lerp_add's fixed rounding
// sequence, dx then dy order, the same BN expression and apply_act4, the same planes split) and
// the GEMM's is conv_gemm.hip's: the output is bit-identical to the two unfused launches
// (tests/test_gpu_ops.py test_upconv_gemm_*).
//
// LDS: z window [5 rows][5 cols][9 taps][32 ch] fp32 (29 KB), Hs [3][5][16][32] (30 KB), the W
// planes double-buffered [2][2 planes][256][64 B] (64 KB), A [256 px][128 B] (32 KB): 155 KB, one
// workgroup per CU. The epilogue's 16-row slabs reuse the z window and Hs.
#include "conv.h"

namespace prpe_k {

struct UpGemmK {
  const float* z; int64_t zsn, zsh, zsw;                 // [N, Hi, Wi, 9 C], channel stride 1
  int Hi, Wi, C;
  int Ho, Wo, ac;
  const float* usc; const float* ubi; const float* usl; int uact;
  const uint16_t* whi; const uint16_t* wlo; int k_pad;   // [Co][k_pad] bf16 planes
  const float* scale; const float* bias; const float* slope; int act;
  float* y; int64_t ysn, ysh, ysw; int Co; int y_planes;
  int tiles_w, tiles_h, nwg;
};

namespace {

constexpr int UG_T = 16;                                  // tile: 16 x 16 output pixels
constexpr int UG_SR = 5, UG_SC = 5;                       // source window bound (host-checked)
constexpr int UG_LINES = UG_SR * UG_SC * 9;               // 128-B lines of one K-step's window: 225
constexpr int UG_ZP = (UG_LINES + 7) / 8;                 // 1-KiB DMA pieces: 29
constexpr int UG_Z_BYTES = UG_ZP * 1024;                  // 29696
constexpr int UG_HS_BYTES = 3 * UG_SR * UG_T * 128;      // 30720
constexpr int UG_B_BYTES = 2 * 256 * 64;                  // one K-step of W (both planes): 32768
constexpr int UG_A_BYTES = 256 * 128;                     // 32768
constexpr int UG_Z_OFF = 0, UG_HS_OFF = UG_Z_BYTES, UG_B_OFF = UG_HS_OFF + UG_HS_BYTES;
constexpr int UG_A_OFF = UG_B_OFF + 2 * UG_B_BYTES;
constexpr int UG_LDS = UG_A_OFF + UG_A_BYTES;             // 158720
static_assert(UG_LDS <= 160 * 1024, "LDS");
static_assert(8 * 16 * (64 + 4) * 4 <= UG_B_OFF, "epilogue slabs in the z window + Hs");

// x + (1 - l) a + l b, pointwise.hip's lerp_add: the same rounding sequence as prpe_upconv3x3
__device__ __forceinline__ float ug_lerp_add(float x, float l, float a, float b) {
  const float t = __builtin_fmaf(1.f - l, a, l * b);
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(t));
  return r;
}
// PyTorch upsample_bilinear2d source index, as pointwise.hip bilin_src
__device__ __forceinline__ void ug_src(int dst, int in, int out, int ac, int& i0, int& i1, float& l1) {
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

__global__ __launch_bounds__(512, 2) void upgemm_kernel(UpGemmK p) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[UG_LDS];
  __shared__ int ty0[UG_T + 2], ty1[UG_T + 2], tx0[UG_T + 2], tx1[UG_T + 2];
  __shared__ float tly[UG_T + 2], tlx[UG_T + 2];
  constexpr int TM = 8, TN = 4, NP = 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int wm = wave >> 2, wn = wave & 3;
  int L = xcd_remap(blockIdx.x, p.nwg);
  const int tw = L % p.tiles_w;
  L /= p.tiles_w;
  const int th = L % p.tiles_h;
  const int n = L / p.tiles_h;
  const int oy0 = th * UG_T, ox0 = tw * UG_T;

  // bilinear tables of the tile's output rows / columns oy0 - 1 .. oy0 + 16 (-1: outside the image)
  if (tid < UG_T + 2) {
    const int yy = oy0 - 1 + tid;
    int y0 = -1, y1 = -1;
    float l = 0.f;
    if ((unsigned)yy < (unsigned)p.Ho) ug_src(yy, p.Hi, p.Ho, p.ac, y0, y1, l);
    ty0[tid] = y0; ty1[tid] = y1; tly[tid] = l;
  } else if (tid >= 64 && tid < 64 + UG_T + 2) {
    const int e = tid - 64, xx = ox0 - 1 + e;
    int x0 = -1, x1 = -1;
    float l = 0.f;
    if ((unsigned)xx < (unsigned)p.Wo) ug_src(xx, p.Wi, p.Wo, p.ac, x0, x1, l);
    tx0[e] = x0; tx1[e] = x1; tlx[e] = l;
  }
  __syncthreads();
  // source window: rows [sr0, sr0 + 5), columns [sc0, sc0 + 5) (the host checked every tile fits)
  int sr0 = p.Hi, sc0 = p.Wi;
#pragma unroll
  for (int e = 0; e < UG_T + 2; ++e) {
    if (ty0[e] >= 0 && ty0[e] < sr0) sr0 = ty0[e];
    if (tx0[e] >= 0 && tx0[e] < sc0) sc0 = tx0[e];
  }

  // ---- DMA sources. z window: piece i (0..28) = lines 8i .. 8i+7, line = (r * 5 + s) * 9 + t,
  // lane -> line 8i + lane / 8, 16-B chunk lane % 8 of its 32 channels. Lines past the frame's
  // rows / columns read zeros (unused).
  const float* zn = p.z + (int64_t)n * p.zsn;
  const int zbytes = (int)(((int64_t)(p.Hi - 1) * p.zsh + (int64_t)(p.Wi - 1) * p.zsw + 9 * p.C) * 4);
  const __amdgpu_buffer_rsrc_t zr = buf_rsrc(zn, zbytes);
  constexpr int ZPW = (UG_ZP + 7) / 8;                    // pieces per wave (4; waves 5-7 issue 3)
  unsigned zvo[ZPW];
#pragma unroll
  for (int k = 0; k < ZPW; ++k) {
    const int i = wave + 8 * k;
    const int line = i * 8 + (lane >> 3);
    const int r = line / 45, s = (line / 9) % 5, t = line % 9;
    const bool ok = i < UG_ZP && line < UG_LINES && sr0 + r < p.Hi && sc0 + s < p.Wi;
    zvo[k] = ok ? (unsigned)((((int64_t)(sr0 + r) * p.zsh + (int64_t)(sc0 + s) * p.zsw) + t * p.C + (lane & 7) * 4) * 4)
                : BL_OOB;
  }
  // W planes: piece j = wave * 4 + u (32 per step): plane j / 16, rows 16 (j % 16) .. + 16, conv_gemm's
  // B image [plane][256 rows][64 B] with its slot swizzle
  const __amdgpu_buffer_rsrc_t wr0 = buf_rsrc(p.whi, p.Co * p.k_pad * 2);
  const __amdgpu_buffer_rsrc_t wr1 = buf_rsrc(p.wlo, p.Co * p.k_pad * 2);
  const bool wq = wave >= 4;                              // pieces 16 .. 31: the lo plane
  const __amdgpu_buffer_rsrc_t wrq = wq ? wr1 : wr0;
  unsigned wvo[4];
  int wdst[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = wave * 4 + u;
    const int rb = j % 16;
    const int nrow = rb * 16 + (lane >> 2);
    const int ch = (lane & 3) ^ swzF(nrow);
    wvo[u] = (unsigned)((nrow * p.k_pad + ch * 8) * 2);
    wdst[u] = ((j / 16) * 256 + rb * 16) * 64;
  }
  auto issue = [&](int kt) {
#pragma unroll
    for (int k = 0; k < ZPW; ++k)
      if (wave + 8 * k < UG_ZP) bl_lds16(zr, lds + UG_Z_OFF + (wave + 8 * k) * 1024, zvo[k], kt * 32 * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) bl_lds16(wrq, lds + UG_B_OFF + (kt & 1) * UG_B_BYTES + wdst[u], wvo[u], kt * 32 * 2);
  };

  // ---- H items of this thread: it = tid + 512 k, (dy, r, ox, cg) = it / 640, it / 128 % 5, it / 8 % 16, it % 8
  // ---- A items: it = tid + 512 k, pixel m = it / 8 (row py = m / 16, column px = m % 16), cg = it % 8
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.C / 32;
  issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");   // step kt's z window + W landed
    __builtin_amdgcn_sched_barrier(0);
    // ---- H: x-interpolated tap rows of the window into Hs
    const float* zw = reinterpret_cast<const float*>(lds + UG_Z_OFF);
    float* hs = reinterpret_cast<float*>(lds + UG_HS_OFF);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int it = tid + 512 * k;
      if (it >= 3 * UG_SR * UG_T * 8) break;
      const int cg = it & 7, ox = (it >> 3) & 15, r = (it >> 7) % UG_SR, dy = it / (UG_SR * 128);
      f32x4 h = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int e = ox + dx;                            // table index of output column ox0 + ox + dx - 1
        const int x0 = tx0[e];
        if (x0 < 0) continue;
        const float lx = tlx[e];
        const f32x4 A = *reinterpret_cast<const f32x4*>(zw + (((r * UG_SC + (x0 - sc0)) * 9 + dy * 3 + dx) * 32 + cg * 4));
        const f32x4 B = *reinterpret_cast<const f32x4*>(zw + (((r * UG_SC + (tx1[e] - sc0)) * 9 + dy * 3 + dx) * 32 + cg * 4));
#pragma unroll
        for (int v = 0; v < 4; ++v) h[v] = ug_lerp_add(h[v], lx, A[v], B[v]);
      }
      *reinterpret_cast<f32x4*>(hs + (((dy * UG_SR + r) * UG_T + ox) * 32 + cg * 4)) = h;
    }
    __syncthreads();                                      // Hs complete; the z window is free
    if (kt + 1 < nk) issue(kt + 1);
    // ---- A: the upconv output of this step's 32 channels for the tile's 256 pixels
    const int c0 = kt * 32;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int it = tid + 512 * k;
      const int cg = it & 7, m = it >> 3, py = m >> 4, px = m & 15;
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int e = py + dy;                            // table index of output row oy0 + py + dy - 1
        const int y0 = ty0[e];
        if (y0 < 0) continue;
        const float ly = tly[e];
        const f32x4 HA = *reinterpret_cast<const f32x4*>(hs + (((dy * UG_SR + (y0 - sr0)) * UG_T + px) * 32 + cg * 4));
        const f32x4 HB = *reinterpret_cast<const f32x4*>(hs + (((dy * UG_SR + (ty1[e] - sr0)) * UG_T + px) * 32 + cg * 4));
#pragma unroll
        for (int v = 0; v < 4; ++v) a[v] = ug_lerp_add(a[v], ly, HA[v], HB[v]);
      }
      const int c = c0 + cg * 4;
      const f4 s4 = *reinterpret_cast<const f4*>(p.usc + c), b4 = *reinterpret_cast<const f4*>(p.ubi + c);
      f32x4 sl4 = {0.f, 0.f, 0.f, 0.f};
      if (p.usl) sl4 = *reinterpret_cast<const f32x4*>(p.usl + c);
      f32x4 pre;
#pragma unroll
      for (int v = 0; v < 4; ++v) pre[v] = a[v] * s4[v] + b4[v];
      const f32x4 o = apply_act4(pre, p.uact, sl4);
      // planes split (common.h store_planes4): hi = RNE(v), lo = RNE(v - hi) by an explicit subtract
      unsigned short hi[4], lo[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float x = o[v];
        const __bf16 hb = (__bf16)x;
        float d;
        asm("v_sub_f32 %0, %1, %2" : "=v"(d) : "v"(x), "v"((float)hb));
        hi[v] = __builtin_bit_cast(unsigned short, hb);
        lo[v] = __builtin_bit_cast(unsigned short, (__bf16)d);
      }
      const unsigned long long h64 = (unsigned long long)(hi[0] | (unsigned)hi[1] << 16) |
                                     (unsigned long long)(hi[2] | (unsigned)hi[3] << 16) << 32;
      const unsigned long long l64 = (unsigned long long)(lo[0] | (unsigned)lo[1] << 16) |
                                     (unsigned long long)(lo[2] | (unsigned)lo[3] << 16) << 32;
      // conv_gemm's A image: row m, 8 slots of 16 B (group g = hi[8] | lo[8]) at slot ^ swz_rows(m)
      const int g = cg >> 1, half = (cg & 1) * 8;
      unsigned char* row = lds + UG_A_OFF + m * 128;
      const int sw = swz_rows(m);
      *reinterpret_cast<unsigned long long*>(row + (((2 * g) ^ sw) << 4) + half) = h64;
      *reinterpret_cast<unsigned long long*>(row + (((2 * g + 1) ^ sw) << 4) + half) = l64;
    }
    // A complete: a raw barrier after the LDS writes drain (a __syncthreads() would also drain
    // the next step's LDS-DMA just issued, vmcnt(0))
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // ---- MFMA: conv_gemm.hip's K-step on the A image and the W stage of step kt
    const unsigned char* sa = lds + UG_A_OFF;
    const unsigned char* sb = lds + UG_B_OFF + (kt & 1) * UG_B_BYTES;
    bf16x8 bfr[TN][NP];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nrow = wn * 64 + j * 16 + fr;
      const unsigned char* bp = sb + nrow * 64 + ((fg ^ swzF(nrow)) << 4);
#pragma unroll
      for (int q = 0; q < NP; ++q) bfr[j][q] = *reinterpret_cast<const bf16x8*>(bp + q * 256 * 64);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * 128 + i * 16 + fr;
      const int sw = swz_rows(row);
      const unsigned char* ap = sa + row * 128;
      bf16x8 af[NP];
      af[0] = *reinterpret_cast<const bf16x8*>(ap + (((2 * fg) ^ sw) << 4));
      af[1] = *reinterpret_cast<const bf16x8*>(ap + (((2 * fg + 1) ^ sw) << 4));
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int s = NP - 1; s >= 0; --s)
#pragma unroll
          for (int qa = s; qa >= 0; --qa) acc[i][j] = mfma16(af[qa], bfr[j][s - qa], acc[i][j]);
    }
  }
  __syncthreads();                                        // every wave done with the stages

  // ---------------- epilogue (conv_gemm.hip's): per-wave 16-row x 64-column slabs, 16-B row
  // stores; row block i of wave (wm, wn) = output row oy0 + 8 wm + i, columns ox0 .. ox0 + 15
  constexpr int WTN = 64, CS = WTN + 4;
  float* ct = reinterpret_cast<float*>(lds) + wave * 16 * CS;
  constexpr int CPR = WTN / 4, RPP = 64 / CPR, EB = 16 / RPP;
  const int cc = lane % CPR, rr0 = lane / CPR;
  const int col = wn * WTN + cc * 4;
  f4 sc4 = {1.f, 1.f, 1.f, 1.f}, bi4 = {0.f, 0.f, 0.f, 0.f}, sl4 = {0.f, 0.f, 0.f, 0.f};
  if (p.scale) sc4 = *reinterpret_cast<const f4*>(p.scale + col);
  if (p.bias) bi4 = *reinterpret_cast<const f4*>(p.bias + col);
  if (p.slope) sl4 = *reinterpret_cast<const f4*>(p.slope + col);
  float* yn = p.y + (int64_t)n * p.ysn;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < TN; ++j) ct[(fg * 4 + r) * CS + j * 16 + fr] = acc[i][j][r];
    __builtin_amdgcn_wave_barrier();
    const int oy = oy0 + wm * 8 + i;
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int px = rr0 + RPP * e;                       // slab row = output column ox0 + px
      f4 v = *reinterpret_cast<const f4*>(ct + px * CS + cc * 4);
      const int ox = ox0 + px;
      if (oy >= p.Ho || ox >= p.Wo) continue;
      v = v * sc4 + bi4;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = apply_act(v[q], p.act, sl4[q]);
      const int64_t yo = (int64_t)oy * p.ysh + (int64_t)ox * p.ysw;
      if (p.y_planes) {
        bf16x4 pl[2];
        split_planes<2>(v, pl);
        uint16_t* y16 = reinterpret_cast<uint16_t*>(yn + yo) + (col >> 3) * 16 + (col & 7);
        *reinterpret_cast<bf16x4*>(y16) = pl[0];
        *reinterpret_cast<bf16x4*>(y16 + 8) = pl[1];
      } else {
        *reinterpret_cast<f4*>(yn + yo + col) = v;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace
}  // namespace prpe_k

extern "C" int prpe_upconv_gemm(const prpe_upgemm_desc* d, void* stream) {
  using namespace prpe_k;
  if (!d || !view_ok(&d->z) || !view_ok(&d->y)) return PRPE_EINVAL;
  const prpe_view& z = d->z; const prpe_view& y = d->y;
  const int C = z.c / 9;
  if (z.c != 9 * C || C % 32 || C <= 0 || y.c != 256 || z.n != y.n || z.sc != 1 || y.sc != 1) return PRPE_EINVAL;
  if (!d->w_hi || !d->w_lo || d->k_pad < C || !d->up_scale || !d->up_bias) return PRPE_EINVAL;
  if ((uintptr_t)z.ptr % 16 || z.sw % 4 || z.sh % 4 || z.sn % 4 || z.sw < 0 || z.sh < 0 || (uintptr_t)y.ptr % 32 ||
      y.sw % 8 || y.sh % 8 || y.sn % 8 || y.sw < y.c || y.sh < 0 || (uintptr_t)d->w_hi % 16 ||
      (uintptr_t)d->w_lo % 16 || d->k_pad % 8 || (uintptr_t)d->up_scale % 16 || (uintptr_t)d->up_bias % 16 ||
      (d->up_slope && (uintptr_t)d->up_slope % 16) || (d->scale && (uintptr_t)d->scale % 16) ||
      (d->bias && (uintptr_t)d->bias % 16) || (d->slope && (uintptr_t)d->slope % 16))
    return PRPE_EINVAL;
  if (((int64_t)(z.h - 1) * z.sh + (int64_t)(z.w - 1) * z.sw + z.c) * 4 >= (1LL << 31) ||
      (int64_t)y.c * d->k_pad * 2 >= (1LL << 31))
    return PRPE_EINVAL;
  {  // not in place
    uintptr_t alo, ahi, blo, bhi;
    view_span(z, alo, ahi);
    view_span(y, blo, bhi);
    if (spans_overlap(alo, ahi, blo, bhi)) return PRPE_EINVAL;
  }
  // every 16-pixel tile's source window (output rows / columns t0 - 1 .. t0 + 16) within 5 x 5
  auto span_ok = [&](int in, int out) {
    for (int t0 = 0; t0 < out; t0 += UG_T) {
      int lo = in, hi = -1;
      for (int e = -1; e <= UG_T; ++e) {
        const int dst = t0 + e;
        if (dst < 0 || dst >= out) continue;
        float src;
        if (d->align_corners) src = (out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f) * (float)dst;
        else { src = (float)in / (float)out * ((float)dst + 0.5f) - 0.5f; if (src < 0.f) src = 0.f; }
        int i0 = (int)src;
        if (i0 > in - 1) i0 = in - 1;
        const int i1 = i0 < in - 1 ? i0 + 1 : i0;
        if (i0 < lo) lo = i0;
        if (i1 > hi) hi = i1;
      }
      if (hi - lo + 1 > UG_SR) return false;
    }
    return true;
  };
  if (!span_ok(z.h, y.h) || !span_ok(z.w, y.w)) return PRPE_EINVAL;
  UpGemmK kp{};
  kp.z = z.ptr; kp.zsn = z.sn; kp.zsh = z.sh; kp.zsw = z.sw; kp.Hi = z.h; kp.Wi = z.w; kp.C = C;
  kp.Ho = y.h; kp.Wo = y.w; kp.ac = d->align_corners ? 1 : 0;
  kp.usc = d->up_scale; kp.ubi = d->up_bias; kp.usl = d->up_slope; kp.uact = d->up_act;
  kp.whi = d->w_hi; kp.wlo = d->w_lo; kp.k_pad = d->k_pad;
  kp.scale = d->scale; kp.bias = d->bias; kp.slope = d->slope; kp.act = d->act;
  kp.y = y.ptr; kp.ysn = y.sn; kp.ysh = y.sh; kp.ysw = y.sw; kp.Co = y.c; kp.y_planes = d->y_planes ? 1 : 0;
  kp.tiles_w = (y.w + UG_T - 1) / UG_T;
  kp.tiles_h = (y.h + UG_T - 1) / UG_T;
  const int64_t nwg = (int64_t)y.n * kp.tiles_w * kp.tiles_h;
  if (nwg <= 0 || nwg >= (1LL << 31)) return PRPE_EINVAL;
  kp.nwg = (int)nwg;
  hipLaunchKernelGGL(upgemm_kernel, dim3(kp.nwg), dim3(512), 0, as_stream(stream), kp);
  return launch_status();
}
