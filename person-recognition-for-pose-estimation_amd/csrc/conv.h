// Shared definitions of the two implicit-GEMM conv kernels (conv_igemm.hip: register-staged,
// any layout; conv_glds.hip: direct global->LDS staging for channel-chunked inputs).
#pragma once
#include "common.h"
#include <type_traits>

namespace prpe_k {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// Kernel arguments of prpe_conv2d (host-validated, see conv_igemm.hip)
struct ConvK {
  const float* x; int64_t xsn, xsh, xsw, xsc; int Hi, Wi, Ci;
  float* y; int64_t ysn, ysh, ysw, ysc; int Ho, Wo, Co;
  const float* r; int64_t rsn, rsh, rsw, rsc;
  int KH, KW, stride, pad, K, k_pad, nk;
  const uint16_t* whi; const uint16_t* wlo; const uint16_t* wlo2;
  const float* scale; const float* bias; const float* slope;
  const float* in_scale; const float* in_bias;
  int act, res_mode, vec_out;
  int M, HoWo, tiles_n, nwg;
  const float* zero;   // &g_zero8 on this device (a kernel argument, so the K-loop does not
                       // re-load the symbol's address from the GOT every step); 32 zero bytes
  int ylin, rlin;      // y (r) offset of pixel m is m * ysw (rsw): contiguous pixels, so the
                       // epilogue skips the m -> (n, oh, ow) division
  const uint16_t* wh16; const uint16_t* wl16;   // precision 3: fp16 planes of the scaled weights
  const float* x_amax;                          // precision 3: upper bound of max|x| (device)
  float* y_amax;                                // optional: raised to max|y| (device, atomic)
  const float* x2; int64_t x2sn, x2sh, x2sw;    // dual input (conv_wave only), see prpe.h
  int nk1;                                      // K-steps of the first input
  const float* x2_amax;
  int x_planes, y_planes;                       // planes format input / output (conv_wave)
  const float* w2; float* y2; int64_t y2sn, y2sh, y2sw; int n2;   // epilogue 1x1 GEMM (conv_halo)
  const float* w3; const float* s2; const float* b2; int act2; int nmid;     // its second stage
};

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// fp32 x4 -> NP bf16 planes, two lanes at a time: hi = RNE(v) (v_cvt_pk_bf16_f32), its fp32
// value rebuilt by a shift / mask, the (exact) remainder by one scalar v_sub_f32 per element,
// and so on per plane. The compiler's per-element lowering of the same casts took 13 VALU per
// float4 at NP 2; its SLP-packed v_pk_add_f32 for the remainder costs extra issue cycles
// beside MFMAs (MI355X_MICROARCH.md, "price of one filler"), hence the explicit scalar subtract
// (measured +2..7 % on the MFMA-bound 3x3 convs, bit-identical).
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float sub_f32(float a, float b) {
  float d;
  asm("v_sub_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
// 16-B slot swizzles of [pixel][128-B line] LDS tiles whose fragments are read by ds_read_b128:
// a read is serviced in four 16-lane groups, each holding fragment rows fr = {0-3, 12-15} at
// logical slot L and rows {4-11} at L ^ 2 (MI355X_MICROARCH.md, LDS), and 128-B lines put even
// and odd pixels in opposite halves of the 256-B bank row. A lane's physical slot is its logical
// slot XOR swz(pixel); conflict-free means all 16 lanes of a group on distinct (parity, slot).
// swz_rows: fragments of 16 consecutive pixels starting at a multiple of 16 (GEMM row blocks):
//   f(r) = (r >> 1) & 5 puts {f} of one row set and {f ^ 2} of the other on all 8 slots per parity.
// swz_halo: 16-pixel windows starting at column 0, 1 or 2 (or 16, 17, 18) of a haloed tile row
//   (the 3x3 taps): a function of the column (rows of 18 or 34 pixels start at even indices),
//   period 16, found by exhaustive search (tools/exp/halo_swizzle.py). The earlier (q >> 1) & 7
//   was 2-way on most groups.
__device__ __forceinline__ int swz_rows(int r) { return (r >> 1) & 5; }
__device__ __forceinline__ int swz_halo(int col) { return (0xb29108 >> (((col >> 1) & 7) * 3)) & 7; }

template <int NP>
__device__ __forceinline__ void split_planes(f4 v, bf16x4 (&pl)[NP]) {
  float r[4] = {v[0], v[1], v[2], v[3]};
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    unsigned u[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bf16x2v b = __builtin_convertvector(f2v{r[2 * h], r[2 * h + 1]}, bf16x2v);
      u[h] = __builtin_bit_cast(unsigned, b);
      if (q + 1 < NP) {
        r[2 * h] = sub_f32(r[2 * h], __builtin_bit_cast(float, u[h] << 16));
        r[2 * h + 1] = sub_f32(r[2 * h + 1], __builtin_bit_cast(float, u[h] & 0xffff0000u));
      }
    }
    pl[q] = __builtin_bit_cast(bf16x4, (unsigned long long)u[0] | ((unsigned long long)u[1] << 32));
  }
}

// fp32 x4 -> two fp16 planes (packed 4 x f16 each) of v * sa: hi = RTZ(v sa)
// (v_cvt_pkrtz_f16_f32), lo = RTZ(v sa - hi) with the remainder exact in fp32; |v sa| < 2^15
// by the choice of sa, so neither plane overflows and v sa = hi + lo to ~2^-21 relative
// (lo can be subnormal for tiny v: absolute error <= 2^-25 in scaled units)
__device__ __forceinline__ void split_planes_f16(f4 v, float sa, unsigned long long (&pl)[2]) {
  float r[4] = {v[0] * sa, v[1] * sa, v[2] * sa, v[3] * sa};
  unsigned u[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const auto hi = __builtin_amdgcn_cvt_pkrtz(r[2 * h], r[2 * h + 1]);
    u[0][h] = __builtin_bit_cast(unsigned, hi);
    // r - hi straight from the packed fp16 halves (v_fma_mix_f32: -1 * f16 + f32, one VALU
    // instead of v_cvt_f32_f16 + v_sub_f32; exact, as the remainder is representable in fp32)
    float d0, d1;
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d0) : "v"(u[0][h]), "v"(r[2 * h]));
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d1) : "v"(u[0][h]), "v"(r[2 * h + 1]));
    u[1][h] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(d0, d1));
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) pl[q] = (unsigned long long)u[q][0] | ((unsigned long long)u[q][1] << 32);
}

// precision 4: fp32 x8 -> ONE fp16 plane of v * sa (RNE, v_cvt_pk_f16_f32), one MFMA per
// product. |v sa| < 2^15 by the choice of sa (as precision 3); operand error 2^-12 relative.
__device__ __forceinline__ f16x8 cvt_f16_one(f4 v0, f4 v1, float sa) {
  typedef _Float16 h2v __attribute__((ext_vector_type(2)));
  const h2v a = __builtin_convertvector(f2v{v0[0] * sa, v0[1] * sa}, h2v);
  const h2v b = __builtin_convertvector(f2v{v0[2] * sa, v0[3] * sa}, h2v);
  const h2v c = __builtin_convertvector(f2v{v1[0] * sa, v1[1] * sa}, h2v);
  const h2v d = __builtin_convertvector(f2v{v1[2] * sa, v1[3] * sa}, h2v);
  return f16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

// the input-side affine s x + b, fused (one rounding per element), so the wave-row and
// haloed-tile kernels round the prologue's output identically
__device__ __forceinline__ f4 affine4(f4 v, f4 s, f4 b) {
  return f4{fmaf(v[0], s[0], b[0]), fmaf(v[1], s[1], b[1]), fmaf(v[2], s[2], b[2]), fmaf(v[3], s[3], b[3])};
}

// precision 4 with an input-side affine (IR-50 pre-BN prologue): an upper bound of
// max|s x + b| over the frame = amax(x) max|s| + max|b|, with max|s| and max|b| over the Ci
// prologue channels reduced here (every lane gets the wave's maxima). A loose bound only costs
// low-order bits of the scaled operand, never range.
__device__ __forceinline__ void prologue_bounds(const float* s, const float* b, int ci, float& ms, float& mb) {
  ms = 0.f;
  mb = 0.f;
  for (int c = threadIdx.x & 63; c < ci; c += 64) {
    ms = fmaxf(ms, fabsf(s[c]));
    mb = fmaxf(mb, fabsf(b[c]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ms = fmaxf(ms, __shfl_xor(ms, o, 64));
    mb = fmaxf(mb, __shfl_xor(mb, o, 64));
  }
}

typedef __attribute__((address_space(1))) void* gbl_ptr_t;

// one LDS-DMA piece: 16 B per lane from src (per lane) to dst_lds + 16 * lane (dst wave-uniform)
__device__ __forceinline__ void glds16(const void* src, void* dst_lds) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src), (lds_ptr_t)(dst_lds), 16, 0, 0);
}

// 16 B per lane into registers through a buffer descriptor (base + voff + soff, bytes); zeros
// at or past num_records
__device__ __forceinline__ f4 bl_f4(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// s_waitcnt vmcnt(N) + s_barrier in one asm statement with a memory clobber, fenced by
// sched_barrier(0) on both sides. It does not drain the LDS-DMA copies still in flight (a
// __syncthreads() would emit vmcnt(0) here). The memory clobber alone does not stop the machine
// scheduler: it hoisted the next K-step's ds_reads above the s_barrier in conv_bneck.hip, i.e.
// a wave read a ring stage before the other waves' DMA pieces of it were known to have landed
// (a race: run-to-run differences at bs = 256; tools/barrier_hoist_check.py finds such reads).
template <int N>
__device__ __forceinline__ void wait_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// a workgroup barrier for LDS traffic only: this wave's LDS writes done, then s_barrier.
// __syncthreads() also fences global memory, i.e. waits vmcnt(0), draining every load, store
// and LDS-DMA in flight (the in-order counter) where only LDS ordering is needed.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// direct global->LDS kernel (conv_glds.hip): Ci % 32 == 0 channel-contiguous input, chunk-major
// weights, precision 0 or 2, no prologue; tile 0 = auto, 10..12 = 256x128 / 256x64 / 128x128.
// Returns PRPE_EINVAL when the shape is not eligible.
bool conv_glds_eligible(const ConvK& kp, int prec, int km);
int conv_glds_launch(const ConvK& kp, int prec, int tile, hipStream_t st);

// wave-row kernel (conv_wave.hip): A straight into MFMA fragment registers, B planes through
// an LDS-DMA ring; chunked inputs, precision 0 / 2, optional prologue affine; tile 20 = auto,
// 21..25 force a configuration.
bool conv_wave_eligible(const ConvK& kp, int prec, int km);
int conv_wave_launch(const ConvK& kp, int prec, int tile, hipStream_t st);

// haloed-tile 3x3 kernel (conv_halo.hip): 3x3 / s1 / p1, chunk-major weights, precision 0
// (fp32 or planes input), 3 or 4; tile 30 = auto, 31..35 force a configuration.
bool conv_halo_eligible(const ConvK& kp, int prec, int km, int tile = 30);   // tile: 30 (auto) or 31..37
bool conv_halo_auto(const ConvK& kp, int prec);   // the automatic choice's shape rule

// 256-row GEMM kernel (conv_gemm.hip) for 1x1 / s1 convs over contiguous pixels, Co % 128 == 0,
// precision 0 (fp32 or planes input) or 3; tiles 40..42.
bool conv_gemm_eligible(const ConvK& kp, int prec);
int conv_gemm_launch(const ConvK& kp, int prec, int tile, hipStream_t st);
int conv_halo_launch(const ConvK& kp, int prec, int tile, hipStream_t st);
bool conv_splitk_eligible(const ConvK& kp, int prec, int k_order);
int64_t conv_splitk_workspace_bytes(const ConvK& kp);
int conv_splitk_launch(const ConvK& kp, float* workspace, hipStream_t st);

}  // namespace prpe_k
