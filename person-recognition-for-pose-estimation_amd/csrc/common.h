// Shared device helpers for the prpe HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "prpe.h"

#define PRPE_EINVAL (-22)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : static_cast<int>(e);
}

// Elementwise helpers for T = float or f32x2v (two lanes' worth in one VGPR pair: in VALU-bound
// kernels without MFMAs -- the upconv -- v_pk_fma_f32 / v_pk_mul_f32 issue one instruction per two
// values). Every multiply-add is an explicit fma and contraction is off, so the float and the
// f32x2v instantiations round identically (bit-identical results whichever a kernel uses).
typedef float f32x2v __attribute__((ext_vector_type(2)));
template <typename T> __device__ __forceinline__ T vfma(T a, T b, T c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ float vexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ f32x2v vexp2(f32x2v x) {
  return f32x2v{__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
}
__device__ __forceinline__ float vrcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ f32x2v vrcp(f32x2v x) { return f32x2v{__builtin_amdgcn_rcpf(x[0]), __builtin_amdgcn_rcpf(x[1])}; }
__device__ __forceinline__ float vsel_lt(float a, float lim, float x, float y) { return a < lim ? x : y; }
__device__ __forceinline__ float vsel_lt0(float a, float x, float y) { return a < 0.f ? x : y; }
__device__ __forceinline__ f32x2v vsel_lt0(f32x2v a, f32x2v x, f32x2v y) {
  return f32x2v{a[0] < 0.f ? x[0] : y[0], a[1] < 0.f ? x[1] : y[1]};
}
__device__ __forceinline__ f32x2v vsel_lt(f32x2v a, float lim, f32x2v x, f32x2v y) {
  return f32x2v{a[0] < lim ? x[0] : y[0], a[1] < lim ? x[1] : y[1]};
}

// exp(x) from the hardware base-2 exponential (v_exp_f32, 1 ulp) with x*log2(e) carried in
// two parts (t + e), so the argument rounding does not grow with |x|: 2^(t+e) = 2^t (1 + e ln2)
// to ~2 ulp over the normal range; overflows to +inf and underflows to 0 like expf.
// 1 + e ln2 is within 2^-20 of 1, so it is finite and positive; r * (1 + e ln2), not
// fma(r, e ln2, r): an overflowed r = inf times a correction below 0 would give inf - inf = NaN
template <typename T>
__device__ __forceinline__ T exp_hw_v(T x) {
#pragma clang fp contract(off)
  const T L = T(1.44269502162933349609375f);     // log2(e) rounded to fp32
  const T Llo = T(1.925963033500011e-08f);       // log2(e) - L
  const T t = x * L;
  const T e = vfma(x, Llo, vfma(x, L, -t));
  return vexp2(t) * vfma(e, T(0.693147180559945309f), T(1.f));
}
__device__ __forceinline__ float exp_hw(float x) { return exp_hw_v<float>(x); }

// GELU(v) = v Phi(v) in ONE branch (round 4; before: 0.5 v (1 + erf(v / sqrt 2)) with a
// two-piece erf, ~31 VALU): with b = min(|v| / sqrt 2, 4) and E = erfc(b) = exp(Q(b)),
//   v >= 0: v - (v / 2) E        v < 0: (v / 2) E
// Q(b) = b R(b), R of degree 10, a weighted least-squares fit of log erfc on [0, 4] made for this
// kernel (Q(0) = 0 exactly, so E(0) = 1); ~24 VALU. fp32 emulation against fp64: <= 1.3 ulp
// for |v| < 2, <= 15 ulp on [-4, -2] (the rounding of Q at |Q| ~ 8; the former erf form lost
// ~400 ulp there to 1 + erf cancelling); past |v| = 5.66 the result is v or -0 (the fp32 CPU
// reference gives -0 there too; the fp64 value is below 5e-8 in magnitude). erfc never cancels: the
// positive branch subtracts at most half of v. test_epilogue_activation_accuracy checks it
// against fp64.
template <typename T>
__device__ __forceinline__ T gelu_v(T v) {
#pragma clang fp contract(off)
  const T h = T(0.5f) * v;
  const T a = __builtin_elementwise_abs(v) * T(0.70710678118654752440f);
  const T b = __builtin_elementwise_min(a, T(4.f));
  T r = T(0x1.578a8cp-24f);
  r = vfma(r, b, T(-0x1.19e418p-19f));
  r = vfma(r, b, T(0x1.9b625ep-16f));
  r = vfma(r, b, T(-0x1.5c96f4p-13f));
  r = vfma(r, b, T(0x1.700bf2p-11f));
  r = vfma(r, b, T(-0x1.b89b64p-10f));
  r = vfma(r, b, T(0x1.37bf18p-14f));
  r = vfma(r, b, T(0x1.3babe4p-6f));
  r = vfma(r, b, T(-0x1.a53a7ap-4f));
  r = vfma(r, b, T(-0x1.45f11cp-1f));
  r = vfma(r, b, T(-0x1.20dd88p+0f));
  // (v/2) E = -0 past the fit (b clamped at 4): v - (v/2) erfc(4) rounds to v anyway. The select
  // is on the product, so v = +-inf gives v - (-0) = +inf / -0 (not inf * 0 = NaN), and the branch
  // test is v < 0, so a NaN takes the v - hE side and stays NaN
  const T hE = vsel_lt(a, 4.f, h * exp_hw_v(r * b), T(-0.f));
  return vsel_lt0(v, hE, v - hE);
}
template <typename T>
__device__ __forceinline__ T sigmoid_v(T v) {
#pragma clang fp contract(off)
  return vrcp(T(1.f) + exp_hw_v(-v));
}

// Activation applied in every epilogue, accurate to a few ulp of the fp32 CPU reference:
// SiLU / sigmoid as v * rcp(1 + exp(-v)) (exp_hw, v_rcp_f32 1 ulp; ~10 VALU instead of the
// ~25 of expf + an IEEE division), GELU in one branch (gelu_v).
__device__ __forceinline__ float apply_act(float v, int act, float slope) {
  switch (act) {
    case PRPE_ACT_RELU: return v > 0.f ? v : 0.f;
    case PRPE_ACT_SILU: return v * sigmoid_v(v);
    case PRPE_ACT_PRELU: return v >= 0.f ? v : v * slope;
    case PRPE_ACT_GELU: return gelu_v(v);
    case PRPE_ACT_SIGMOID: return sigmoid_v(v);
    default: return v;
  }
}

// the same activation on 4 values, two at a time in packed fp32 (VALU-only kernels: the
// upconv); bit-identical to apply_act element by element
__device__ __forceinline__ f32x4 apply_act4(f32x4 v, int act, f32x4 slope) {
  if (act == PRPE_ACT_GELU || act == PRPE_ACT_SILU || act == PRPE_ACT_SIGMOID) {
    f32x2v lo = {v[0], v[1]}, hi = {v[2], v[3]};
    if (act == PRPE_ACT_GELU) {
      lo = gelu_v(lo);
      hi = gelu_v(hi);
    } else if (act == PRPE_ACT_SILU) {
      lo = lo * sigmoid_v(lo);
      hi = hi * sigmoid_v(hi);
    } else {
      lo = sigmoid_v(lo);
      hi = sigmoid_v(hi);
    }
    return f32x4{lo[0], lo[1], hi[0], hi[1]};
  }
  f32x4 r;
#pragma unroll
  for (int q = 0; q < 4; ++q) r[q] = apply_act(v[q], act, slope[q]);
  return r;
}

// fp32 -> (hi, lo) bf16 pair, hi = RNE(x), lo = RNE(x - hi). |x - hi - lo| <= 2^-17 |x|.
__device__ __forceinline__ void split_bf16(float x, __bf16& hi, __bf16& lo) {
  hi = (__bf16)x;
  lo = (__bf16)(x - (float)hi);
}

// 4 consecutive channels c .. c+3 (c % 4 == 0) of one pixel in the planes format (prpe.h,
// prpe_conv_desc): channel group c / 8 holds hi[8] then lo[8], hi = RNE(v), lo = RNE(v - hi).
// row16: the pixel's first bf16 slot. The remainder is an explicit v_sub_f32: with FP
// contraction the compiler would fuse a producing multiply into it (fma(a, b, -hi)) and the
// planes would no longer be the split of the stored fp32 value.
// NT: non-temporal stores (streaming; the output is not re-read by this kernel)
template <bool NT = false>
__device__ __forceinline__ void store_planes4(uint16_t* row16, int c, f32x4 v) {
  uint16_t* y16 = row16 + (c >> 3) * 16 + (c & 7);
  unsigned short hi[4], lo[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x = v[e];
    const __bf16 h = (__bf16)x;
    float d;
    asm("v_sub_f32 %0, %1, %2" : "=v"(d) : "v"(x), "v"((float)h));
    hi[e] = __builtin_bit_cast(unsigned short, h);
    lo[e] = __builtin_bit_cast(unsigned short, (__bf16)d);
  }
  const unsigned long long h64 = (unsigned long long)(hi[0] | (unsigned)hi[1] << 16) |
                                 (unsigned long long)(hi[2] | (unsigned)hi[3] << 16) << 32;
  const unsigned long long l64 = (unsigned long long)(lo[0] | (unsigned)lo[1] << 16) |
                                 (unsigned long long)(lo[2] | (unsigned)lo[3] << 16) << 32;
  if constexpr (NT) {
    __builtin_nontemporal_store(h64, reinterpret_cast<unsigned long long*>(y16));
    __builtin_nontemporal_store(l64, reinterpret_cast<unsigned long long*>(y16 + 8));
  } else {
    *reinterpret_cast<unsigned long long*>(y16) = h64;
    *reinterpret_cast<unsigned long long*>(y16 + 8) = l64;
  }
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double warp_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware block remap (MI355X: blocks b and b+8 share an XCD/L2).
// Consecutive logical ids land on the same XCD, so tiles that share an operand panel
// share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  int xcd = bid % nx, q = nwg / nx, r = nwg % nx;
  int start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + bid / nx;
}

// max |v| of a float4 (NaN lanes are ignored by fmaxf)
__device__ __forceinline__ float amax4(f32x4 v) {
  return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
}
// raise *slot to the wave's maximum of m (m >= 0: float order == unsigned bit order); every
// lane of the wave must call it
__device__ __forceinline__ void amax_raise(float* slot, float m) {
  // the slot only grows, so read it first (an agent-scope load, past the non-coherent L1) and
  // only raise it when m is larger -- a stale read can only cost a redundant atomic
  unsigned* u = reinterpret_cast<unsigned*>(slot);
  const unsigned b = __float_as_uint(m);
  if (b > __hip_atomic_load(u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(u, b);
}
__device__ __forceinline__ void amax_commit(float* slot, float m) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0 && m > 0.f) amax_raise(slot, m);
}

// Per-FRAME max|y| (prpe.h, "max|y| slots"): slots[n] bounds |y| over frame n only, so a
// frame's precision-3 scale never depends on its batch-mates. A lane visits its rows in
// increasing order and keeps (frame, running max); when its frame changes it raises the old
// frame's slot itself. frame_amax_final: when every lane with a maximum is on the same frame
// (a wave inside one frame: the common case) one wave reduction and one atomic, else one
// atomic per lane. Every lane of the wave must call it.
struct FrameMax {
  int n = -1;
  float m = 0.f;
  __device__ __forceinline__ void add(float* slots, int frame, float v) {
    if (frame != n) {
      if (n >= 0 && m > 0.f) amax_raise(slots + n, m);
      n = frame;
      m = 0.f;
    }
    m = fmaxf(m, v);
  }
};
__device__ __forceinline__ void frame_amax_final(float* slots, FrameMax f) {
  int nmax = f.m > 0.f ? f.n : -1;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nmax = max(nmax, __shfl_xor(nmax, o, 64));
  if (nmax < 0) return;
  if (__all(f.m <= 0.f || f.n == nmax)) {
    amax_commit(slots + nmax, f.m > 0.f ? f.m : 0.f);
  } else if (f.n >= 0 && f.m > 0.f) {
    amax_raise(slots + f.n, f.m);
  }
}

// precision-3 activation scale of one frame: max|x| < 2^e -> x 2^(15-e) (e clamped; an
// all-zero frame takes e = 15, scale 1). Both the operand split and the epilogue's inverse
// derive from this one function, so they agree exactly.
__device__ __forceinline__ int f16_scale_exp(float amax) {
  int e = 0;
  (void)frexpf(amax, &e);
  return amax > 0.f ? (e < -60 ? -60 : (e > 60 ? 60 : e)) : 15;
}

// F = {0,2,3,1} indexed by (row >> 2) & 3, branch-free
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// buffer-descriptor LDS-DMA: one piece of 16 B per lane from the descriptor's base + voff + soff
// (bytes; voff per lane, soff wave-uniform) to dst_lds + 16 * lane (dst wave-uniform). An offset
// at or past the descriptor's num_records reads zeros (the padding idiom of conv_halo.hip).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, int num_bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, num_bytes, 0x00020000);
}
__device__ __forceinline__ void bl_lds16(__amdgpu_buffer_rsrc_t r, void* dst_lds, unsigned voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(dst_lds), 16, voff, soff, 0, 0);
}
// the same with the non-temporal policy (cache-policy bit nt): for input streamed once per tile,
// so L2 evicts it first and keeps the weight planes every workgroup re-reads (conv_halo.hip)
__device__ __forceinline__ void bl_lds16_nt(__amdgpu_buffer_rsrc_t r, void* dst_lds, unsigned voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(dst_lds), 16, voff, soff, 0, 2);
}
constexpr unsigned BL_OOB = 0x80000000u;   // a voffset past every descriptor's range (num_records < 2^31)

__device__ __forceinline__ int swzF(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }

// native vector types: HIP's float4/uint4 are structs, and arrays of them cannot be promoted
// to registers (the compiler moved them to a per-thread LDS array with 64-B lane stride)

static inline bool view_ok(const prpe_view* v) {
  return v && v->ptr && v->n > 0 && v->h > 0 && v->w > 0 && v->c > 0;
}

// byte range [lo, hi) a view can touch (float elements; negative strides included)
static inline void view_span(const prpe_view& v, uintptr_t& lo, uintptr_t& hi) {
  const int64_t ext[4] = {(int64_t)(v.n - 1) * v.sn, (int64_t)(v.h - 1) * v.sh, (int64_t)(v.w - 1) * v.sw,
                          (int64_t)(v.c - 1) * v.sc};
  int64_t a = 0, b = 0;
  for (int i = 0; i < 4; ++i) (ext[i] < 0 ? a : b) += ext[i];
  lo = (uintptr_t)v.ptr + a * 4;
  hi = (uintptr_t)v.ptr + (b + 1) * 4;
}
// do two byte ranges intersect (kernels that read one tensor's neighbourhood while writing the
// other must not run in place)
static inline bool spans_overlap(uintptr_t alo, uintptr_t ahi, uintptr_t blo, uintptr_t bhi) {
  return alo < bhi && blo < ahi;
}
static inline bool views_overlap(const prpe_view& a, const prpe_view& b) {
  uintptr_t alo, ahi, blo, bhi;
  view_span(a, alo, ahi);
  view_span(b, blo, bhi);
  return spans_overlap(alo, ahi, blo, bhi);
}
