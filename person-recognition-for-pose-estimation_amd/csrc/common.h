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

// exp(x) from the hardware base-2 exponential (v_exp_f32, 1 ulp) with x*log2(e) carried in
// two parts (t + e), so the argument rounding does not grow with |x|: 2^(t+e) = 2^t (1 + e ln2)
// to ~2 ulp over the normal range; overflows to +inf and underflows to 0 like expf.
// 1 + e ln2 is within 2^-20 of 1, so it is finite and positive.
__device__ __forceinline__ float exp_hw(float x) {
  const float L = 1.44269502162933349609375f;     // log2(e) rounded to fp32
  const float Llo = 1.925963033500011e-08f;       // log2(e) - L
  const float t = x * L;
  const float e = fmaf(x, L, -t) + x * Llo;
  // r * (1 + e ln2), not fma(r, e ln2, r): an overflowed r = inf times a correction below 0
  // would give inf - inf = NaN
  return __builtin_amdgcn_exp2f(t) * (1.f + e * 0.693147180559945309f);
}

// erf(x) without branches (both pieces are evaluated; the select is per lane), ~24 VALU
// instead of libm erff's two-branch form with a full expf (~45 VALU under divergence):
//   |x| < 1 : x P(x^2), P of degree 5
//   |x| >= 1: 1 - exp(Q(min(|x|, 4))), Q of degree 8 fitted to log(erfc) on [1, 4] (erf
//             rounds to 1 in fp32 from |x| = 3.92 on)
// least-squares fits made for this kernel (relative error of erf(x)/x, absolute error of
// log erfc); max error 2.3 ulp over [-6, 6] in an fp32 emulation with exp_hw's 2 ulp, 1.5e-7
// absolute. test_epilogue_activation_accuracy checks GELU through it against fp64.
__device__ __forceinline__ float erf_fast(float x) {
  const float a = fabsf(x);
  const float t = a * a;
  float p = -0x1.26eecap-11f;
  p = fmaf(p, t, 0x1.422d30p-8f);
  p = fmaf(p, t, -0x1.b59da6p-6f);
  p = fmaf(p, t, 0x1.ce08bep-4f);
  p = fmaf(p, t, -0x1.812670p-2f);
  p = fmaf(p, t, 0x1.20dd74p+0f);
  const float ra = a * p;
  const float b = fminf(a, 4.f);
  float q = 0x1.b14578p-20f;
  q = fmaf(q, b, -0x1.7e711ep-15f);
  q = fmaf(q, b, 0x1.36c82ep-11f);
  q = fmaf(q, b, -0x1.36a7bcp-8f);
  q = fmaf(q, b, 0x1.aff5a4p-6f);
  q = fmaf(q, b, -0x1.c2788cp-4f);
  q = fmaf(q, b, -0x1.438d42p-1f);
  q = fmaf(q, b, -0x1.21529ap+0f);
  q = fmaf(q, b, 0x1.3df11ep-12f);
  const float rb = 1.f - exp_hw(q);
  return copysignf(a < 1.f ? ra : rb, x);
}

// Activation applied in every epilogue, accurate to a few ulp of the fp32 CPU reference:
// SiLU / sigmoid as v * rcp(1 + exp(-v)) (exp_hw, v_rcp_f32 1 ulp; ~10 VALU instead of the
// ~25 of expf + an IEEE division), GELU with erf_fast.
__device__ __forceinline__ float apply_act(float v, int act, float slope) {
  switch (act) {
    case PRPE_ACT_RELU: return v > 0.f ? v : 0.f;
    case PRPE_ACT_SILU: return v * __builtin_amdgcn_rcpf(1.f + exp_hw(-v));
    case PRPE_ACT_PRELU: return v >= 0.f ? v : v * slope;
    case PRPE_ACT_GELU: return 0.5f * v * (1.f + erf_fast(v * 0.70710678118654752440f));
    case PRPE_ACT_SIGMOID: return __builtin_amdgcn_rcpf(1.f + exp_hw(-v));
    default: return v;
  }
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
__device__ __forceinline__ int swzF(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }

// native vector types: HIP's float4/uint4 are structs, and arrays of them cannot be promoted
// to registers (the compiler moved them to a per-thread LDS array with 64-B lane stride)

static inline bool view_ok(const prpe_view* v) {
  return v && v->ptr && v->n > 0 && v->h > 0 && v->w > 0 && v->c > 0;
}
