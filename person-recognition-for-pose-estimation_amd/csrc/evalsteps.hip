// Device halves of the reference eval steps around the model.
//   flip_average : pose flip test, flip-back + pair handling + average
//                  (pose_estimation/module.py:470-484)
//   ce_argmax    : face-recognition eval head, per-row cross-entropy and argmax of the
//                  scaled cosine logits (face_recognition/module.py:137-145)
#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr int MAX_K = 64;

struct FlipK {
  const float* heat; const float* flip; float* out;
  int B, K, H, W, mode;
  int partner[MAX_K];
};

// out[b,k,h,w] = (heat[b,k,h,w] + flip[b', k', h, W-1-w]) * 0.5
//   mode 0 (reference): k' = k, b' = B-1-b for every channel of a flip pair
//          (``flipped[:, pair] = flipped[:, pair].flip(0)`` reverses the batch dimension)
//   mode 1 (channel swap): b' = b, k' = partner[k]
// grid: one block per (b, k, h) row, threads over w
__global__ __launch_bounds__(256) void flip_average_kernel(FlipK p) {
  const int row = blockIdx.x;
  const int h = row % p.H;
  const int bk = row / p.H;
  const int k = bk % p.K, b = bk / p.K;
  int b2 = b, k2 = k;
  const int pk = p.partner[k];
  if (pk >= 0) {
    if (p.mode == 0) b2 = p.B - 1 - b;
    else k2 = pk;
  }
  const float* src = p.heat + ((int64_t)bk * p.H + h) * p.W;
  const float* fs = p.flip + (((int64_t)b2 * p.K + k2) * p.H + h) * p.W;
  float* dst = p.out + ((int64_t)bk * p.H + h) * p.W;
  for (int w = threadIdx.x; w < p.W; w += blockDim.x) dst[w] = (src[w] + fs[p.W - 1 - w]) * 0.5f;
}

// one block per row: first-occurrence argmax (NaN counts as the maximum, like torch.max), and
// loss = logsumexp(row) - row[label] (double accumulation of the exponentials)
__global__ __launch_bounds__(256) void ce_argmax_kernel(const float* logits, int64_t ld, int C,
                                                        const int64_t* labels, float* loss, int* amax) {
  const int r = blockIdx.x;
  const float* x = logits + (int64_t)r * ld;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ float s_v[4];
  __shared__ int s_i[4];
  __shared__ double s_d[4];
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float v = x[c];
    const bool better = (v != v) ? !(bv != bv) : (v > bv);   // first NaN wins, then strict >
    if (better) { bv = v; bi = c; }
  }
  // combine (value, index): larger value, NaN above all, ties -> smaller index
  auto take = [](float av, int ai, float ov, int oi, float& rv, int& ri) {
    const bool an = av != av, on = ov != ov;
    bool pick_o;
    if (an || on) pick_o = on && (!an || oi < ai);
    else pick_o = ov > av || (ov == av && oi < ai);
    rv = pick_o ? ov : av;
    ri = pick_o ? oi : ai;
  };
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(bv, off);
    const int oi = __shfl_xor(bi, off);
    take(bv, bi, ov, oi, bv, bi);
  }
  if (lane == 0) { s_v[wave] = bv; s_i[wave] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) take(bv, bi, s_v[w], s_i[w], bv, bi);
    s_v[0] = bv; s_i[0] = bi;
    amax[r] = bi;
  }
  __syncthreads();
  if (!labels) return;
  const float mx = s_v[0];
  double s = 0.0;
  for (int c = threadIdx.x; c < C; c += blockDim.x) s += exp((double)x[c] - (double)mx);
  s = warp_sum_d(s);
  if (lane == 0) s_d[wave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double tot = s_d[0] + s_d[1] + s_d[2] + s_d[3];
    const int64_t lb = labels[r];
    const float xl = (lb >= 0 && lb < C) ? x[lb] : NAN;
    loss[r] = (float)(log(tot) + (double)mx - (double)xl);
  }
}

// summary[0] = mean loss (F.cross_entropy 'mean'), summary[1] = mean(argmax == label)
__global__ __launch_bounds__(256) void ce_summary_kernel(const float* loss, const int* amax, const int64_t* labels,
                                                         int B, float* summary) {
  double s = 0.0, a = 0.0;
  for (int r = threadIdx.x; r < B; r += blockDim.x) {
    s += loss[r];
    a += (amax[r] == labels[r]) ? 1.0 : 0.0;
  }
  __shared__ double red[2][4];
  s = warp_sum_d(s); a = warp_sum_d(a);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { red[0][wave] = s; red[1][wave] = a; }
  __syncthreads();
  if (threadIdx.x == 0) {
    summary[0] = (float)((red[0][0] + red[0][1] + red[0][2] + red[0][3]) / B);
    summary[1] = (float)((red[1][0] + red[1][1] + red[1][2] + red[1][3]) / B);
  }
}

}  // namespace

extern "C" int prpe_flip_average(const float* heat, const float* heat_flipped, float* out, int32_t B, int32_t K,
                                 int32_t H, int32_t W, const int32_t* partner, int32_t mode, void* stream) {
  if (!heat || !heat_flipped || !out || B <= 0 || K <= 0 || K > MAX_K || H <= 0 || W <= 0) return PRPE_EINVAL;
  if (mode != 0 && mode != 1) return PRPE_EINVAL;
  if (out == heat_flipped) return PRPE_EINVAL;   // the flipped map is read at other (b, k, w)
  FlipK p{};
  p.heat = heat; p.flip = heat_flipped; p.out = out;
  p.B = B; p.K = K; p.H = H; p.W = W; p.mode = mode;
  for (int k = 0; k < K; ++k) {
    const int q = partner ? partner[k] : -1;
    if (q >= K) return PRPE_EINVAL;
    p.partner[k] = q;
  }
  const int64_t rows = (int64_t)B * K * H;
  if (rows >= (1LL << 31)) return PRPE_EINVAL;
  hipLaunchKernelGGL(flip_average_kernel, dim3((unsigned)rows), dim3(W >= 256 ? 256 : 64), 0, as_stream(stream), p);
  return launch_status();
}

extern "C" int prpe_ce_argmax(const float* logits, int64_t ld, int32_t B, int32_t C, const int64_t* labels,
                              float* loss, int32_t* argmax, float* summary, void* stream) {
  if (!logits || !argmax || B <= 0 || C <= 0 || ld < C) return PRPE_EINVAL;
  if (labels && !loss) return PRPE_EINVAL;
  if (summary && !labels) return PRPE_EINVAL;
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(ce_argmax_kernel, dim3(B), dim3(256), 0, st, logits, ld, C, labels, loss, argmax);
  if (summary) hipLaunchKernelGGL(ce_summary_kernel, dim3(1), dim3(256), 0, st, loss, argmax, labels, B, summary);
  return launch_status();
}
