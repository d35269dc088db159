// Post-processing: batched NMS and heatmap soft-argmax (wavefront-reduction kernels).
//
// prpe_nms — yolopt.util.non_max_suppression (training/yolopt/util.py:123-169) incl. the
// torchvision.ops.nms it calls (util.py:162), one 1024-thread workgroup per image:
//   1. candidates in the reference's enumeration order: box a ascending, class j ascending
//      (nc==1: best class of a box; nc>1: every (a,j) with a passing box-max and score>conf),
//      compacted with a block prefix sum;
//   2. 64-bit keys (~orderable(score) << 32 | enumeration index) sorted ascending by an LDS
//      bitonic sort == stable descending score sort (ties by index);
//   3. greedy suppression by one wavefront against the kept list (<= max_det boxes, LDS):
//      each lane tests a slice of the kept boxes, __ballot decides; keep until max_det.
// IoU in fp32 exactly as torchvision's CPU kernel (boxes offset by 7680*cls first,
// area = (x2-x1)*(y2-y1), inter / (area_i + area_j - inter) > thr). FP contraction is off
// in this file so every product/sum rounds like the reference.
//
// prpe_softargmax — PoseEstimationModule._get_keypoints_from_heatmaps
// (training/lightning/pose_estimation/module.py:237-296), one 256-thread workgroup per
// (frame, keypoint): max, sum exp, expectation of x and y, max prob, optional box scale.
#pragma clang fp contract(off)
#include "common.h"

namespace {

constexpr int NMS_THREADS = 1024;
constexpr int NMS_MAX_CAND = 16384;   // LDS key capacity (128 KiB)
constexpr int NMS_MAX_DET = 1024;

__device__ __forceinline__ uint32_t orderable(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

struct NmsK {
  const float* pred; int B, N, nc; int64_t s_img, s_c, s_a;
  float conf, iou; int max_nms, max_det;
  float* out; int* count;
};

__device__ __forceinline__ float pred_at(const NmsK& p, int b, int c, int a) {
  return p.pred[(int64_t)b * p.s_img + (int64_t)c * p.s_c + (int64_t)a * p.s_a];
}

__global__ __launch_bounds__(NMS_THREADS) void nms_kernel(NmsK p) {
  __shared__ unsigned long long keys[NMS_MAX_CAND];
  __shared__ float kept[NMS_MAX_DET][5];   // offset box x1,y1,x2,y2 + area
  __shared__ int wsum[NMS_THREADS / 64];
  __shared__ int s_total, s_nk;
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t npairs = (int64_t)p.N * p.nc;

  // ---- 1. enumerate candidates in reference order, compacted
  if (tid == 0) s_total = 0;
  __syncthreads();
  for (int64_t base = 0; base < npairs; base += NMS_THREADS) {
    const int64_t e = base + tid;
    int flag = 0;
    float score = 0.f;
    if (e < npairs) {
      const int a = (int)(e / p.nc), j = (int)(e % p.nc);
      // box-level candidate mask xc: amax over classes (NaN propagates, torch amax)
      float mx = -INFINITY;
      bool nan = false;
      for (int c = 0; c < p.nc; ++c) {
        const float v = pred_at(p, b, 4 + c, a);
        nan |= (v != v);
        mx = fmaxf(mx, v);
      }
      const bool xc = !nan && mx > p.conf;
      if (p.nc == 1) {
        score = mx;
        flag = xc && score > p.conf;
      } else {
        score = pred_at(p, b, 4 + j, a);
        flag = xc && score > p.conf;
      }
    }
    // block exclusive scan of flags
    const unsigned long long bal = __ballot(flag);
    const int wpre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < NMS_THREADS / 64; ++w) {
      if (w < wave) off += wsum[w];
      tot += wsum[w];
    }
    const int pos = s_total + off + wpre;
    if (flag && pos < NMS_MAX_CAND)
      keys[pos] = ((unsigned long long)(~orderable(score)) << 32) | (unsigned long long)(uint32_t)e;
    __syncthreads();
    if (tid == 0) s_total += tot;
    __syncthreads();
  }
  const int total = s_total < NMS_MAX_CAND ? s_total : NMS_MAX_CAND;

  // ---- 2. bitonic sort of keys[0..P) ascending, P = next pow2
  int P = 1;
  while (P < total) P <<= 1;
  for (int i = total + tid; i < P; i += NMS_THREADS) keys[i] = ~0ull;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += NMS_THREADS) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = keys[i], c = keys[ixj];
          const bool up = (i & k) == 0;
          if ((a > c) == up) { keys[i] = c; keys[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }

  // ---- 3. greedy suppression (wave 0)
  const int ncand = total < p.max_nms ? total : p.max_nms;
  float* outb = p.out + (int64_t)b * p.max_det * 6;
  if (wave == 0) {
    int nk = 0;
    for (int i = 0; i < ncand && nk < p.max_det; ++i) {
      const unsigned long long key = keys[i];
      const int e = (int)(uint32_t)(key & 0xffffffffull);
      const int a = e / p.nc, j = e % p.nc;
      const float cx = pred_at(p, b, 0, a), cy = pred_at(p, b, 1, a);
      const float w = pred_at(p, b, 2, a), h = pred_at(p, b, 3, a);
      const float x1 = cx - w / 2.f, y1 = cy - h / 2.f, x2 = cx + w / 2.f, y2 = cy + h / 2.f;
      const float score = p.nc == 1 ? pred_at(p, b, 4, a) : pred_at(p, b, 4 + j, a);
      const float cls = (float)j;
      const float off = cls * 7680.f;
      const float ox1 = x1 + off, oy1 = y1 + off, ox2 = x2 + off, oy2 = y2 + off;
      const float area = (ox2 - ox1) * (oy2 - oy1);
      bool sup = false;
      for (int t = lane; t < nk; t += 64) {
        const float xx1 = fmaxf(kept[t][0], ox1), yy1 = fmaxf(kept[t][1], oy1);
        const float xx2 = fminf(kept[t][2], ox2), yy2 = fminf(kept[t][3], oy2);
        const float iw = fmaxf(0.f, xx2 - xx1), ih = fmaxf(0.f, yy2 - yy1);
        const float inter = iw * ih;
        const float ovr = inter / (kept[t][4] + area - inter);
        sup |= ovr > p.iou;
      }
      const bool any = __ballot(sup) != 0ull;
      if (!any) {
        if (lane == 0) {
          kept[nk][0] = ox1; kept[nk][1] = oy1; kept[nk][2] = ox2; kept[nk][3] = oy2; kept[nk][4] = area;
          float* o = outb + (int64_t)nk * 6;
          o[0] = x1; o[1] = y1; o[2] = x2; o[3] = y2; o[4] = score; o[5] = cls;
        }
        ++nk;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
    }
    if (lane == 0) s_nk = nk;
  }
  __syncthreads();
  const int nk = s_nk;
  for (int i = nk * 6 + tid; i < p.max_det * 6; i += NMS_THREADS) outb[i] = 0.f;
  // -1 flags a candidate overflow (> NMS_MAX_CAND): the result would not be exact
  if (tid == 0) p.count[b] = s_total > NMS_MAX_CAND ? -1 : nk;
}

// ----------------------------------------------------------------------------- soft-argmax
__global__ __launch_bounds__(256) void softargmax_kernel(const float* heat, int K, int H, int W, const float* boxes,
                                                         float* coords, float* scores, int* argmax) {
  const int bk = blockIdx.x;
  const int b = bk / K;
  const int HW = H * W;
  const float* x = heat + (int64_t)bk * HW;
  __shared__ float rm[4];
  __shared__ int ri[4];
  __shared__ float rs[4][3];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float m = -INFINITY;
  int mi = 0x7fffffff;
  for (int i = tid; i < HW; i += 256) {
    const float v = x[i];
    if (v > m || (v == m && i < mi)) { m = v; mi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oi = __shfl_xor(mi, o, 64);
    if (om > m || (om == m && oi < mi)) { m = om; mi = oi; }
  }
  if (lane == 0) { rm[wave] = m; ri[wave] = mi; }
  __syncthreads();
  m = rm[0]; mi = ri[0];
  for (int w = 1; w < 4; ++w)
    if (rm[w] > m || (rm[w] == m && ri[w] < mi)) { m = rm[w]; mi = ri[w]; }
  float se = 0.f, sx = 0.f, sy = 0.f;
  for (int i = tid; i < HW; i += 256) {
    const float e = expf(x[i] - m);
    se += e;
    sx += e * (float)(i % W);
    sy += e * (float)(i / W);
  }
  se = warp_sum(se); sx = warp_sum(sx); sy = warp_sum(sy);
  if (lane == 0) { rs[wave][0] = se; rs[wave][1] = sx; rs[wave][2] = sy; }
  __syncthreads();
  if (tid == 0) {
    const float S = (rs[0][0] + rs[1][0]) + (rs[2][0] + rs[3][0]);
    const float X = (rs[0][1] + rs[1][1]) + (rs[2][1] + rs[3][1]);
    const float Y = (rs[0][2] + rs[1][2]) + (rs[2][2] + rs[3][2]);
    const float cx = (X / S + 0.5f) / (float)W;
    const float cy = (Y / S + 0.5f) / (float)H;
    float sc = 1.f / S;   // max prob = exp(0)/sum
    if (boxes) {
      const float* bx = boxes + (int64_t)b * 4;
      const float area = (bx[2] - bx[0]) * (bx[3] - bx[1]);
      float w = sqrtf(area) / 96.f;
      w = w < 0.5f ? 0.5f : (w > 2.f ? 2.f : w);
      sc = sc * w;
    }
    coords[(int64_t)bk * 2] = cx;
    coords[(int64_t)bk * 2 + 1] = cy;
    scores[bk] = sc;
    if (argmax) argmax[bk] = mi;
  }
}

}  // namespace

extern "C" int64_t prpe_nms_workspace_bytes(int32_t, int32_t, int32_t, int32_t) { return 0; }

extern "C" int prpe_nms(const float* pred, int32_t B, int32_t N, int32_t nc, int32_t layout, float conf, float iou,
                        int32_t max_nms, int32_t max_det, float* out, int32_t* count, void* workspace,
                        int64_t workspace_bytes, void* stream) {
  (void)workspace; (void)workspace_bytes;
  if (!pred || !out || !count || B <= 0 || N <= 0 || nc <= 0) return PRPE_EINVAL;
  if (max_det <= 0 || max_det > NMS_MAX_DET || max_nms <= 0) return PRPE_EINVAL;
  if ((int64_t)N * nc >= (1LL << 31)) return PRPE_EINVAL;
  NmsK p{};
  p.pred = pred; p.B = B; p.N = N; p.nc = nc;
  if (layout == 0) { p.s_img = (int64_t)(4 + nc) * N; p.s_c = N; p.s_a = 1; }
  else if (layout == 1) { p.s_img = (int64_t)(4 + nc) * N; p.s_c = 1; p.s_a = 4 + nc; }
  else return PRPE_EINVAL;
  p.conf = conf; p.iou = iou; p.max_nms = max_nms; p.max_det = max_det; p.out = out; p.count = count;
  hipLaunchKernelGGL(nms_kernel, dim3(B), dim3(NMS_THREADS), 0, as_stream(stream), p);
  return launch_status();
}

extern "C" int prpe_softargmax(const float* heat, int32_t B, int32_t K, int32_t H, int32_t W, const float* boxes,
                               float* coords, float* scores, int32_t* argmax, void* stream) {
  if (!heat || !coords || !scores || B <= 0 || K <= 0 || H <= 0 || W <= 0) return PRPE_EINVAL;
  hipLaunchKernelGGL(softargmax_kernel, dim3(B * K), dim3(256), 0, as_stream(stream), heat, K, H, W, boxes, coords,
                     scores, argmax);
  return launch_status();
}

extern "C" int prpe_abi_version(void) { return PRPE_ABI_VERSION; }
extern "C" const char* prpe_build_info(void) { return "prpe gfx950 (CDNA4) split-bf16x3 MFMA; " __DATE__; }
