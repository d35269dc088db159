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
// More candidate pairs than the LDS key array holds (N*nc > 16384, e.g. a raw 80-class
// output) take the global path: keys into the caller's workspace, one rocPRIM device radix
// sort per image, then the same greedy pass.
// IoU in fp32 exactly as torchvision's CPU kernel (boxes offset by 7680*cls first,
// area = (x2-x1)*(y2-y1), inter / (area_i + area_j - inter) > thr). FP contraction is off
// in this file so every product/sum rounds like the reference.
//
// prpe_softargmax — PoseEstimationModule._get_keypoints_from_heatmaps
// (training/lightning/pose_estimation/module.py:237-296), one 256-thread workgroup per
// (frame, keypoint): max, sum exp, expectation of x and y, max prob, optional box scale.
#pragma clang fp contract(off)
#include "common.h"
#include <cstring>
#include <rocprim/rocprim.hpp>

namespace {

constexpr int NMS_THREADS = 1024;
constexpr int NMS_MAX_CAND = 16384;   // LDS key capacity (128 KiB): N*nc above it takes the global path
constexpr int NMS_MAX_DET = 1024;
constexpr int NMS_CHUNK = 256;        // candidates decoded per greedy round

__device__ __forceinline__ uint32_t orderable(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

struct NmsK {
  const float* pred; int B, N, nc; int64_t s_img, s_c, s_a;
  float conf, iou; int max_nms, max_det;
  float* out; int* count;
  unsigned long long* gkeys;          // global path: [B][N*nc] keys (unused tail = ~0: sorts last)
  const unsigned long long* gsorted;  // global path: [B][N*nc] sorted keys
  int* gtotal;                        // global path: [B] candidate count per image
};

__device__ __forceinline__ float pred_at(const NmsK& p, int b, int c, int a) {
  return p.pred[(int64_t)b * p.s_img + (int64_t)c * p.s_c + (int64_t)a * p.s_a];
}

// block-wide exclusive prefix sum of v (every thread calls); *total = the block's sum
__device__ __forceinline__ int block_scan_excl(int v, int* wsum, int& total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int off = 0, tot = 0;
  for (int w = 0; w < NMS_THREADS / 64; ++w) {
    if (w < wave) off += wsum[w];
    tot += wsum[w];
  }
  __syncthreads();
  total = tot;
  return off + incl - v;
}

// 1. candidates in the reference's enumeration order (box a ascending, class j ascending:
// util.py:137-152 filters boxes by max class score, then nc == 1 takes the best class, nc > 1
// every (a, j) with score > conf, in nonzero()'s row-major order). One thread per box: the box
// maximum is read once; the box's passing classes land at consecutive positions after a block
// prefix sum. key = ~orderable(score) << 32 | e (e = a*nc + j): ascending key order == the
// stable descending score sort. Keys past ``cap`` are dropped (counted in the total).
__device__ int nms_enumerate(const NmsK& p, int b, unsigned long long* keys, int cap, int* wsum) {
  const int tid = threadIdx.x;
  int running = 0;
  for (int base = 0; base < p.N; base += NMS_THREADS) {
    const int a = base + tid;
    int cnt = 0;
    float mx = -INFINITY;
    bool xc = false;
    if (a < p.N) {
      bool nan = false;
      for (int c = 0; c < p.nc; ++c) {
        const float v = pred_at(p, b, 4 + c, a);
        nan |= (v != v);
        mx = fmaxf(mx, v);
      }
      xc = !nan && mx > p.conf;     // xc (torch amax: NaN propagates, NaN > conf is false)
      if (xc) {
        if (p.nc == 1) cnt = 1;     // conf = max over the one class = mx > conf
        else
          for (int c = 0; c < p.nc; ++c) cnt += pred_at(p, b, 4 + c, a) > p.conf;
      }
    }
    int tot;
    const int off = running + block_scan_excl(cnt, wsum, tot);
    if (cnt) {
      int pos = off;
      for (int j = 0; j < p.nc && pos - off < cnt; ++j) {
        const float sc = p.nc == 1 ? mx : pred_at(p, b, 4 + j, a);
        if (p.nc > 1 && !(sc > p.conf)) continue;
        if (pos < cap)
          keys[pos] = ((unsigned long long)(~orderable(sc)) << 32) | (unsigned long long)(uint32_t)(a * p.nc + j);
        ++pos;
      }
    }
    running += tot;
  }
  return running;
}

struct NmsLds {
  float kept[NMS_MAX_DET][5];        // offset box x1,y1,x2,y2 + area of the kept boxes
  float cand[NMS_CHUNK][8];          // decoded chunk: ox1,oy1,ox2,oy2,area,score,cls,(x1 via off)
  int wsum[NMS_THREADS / 64];
  int nk;
};

// 3. greedy suppression (torchvision.ops.nms, util.py:162) over keys[0 .. ncand): the block
// decodes NMS_CHUNK candidates into LDS, then wave 0 tests them in order against the kept
// list (each lane a slice of it, __ballot decides) until max_det are kept. Writes out/count.
__device__ void nms_greedy(const NmsK& p, int b, const unsigned long long* keys, int ncand, NmsLds& L,
                           bool overflow) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* outb = p.out + (int64_t)b * p.max_det * 6;
  if (tid == 0) L.nk = 0;
  __syncthreads();
  for (int c0 = 0; c0 < ncand; c0 += NMS_CHUNK) {
    if (L.nk >= p.max_det) break;                    // block-uniform (read after a barrier)
    const int n = ncand - c0 < NMS_CHUNK ? ncand - c0 : NMS_CHUNK;
    if (tid < n) {
      const unsigned long long key = keys[c0 + tid];
      const int e = (int)(uint32_t)(key & 0xffffffffull);
      const int a = e / p.nc, j = e % p.nc;
      const float cx = pred_at(p, b, 0, a), cy = pred_at(p, b, 1, a);
      const float w = pred_at(p, b, 2, a), h = pred_at(p, b, 3, a);
      // wh2xy (util.py:76-82) then the class offset (util.py:160-161), in that order
      const float x1 = cx - w / 2.f, y1 = cy - h / 2.f, x2 = cx + w / 2.f, y2 = cy + h / 2.f;
      const float cls = (float)j;
      const float off = cls * 7680.f;
      const float ox1 = x1 + off, oy1 = y1 + off, ox2 = x2 + off, oy2 = y2 + off;
      float* q = L.cand[tid];
      q[0] = ox1; q[1] = oy1; q[2] = ox2; q[3] = oy2; q[4] = (ox2 - ox1) * (oy2 - oy1);
      q[5] = p.nc == 1 ? pred_at(p, b, 4, a) : pred_at(p, b, 4 + j, a);
      q[6] = cls;
      q[7] = __int_as_float(a);
    }
    __syncthreads();
    if (wave == 0) {
      int nk = L.nk;
      for (int i = 0; i < n && nk < p.max_det; ++i) {
        const float* q = L.cand[i];
        const float ox1 = q[0], oy1 = q[1], ox2 = q[2], oy2 = q[3], area = q[4];
        bool sup = false;
        for (int t = lane; t < nk; t += 64) {
          const float xx1 = fmaxf(L.kept[t][0], ox1), yy1 = fmaxf(L.kept[t][1], oy1);
          const float xx2 = fminf(L.kept[t][2], ox2), yy2 = fminf(L.kept[t][3], oy2);
          const float iw = fmaxf(0.f, xx2 - xx1), ih = fmaxf(0.f, yy2 - yy1);
          const float inter = iw * ih;
          const float ovr = inter / (L.kept[t][4] + area - inter);
          sup |= ovr > p.iou;
        }
        if (__ballot(sup) == 0ull) {
          if (lane == 0) {
            L.kept[nk][0] = ox1; L.kept[nk][1] = oy1; L.kept[nk][2] = ox2; L.kept[nk][3] = oy2;
            L.kept[nk][4] = area;
            // the reference returns x[keep]: the un-offset xyxy box, conf, class
            const int a = __float_as_int(q[7]);
            const float cx = pred_at(p, b, 0, a), cy = pred_at(p, b, 1, a);
            const float w = pred_at(p, b, 2, a), h = pred_at(p, b, 3, a);
            float* o = outb + (int64_t)nk * 6;
            o[0] = cx - w / 2.f; o[1] = cy - h / 2.f; o[2] = cx + w / 2.f; o[3] = cy + h / 2.f;
            o[4] = q[5]; o[5] = q[6];
          }
          ++nk;
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
        }
      }
      if (lane == 0) L.nk = nk;
    }
    __syncthreads();
  }
  const int nk = L.nk;
  for (int i = nk * 6 + tid; i < p.max_det * 6; i += NMS_THREADS) outb[i] = 0.f;
  // -1 flags a candidate overflow of the LDS path (cannot happen through prpe_nms, which
  // routes N*nc > NMS_MAX_CAND to the global path)
  if (tid == 0) p.count[b] = overflow ? -1 : nk;
}

// LDS path (N*nc <= NMS_MAX_CAND): enumerate, bitonic-sort in LDS, greedy; one block per image
__global__ __launch_bounds__(NMS_THREADS) void nms_kernel(NmsK p) {
  __shared__ unsigned long long keys[NMS_MAX_CAND];
  __shared__ NmsLds L;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int s_total = nms_enumerate(p, b, keys, NMS_MAX_CAND, L.wsum);
  const int total = s_total < NMS_MAX_CAND ? s_total : NMS_MAX_CAND;
  // 2. bitonic sort of keys[0..P) ascending, P = next pow2
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
  nms_greedy(p, b, keys, total < p.max_nms ? total : p.max_nms, L, s_total > NMS_MAX_CAND);
}

// global path, step 1: enumerate into the workspace, pad the image's key range with ~0
// (sorts after every real key), record the count
__global__ __launch_bounds__(NMS_THREADS) void nms_enum_global_kernel(NmsK p) {
  __shared__ int wsum[NMS_THREADS / 64];
  const int b = blockIdx.x;
  const int npairs = p.N * p.nc;
  unsigned long long* keys = p.gkeys + (int64_t)b * npairs;
  const int total = nms_enumerate(p, b, keys, npairs, wsum);
  for (int i = total + (int)threadIdx.x; i < npairs; i += NMS_THREADS) keys[i] = ~0ull;
  if (threadIdx.x == 0) p.gtotal[b] = total;
}

// global path, step 3: greedy over the image's sorted keys (the first min(total, max_nms))
__global__ __launch_bounds__(NMS_THREADS) void nms_greedy_global_kernel(NmsK p) {
  __shared__ NmsLds L;
  const int b = blockIdx.x;
  const int npairs = p.N * p.nc;
  const int total = p.gtotal[b];
  nms_greedy(p, b, p.gsorted + (int64_t)b * npairs, total < p.max_nms ? total : p.max_nms, L, false);
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

// global path workspace (8-B aligned pieces): keys [B][N*nc] (enumerated), sorted keys
// [B][N*nc], counts [B] (padded to 256 B), and the temporary storage of one rocPRIM device
// radix sort over N*nc keys (one sort per image: the images' ranges are sorted in turn)
static int64_t nms_sort_temp_bytes(int64_t npairs) {
  size_t bytes = 0;
  if (rocprim::radix_sort_keys((void*)nullptr, bytes, (const unsigned long long*)nullptr,
                               (unsigned long long*)nullptr, (size_t)npairs, 0, 64) != hipSuccess)
    return -1;
  return (int64_t)((bytes + 255) / 256 * 256);
}

extern "C" int64_t prpe_nms_workspace_bytes(int32_t B, int32_t N, int32_t nc, int32_t) {
  if (B <= 0 || N <= 0 || nc <= 0) return 0;
  const int64_t npairs = (int64_t)N * nc;
  if (npairs <= NMS_MAX_CAND) return 0;                 // LDS path
  const int64_t t = nms_sort_temp_bytes(npairs);
  if (t < 0) return -1;
  return 2 * 8 * B * npairs + (int64_t)((4 * B + 255) / 256 * 256) + t;
}

extern "C" int prpe_nms(const float* pred, int32_t B, int32_t N, int32_t nc, int32_t layout, float conf, float iou,
                        int32_t max_nms, int32_t max_det, float* out, int32_t* count, void* workspace,
                        int64_t workspace_bytes, void* stream) {
  if (!pred || !out || !count || B <= 0 || N <= 0 || nc <= 0) return PRPE_EINVAL;
  if (max_det <= 0 || max_det > NMS_MAX_DET || max_nms <= 0) return PRPE_EINVAL;
  const int64_t npairs = (int64_t)N * nc;
  if (npairs >= (1LL << 31)) return PRPE_EINVAL;
  NmsK p{};
  p.pred = pred; p.B = B; p.N = N; p.nc = nc;
  if (layout == 0) { p.s_img = (int64_t)(4 + nc) * N; p.s_c = N; p.s_a = 1; }
  else if (layout == 1) { p.s_img = (int64_t)(4 + nc) * N; p.s_c = 1; p.s_a = 4 + nc; }
  else return PRPE_EINVAL;
  p.conf = conf; p.iou = iou; p.max_nms = max_nms; p.max_det = max_det; p.out = out; p.count = count;
  hipStream_t st = as_stream(stream);
  if (npairs <= NMS_MAX_CAND) {
    hipLaunchKernelGGL(nms_kernel, dim3(B), dim3(NMS_THREADS), 0, st, p);
    return launch_status();
  }
  // global path: more candidate pairs than the LDS holds (e.g. a raw 80-class YOLO output,
  // A = 8400 x nc = 80 at conf 0.001; the reference sorts any count, util.py:157)
  const int64_t need = prpe_nms_workspace_bytes(B, N, nc, max_nms);
  if (need <= 0 || !workspace || workspace_bytes < need || (uintptr_t)workspace % 256) return PRPE_EINVAL;
  unsigned char* w = static_cast<unsigned char*>(workspace);
  p.gkeys = reinterpret_cast<unsigned long long*>(w);
  unsigned long long* sorted = p.gkeys + B * npairs;
  p.gsorted = sorted;
  p.gtotal = reinterpret_cast<int*>(sorted + B * npairs);
  const int64_t head = 2 * 8 * B * npairs + (4 * B + 255) / 256 * 256;
  void* temp = w + head;
  hipLaunchKernelGGL(nms_enum_global_kernel, dim3(B), dim3(NMS_THREADS), 0, st, p);
  int rc = launch_status();
  if (rc) return rc;
  for (int b = 0; b < B; ++b) {
    size_t tb = (size_t)(need - head);
    const hipError_t e = rocprim::radix_sort_keys(temp, tb, (const unsigned long long*)(p.gkeys + b * npairs),
                                                  sorted + b * npairs, (size_t)npairs, 0, 64, st);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(nms_greedy_global_kernel, dim3(B), dim3(NMS_THREADS), 0, st, p);
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
// prpe_build_info / prpe_source_hash: generated by build.py (build/build_info.c)
