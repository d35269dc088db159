// Detection eval metrics on device: the face/person detection
// validation step's DetectionMetrics (training/lightning/face_detection/module_v2.py:13-127,
// driven by validation_step :458-499). The reference loops over every NMS prediction in
// Python with two .item() syncs each; here one launch matches a whole batch and appends the
// (score, best IoU) records to a device list, and the epoch-end compute() is a stable
// descending sort + ten masked scans + trapezoid sums.
//
// update (per image i of the batch, only if it has >= 1 prediction and >= 1 ground-truth box,
// as validation_step skips the others):
//   iou[j, g] = inter / (area_j + area_g - inter + 1e-6)            (DetectionMetrics.box_iou)
//   best_j = max_g iou[j, g];  tp += (best_j > 0.5);  fp += !(best_j > 0.5);  gt += G_i
//   records += (score_j, best_j) in image order, then prediction order
// compute: precision = tp / (tp + fp + 1e-6), recall = tp / (gt + 1e-6),
//   f1 = 2 p r / (p + r + 1e-6) (all in double, like the reference's Python ints / floats);
//   for each threshold t of linspace(0.5, 0.95, 10): the records with iou >= t, in stable
//   descending score order, give cumulative tp (iou > 0.5) / fp counts c_k, f_k;
//   recall_k = c_k / (gt + 1e-6), precision_k = c_k / (c_k + f_k + 1e-6) (fp32, as torch),
//   AP_t = trapz([1, p.., 0], [0, r.., 1]); mAP50 = AP_0.5, mAP75 = AP_0.75, mAP = mean.
// IoUs use the reference's fp32 operation order with contraction off (bit-exact values).
#include "common.h"
#include <cstring>
#include <rocprim/rocprim.hpp>

#pragma clang fp contract(off)

namespace {

constexpr int NT = 10;                 // IoU thresholds
constexpr int SCAN_BLOCK = 256, SCAN_ITEMS = 8, SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

struct MatchK {
  const float* dets; const int32_t* counts; int B, max_det;
  const float* gt; const int64_t* gt_batch; int G;
  const int32_t* gt_count;             // per image (workspace)
  unsigned long long* counters;        // [4]: tp, fp, gt, records
  float* records; int64_t cap;
};

__global__ void gt_count_kernel(const int64_t* gt_batch, int G, int B, int32_t* gt_count) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < G) {
    const int64_t b = gt_batch[g];
    if (b >= 0 && b < B) atomicAdd(&gt_count[b], 1);
  }
}

__device__ __forceinline__ float box_iou(const float* a, const float* g) {
  const float area1 = (a[2] - a[0]) * (a[3] - a[1]);
  const float area2 = (g[2] - g[0]) * (g[3] - g[1]);
  const float ltx = fmaxf(a[0], g[0]), lty = fmaxf(a[1], g[1]);
  const float rbx = fminf(a[2], g[2]), rby = fminf(a[3], g[3]);
  const float w = fmaxf(rbx - ltx, 0.f), h = fmaxf(rby - lty, 0.f);
  const float inter = w * h;
  const float uni = area1 + area2 - inter;
  return inter / (uni + 1e-6f);
}

// one block per image; threads over its predictions
__global__ __launch_bounds__(320) void match_kernel(MatchK p) {
  const int i = blockIdx.x;
  const int n = p.counts[i] < p.max_det ? p.counts[i] : p.max_det;
  const int gi = p.gt_count[i];
  if (n <= 0 || gi <= 0) return;                     // validation_step's two `continue`s
  __shared__ unsigned long long base_s;
  __shared__ int tp_s;
  if (threadIdx.x == 0) {
    unsigned long long b = p.counters[3];
    for (int k = 0; k < i; ++k) {
      const int nk = p.counts[k] < p.max_det ? p.counts[k] : p.max_det;
      if (nk > 0 && p.gt_count[k] > 0) b += nk;
    }
    base_s = b;
    tp_s = 0;
  }
  __syncthreads();
  int tp = 0;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const float* d = p.dets + ((int64_t)i * p.max_det + j) * 6;
    // ious.max(dim=1): the row maximum, NaN if any entry is NaN
    float best = 0.f;
    bool first = true;
    for (int g = 0; g < p.G; ++g) {
      if (p.gt_batch[g] != i) continue;
      const float v = box_iou(d, p.gt + (int64_t)g * 4);
      if (first) best = v;
      else if (best == best && (v != v || v > best)) best = v;
      first = false;
    }
    const bool is_tp = best > 0.5f;
    tp += is_tp ? 1 : 0;
    const unsigned long long idx = base_s + j;
    if (idx < (unsigned long long)p.cap) {
      p.records[idx * 2] = d[4];
      p.records[idx * 2 + 1] = best;
    }
  }
  atomicAdd(&tp_s, tp);
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&p.counters[0], (unsigned long long)tp_s);
    atomicAdd(&p.counters[1], (unsigned long long)(n - tp_s));
    atomicAdd(&p.counters[2], (unsigned long long)gi);
  }
}

// records += sum over used images (after match_kernel read the old count)
__global__ void finalize_kernel(const int32_t* counts, const int32_t* gt_count, int B, int max_det,
                                unsigned long long* counters) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  unsigned long long add = 0;
  for (int k = 0; k < B; ++k) {
    const int nk = counts[k] < max_det ? counts[k] : max_det;
    if (nk > 0 && gt_count[k] > 0) add += nk;
  }
  counters[3] += add;
}

struct ApK {
  const float* iou;                    // sorted by score, descending, stable
  int64_t n;
  float thr[NT];
  const unsigned long long* counters;  // gt = counters[2]
  int* tile_counts;                    // [tiles][2*NT]: kept tp / fp per threshold
  double* tile_area;                   // [tiles][NT]
};

// torch: tp_cumsum / (self.total_gt + 1e-6) -- the Python-float scalar is cast to fp32
__device__ __forceinline__ float gt_den(const unsigned long long* counters) {
  return (float)((double)counters[2] + 1e-6);
}

// per tile: kept tp / fp counts per threshold
__global__ __launch_bounds__(SCAN_BLOCK) void ap_count_kernel(ApK p) {
  __shared__ int cnt[2 * NT];
  if (threadIdx.x < 2 * NT) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int c[2 * NT] = {};
  for (int e = 0; e < SCAN_ITEMS; ++e) {
    const int64_t k = base + e;
    if (k >= p.n) break;
    const float v = p.iou[k];
    const int tp = v > 0.5f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (v >= p.thr[t]) c[2 * t + (tp ? 0 : 1)] += 1;
  }
#pragma unroll
  for (int q = 0; q < 2 * NT; ++q)
    if (c[q]) atomicAdd(&cnt[q], c[q]);
  __syncthreads();
  if (threadIdx.x < 2 * NT) p.tile_counts[(int64_t)blockIdx.x * 2 * NT + threadIdx.x] = cnt[threadIdx.x];
}

// exclusive scan of the tile counts (single thread; tiles = n / 2048)
__global__ void ap_scan_tiles_kernel(int* tile_counts, int tiles, int* totals) {
  if (threadIdx.x >= 2 * NT || blockIdx.x != 0) return;
  const int q = threadIdx.x;
  int run = 0;
  for (int b = 0; b < tiles; ++b) {
    const int v = tile_counts[(int64_t)b * 2 * NT + q];
    tile_counts[(int64_t)b * 2 * NT + q] = run;
    run += v;
  }
  totals[q] = run;
}

__device__ __forceinline__ void pr_point(int c, int f, float gt_den, float& r, float& pr) {
  // torch: recalls = tp_cumsum / (total_gt + 1e-6); precisions = tp_cumsum / (tp_cumsum +
  // fp_cumsum + 1e-6), int64 tensors promoted to fp32
  r = (float)c / gt_den;
  pr = (float)c / ((float)(c + f) + 1e-6f);
}

// per tile: trapezoid contributions of the kept records (previous point from the running
// counts; the prepended (0, 1) point for the first kept record)
__global__ __launch_bounds__(SCAN_BLOCK) void ap_area_kernel(ApK p) {
  __shared__ int pre[SCAN_BLOCK][2 * NT + 1];        // per-thread inclusive counts (+1 pad)
  __shared__ double area[NT];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int c[2 * NT] = {};
  for (int e = 0; e < SCAN_ITEMS; ++e) {
    const int64_t k = base + e;
    if (k >= p.n) break;
    const float v = p.iou[k];
    const int tp = v > 0.5f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (v >= p.thr[t]) c[2 * t + (tp ? 0 : 1)] += 1;
  }
#pragma unroll
  for (int q = 0; q < 2 * NT; ++q) pre[threadIdx.x][q] = c[q];
  if (threadIdx.x < NT) area[threadIdx.x] = 0.0;
  __syncthreads();
  // exclusive prefix of the threads before this one (serial over <= 255 entries per counter)
  int run[2 * NT];
#pragma unroll
  for (int q = 0; q < 2 * NT; ++q) run[q] = p.tile_counts[(int64_t)blockIdx.x * 2 * NT + q];
  for (int u = 0; u < (int)threadIdx.x; ++u)
#pragma unroll
    for (int q = 0; q < 2 * NT; ++q) run[q] += pre[u][q];
  double a[NT] = {};
  const float den = gt_den(p.counters);
  for (int e = 0; e < SCAN_ITEMS; ++e) {
    const int64_t k = base + e;
    if (k >= p.n) break;
    const float v = p.iou[k];
    const int tp = v > 0.5f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (!(v >= p.thr[t])) continue;
      const int c0 = run[2 * t], f0 = run[2 * t + 1];
      float r0 = 0.f, p0 = 1.f;
      if (c0 + f0 > 0) pr_point(c0, f0, den, r0, p0);
      run[2 * t + (tp ? 0 : 1)] += 1;
      float r1, p1;
      pr_point(run[2 * t], run[2 * t + 1], den, r1, p1);
      a[t] += (double)((r1 - r0) * (p1 + p0) / 2.f);
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
    if (a[t] != 0.0) atomicAdd(&area[t], a[t]);
  __syncthreads();
  if (threadIdx.x < NT) p.tile_area[(int64_t)blockIdx.x * NT + threadIdx.x] = area[threadIdx.x];
}

// out: precision, recall, f1, mAP50, mAP75, mAP (double)
__global__ void ap_final_kernel(const unsigned long long* counters, const int* totals, const double* tile_area,
                                int tiles, double* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double tp = (double)counters[0], fp = (double)counters[1], gt = (double)counters[2];
  const double prec = tp / (tp + fp + 1e-6), rec = tp / (gt + 1e-6);
  const double f1 = 2 * (prec * rec) / (prec + rec + 1e-6);
  double ap[NT];
  for (int t = 0; t < NT; ++t) {
    const int c = totals[2 * t], f = totals[2 * t + 1];
    if (c + f == 0) { ap[t] = 0.0; continue; }
    double s = 0.0;
    for (int b = 0; b < tiles; ++b) s += tile_area[(int64_t)b * NT + t];
    float r, pr;
    pr_point(c, f, gt_den(counters), r, pr);
    s += (double)((1.f - r) * (0.f + pr) / 2.f);     // to the appended (1, 0) point
    ap[t] = (double)(float)s;                        // torch.trapz returns fp32
  }
  double m = 0.0;
  for (int t = 0; t < NT; ++t) m += ap[t];
  out[0] = prec; out[1] = rec; out[2] = f1; out[3] = ap[0]; out[4] = ap[5]; out[5] = m / NT;
}

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

size_t sort_temp_bytes(int64_t n) {
  size_t bytes = 0;
  rocprim::radix_sort_pairs_desc((void*)nullptr, bytes, (const float*)nullptr, (float*)nullptr,
                                 (const float*)nullptr, (float*)nullptr, (size_t)n);
  return bytes;
}

}  // namespace

extern "C" int64_t prpe_det_metrics_update_workspace_bytes(int32_t B) {
  return B > 0 ? (int64_t)align256((size_t)B * sizeof(int32_t)) : 0;
}

extern "C" int prpe_det_metrics_update(const float* dets, const int32_t* counts, int32_t B, int32_t max_det,
                                       const float* gt_boxes, const int64_t* gt_batch, int32_t G,
                                       uint64_t* counters, float* records, int64_t capacity, void* workspace,
                                       int64_t workspace_bytes, void* stream) {
  if (!dets || !counts || B <= 0 || max_det <= 0 || max_det > 1024 || G < 0 || (G > 0 && (!gt_boxes || !gt_batch)) ||
      !counters || !records || capacity <= 0 || !workspace || workspace_bytes < prpe_det_metrics_update_workspace_bytes(B))
    return PRPE_EINVAL;
  hipStream_t st = as_stream(stream);
  int32_t* gt_count = static_cast<int32_t*>(workspace);
  if (hipMemsetAsync(gt_count, 0, (size_t)B * sizeof(int32_t), st) != hipSuccess) return launch_status();
  if (G > 0) hipLaunchKernelGGL(gt_count_kernel, dim3((G + 255) / 256), dim3(256), 0, st, gt_batch, G, B, gt_count);
  MatchK p{dets, counts, B, max_det, gt_boxes, gt_batch, G, gt_count,
           reinterpret_cast<unsigned long long*>(counters), records, capacity};
  hipLaunchKernelGGL(match_kernel, dim3(B), dim3(320), 0, st, p);
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, st, counts, (const int32_t*)gt_count, B, max_det,
                     reinterpret_cast<unsigned long long*>(counters));
  return launch_status();
}

extern "C" int64_t prpe_det_metrics_compute_workspace_bytes(int64_t n) {
  if (n < 0) return 0;
  const int64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE + 1;
  return (int64_t)(align256((size_t)(n > 0 ? n : 1) * 4) * 4 + align256(sort_temp_bytes(n > 0 ? n : 1)) +
                   align256((size_t)tiles * 2 * NT * 4) + align256((size_t)tiles * NT * 8) + align256(2 * NT * 4));
}

extern "C" int prpe_det_metrics_compute(const uint64_t* counters, const float* records, int64_t n,
                                        const float* thresholds, double* out, void* workspace,
                                        int64_t workspace_bytes, void* stream) {
  if (!counters || !out || !thresholds || n < 0 || (n > 0 && !records) || !workspace ||
      workspace_bytes < prpe_det_metrics_compute_workspace_bytes(n) || n >= (1LL << 31))
    return PRPE_EINVAL;
  hipStream_t st = as_stream(stream);
  const size_t nb = align256((size_t)(n > 0 ? n : 1) * 4);
  char* w = static_cast<char*>(workspace);
  float* keys_in = reinterpret_cast<float*>(w); w += nb;
  float* vals_in = reinterpret_cast<float*>(w); w += nb;
  float* keys_out = reinterpret_cast<float*>(w); w += nb;
  float* vals_out = reinterpret_cast<float*>(w); w += nb;
  size_t tb = sort_temp_bytes(n > 0 ? n : 1);
  void* temp = w; w += align256(tb);
  const int tiles = (int)((n + SCAN_TILE - 1) / SCAN_TILE);
  int* tile_counts = reinterpret_cast<int*>(w); w += align256((size_t)(tiles + 1) * 2 * NT * 4);
  double* tile_area = reinterpret_cast<double*>(w); w += align256((size_t)(tiles + 1) * NT * 8);
  int* totals = reinterpret_cast<int*>(w);
  if (hipMemsetAsync(totals, 0, 2 * NT * 4, st) != hipSuccess) return launch_status();
  if (n > 0) {
    // split the interleaved (score, iou) records, then a stable descending sort by score
    // (Python's sorted(..., reverse=True) keeps equal scores in insertion order; so does LSD radix)
    if (hipMemcpy2DAsync(keys_in, 4, records, 8, 4, (size_t)n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpy2DAsync(vals_in, 4, records + 1, 8, 4, (size_t)n, hipMemcpyDeviceToDevice, st) != hipSuccess)
      return launch_status();
    if (rocprim::radix_sort_pairs_desc(temp, tb, keys_in, keys_out, vals_in, vals_out, (size_t)n, 0, 32, st) !=
        hipSuccess)
      return launch_status();
    ApK p{};
    p.iou = vals_out; p.n = n;
    for (int t = 0; t < NT; ++t) p.thr[t] = thresholds[t];
    p.counters = reinterpret_cast<const unsigned long long*>(counters);
    p.tile_counts = tile_counts; p.tile_area = tile_area;
    hipLaunchKernelGGL(ap_count_kernel, dim3(tiles), dim3(SCAN_BLOCK), 0, st, p);
    hipLaunchKernelGGL(ap_scan_tiles_kernel, dim3(1), dim3(64), 0, st, tile_counts, tiles, totals);
    hipLaunchKernelGGL(ap_area_kernel, dim3(tiles), dim3(SCAN_BLOCK), 0, st, p);
  }
  hipLaunchKernelGGL(ap_final_kernel, dim3(1), dim3(64), 0, st, reinterpret_cast<const unsigned long long*>(counters),
                     (const int*)totals, (const double*)tile_area, tiles, out);
  return launch_status();
}

// ------------------------------------------------------------------ detection eval loss
// FaceDetectionModule.compute_loss (module_v2.py:178-303) on the eval-mode head output, as
// validation_step calls it (:467): boxes [B, 4, N] (taken as x1y1x2y2 by compute_iou, as the
// reference does), scores [B, C, N]; one block per image:
//   keep = max_c score > 0.01 (order kept); no ground truth in the image: skipped (loss 0);
//   no kept prediction or no box: bg loss on the kept ones if any;
//   else ious = compute_iou(kept, gt) (utils.py:8-76, eps 1e-7), best = max over gt (first
//   index on ties), pos = best > 0.5; with positives: box = -mean over the P x P matrix
//   compute_iou(kept[pos], gt[idx[pos]], CIoU=True) (the reference takes the mean of the full
//   pairwise matrix), cls = cross_entropy(scores[pos], gt_class[idx[pos]]), bg = mean BCE-
//   with-logits(max score of the non-positives, 0); loss_b = box + cls + 0.5 bg;
//   without positives: loss_b = bg over all kept. loss = sum_b loss_b / B.
namespace {

constexpr int LOSS_MAX_N = 1024;

__device__ __forceinline__ float bce0(float x) {
  // F.binary_cross_entropy_with_logits(x, 0): (1 - 0) x + max_val + log(exp(-max_val) + exp(-x - max_val))
  const float m = fmaxf(-x, 0.f);
  return x + m + logf(expf(-m) + expf(-x - m));
}

// compute_iou (utils.py:8-76) for one pair, fp32 in the reference's operation order
__device__ float ref_iou(const float* a, const float* b, bool ciou) {
  const float eps = 1e-7f;
  const float w1 = a[2] - a[0], h1 = a[3] - a[1], w2 = b[2] - b[0], h2 = b[3] - b[1];
  const float area1 = fmaxf(w1, 0.f) * fmaxf(h1, 0.f), area2 = fmaxf(w2, 0.f) * fmaxf(h2, 0.f);
  const float iw = fmaxf(fminf(a[2], b[2]) - fmaxf(a[0], b[0]), 0.f);
  const float ih = fmaxf(fminf(a[3], b[3]) - fmaxf(a[1], b[1]), 0.f);
  const float inter = iw * ih;
  const float uni = area1 + area2 - inter + eps;
  const float iou = inter / uni;
  if (!ciou) return iou;
  const float cw = fmaxf(a[2], b[2]) - fminf(a[0], b[0]);
  const float ch = fmaxf(a[3], b[3]) - fminf(a[1], b[1]);
  const float c2 = (cw * cw + ch * ch) + eps;
  const float dx = a[0] + a[2] - b[0] - b[2], dy = a[1] + a[3] - b[1] - b[3];
  const float rho2 = (dx * dx + dy * dy) / 4.f;
  const float d = atanf(w2 / (h2 + eps)) - atanf(w1 / (h1 + eps));
  const float v = (float)(4.0 / (M_PI * M_PI)) * (d * d);       // Python-float constant, cast to fp32
  const float alpha = v / (v - iou + (1.f + eps));
  return iou - (rho2 / c2 + v * alpha);
}

struct LossK {
  const float* boxes; int64_t bs_b, bs_c, bs_n;     // [B, 4, N] element strides
  const float* scores; int64_t ss_b, ss_c, ss_n;    // [B, C, N]
  int B, C, N;
  const float* gt; const int64_t* gt_batch; const int64_t* gt_cls; int G;
  float* per_image;                                 // [B][4]: loss_b, box, cls, bg (NaN = not computed)
};

__global__ __launch_bounds__(256) void det_loss_kernel(LossK p) {
  const int b = blockIdx.x;
  __shared__ int keep_idx[LOSS_MAX_N];
  __shared__ float best_s[LOSS_MAX_N];
  __shared__ int gidx_s[LOSS_MAX_N];
  __shared__ int nkeep, npos, ngt;
  __shared__ double red[4];
  const int tid = threadIdx.x;
  if (tid == 0) {
    // kept predictions in order, and the image's ground-truth count
    int k = 0;
    for (int j = 0; j < p.N; ++j) {
      float m = -INFINITY;
      for (int c = 0; c < p.C; ++c) m = fmaxf(m, p.scores[b * p.ss_b + c * p.ss_c + (int64_t)j * p.ss_n]);
      if (m > 0.01f) keep_idx[k++] = j;
    }
    nkeep = k;
    int g = 0;
    for (int q = 0; q < p.G; ++q) g += p.gt_batch[q] == b;
    ngt = g;
    npos = 0;
    for (int q = 0; q < 4; ++q) red[q] = 0.0;
  }
  __syncthreads();
  float* out = p.per_image + (int64_t)b * 4;
  if (ngt == 0) {                                   // "No targets in this batch, skipping"
    if (tid == 0) { out[0] = 0.f; out[1] = out[2] = out[3] = NAN; }
    return;
  }
  auto maxscore = [&](int j) {
    float m = -INFINITY;
    for (int c = 0; c < p.C; ++c) m = fmaxf(m, p.scores[b * p.ss_b + c * p.ss_c + (int64_t)j * p.ss_n]);
    return m;
  };
  auto box_of = [&](int j, float* o) {
    for (int c = 0; c < 4; ++c) o[c] = p.boxes[b * p.bs_b + c * p.bs_c + (int64_t)j * p.bs_n];
  };
  const int M = nkeep;
  // best IoU over the image's ground truth per kept prediction (first index on ties)
  for (int k = tid; k < M; k += blockDim.x) {
    float a[4];
    box_of(keep_idx[k], a);
    float best = 0.f;
    int bi = -1, gl = 0;
    for (int q = 0; q < p.G; ++q) {
      if (p.gt_batch[q] != b) continue;
      const float v = ref_iou(a, p.gt + (int64_t)q * 4, false);
      if (bi < 0 || v > best || (v != v && best == best)) { best = v; bi = q; }
      ++gl;
    }
    best_s[k] = best;
    gidx_s[k] = bi;
    if (best > 0.5f) atomicAdd(&npos, 1);
  }
  __syncthreads();
  const int P = npos;
  // positives in order (prefix by one thread: M <= LOSS_MAX_N)
  __shared__ int pos_idx[LOSS_MAX_N];
  __shared__ int neg_cnt;
  if (tid == 0) {
    int q = 0, r = 0;
    for (int k = 0; k < M; ++k) {
      if (best_s[k] > 0.5f) pos_idx[q++] = k;
      else ++r;
    }
    neg_cnt = r;
  }
  __syncthreads();
  if (M == 0) {
    if (tid == 0) { out[0] = 0.f; out[1] = out[2] = out[3] = NAN; }
    return;
  }
  double bg = 0.0, box = 0.0, cls = 0.0;
  if (P == 0) {
    for (int k = tid; k < M; k += blockDim.x) bg += (double)bce0(maxscore(keep_idx[k]));
  } else {
    for (int k = tid; k < M; k += blockDim.x)
      if (!(best_s[k] > 0.5f)) bg += (double)bce0(maxscore(keep_idx[k]));
    // box: mean of the P x P CIoU matrix between positives i and matched boxes of positives j
    for (int e = tid; e < P * P; e += blockDim.x) {
      const int i = e / P, jj = e % P;
      float a[4];
      box_of(keep_idx[pos_idx[i]], a);
      box += (double)ref_iou(a, p.gt + (int64_t)gidx_s[pos_idx[jj]] * 4, true);
    }
    // cross_entropy(scores[pos] [P, C], labels): logsumexp - score[label]
    for (int i = tid; i < P; i += blockDim.x) {
      const int j = keep_idx[pos_idx[i]];
      const int64_t lab = p.gt_cls ? p.gt_cls[gidx_s[pos_idx[i]]] : 0;
      float m = -INFINITY;
      for (int c = 0; c < p.C; ++c) m = fmaxf(m, p.scores[b * p.ss_b + c * p.ss_c + (int64_t)j * p.ss_n]);
      float s = 0.f;
      for (int c = 0; c < p.C; ++c) s += expf(p.scores[b * p.ss_b + c * p.ss_c + (int64_t)j * p.ss_n] - m);
      cls += (double)(m + logf(s) - p.scores[b * p.ss_b + lab * p.ss_c + (int64_t)j * p.ss_n]);
    }
  }
  atomicAdd(&red[0], bg);
  atomicAdd(&red[1], box);
  atomicAdd(&red[2], cls);
  __syncthreads();
  if (tid == 0) {
    if (P == 0) {
      const float bgm = (float)(red[0] / M);
      out[0] = bgm; out[1] = NAN; out[2] = NAN; out[3] = bgm;
    } else {
      const float boxm = -(float)(red[1] / ((double)P * P));
      const float clsm = (float)(red[2] / P);
      const float bgm = neg_cnt > 0 ? (float)(red[0] / neg_cnt) : NAN;   // mean of an empty tensor
      out[0] = boxm + clsm + 0.5f * bgm; out[1] = boxm; out[2] = clsm; out[3] = bgm;
    }
  }
}

__global__ void det_loss_mean_kernel(const float* per_image, int B, float* loss) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float t = 0.f;
  for (int b = 0; b < B; ++b) t += per_image[b * 4];
  loss[0] = t / (float)B;
}

}  // namespace

extern "C" int prpe_det_eval_loss(const float* boxes, const int64_t* box_strides, const float* scores,
                                  const int64_t* score_strides, int32_t B, int32_t C, int32_t N,
                                  const float* gt_boxes, const int64_t* gt_batch, const int64_t* gt_classes,
                                  int32_t G, float* per_image, float* loss, void* stream) {
  if (!boxes || !box_strides || !scores || !score_strides || B <= 0 || C <= 0 || N <= 0 || N > LOSS_MAX_N ||
      G < 0 || (G > 0 && (!gt_boxes || !gt_batch)) || !per_image || !loss)
    return PRPE_EINVAL;
  LossK p{};
  p.boxes = boxes; p.bs_b = box_strides[0]; p.bs_c = box_strides[1]; p.bs_n = box_strides[2];
  p.scores = scores; p.ss_b = score_strides[0]; p.ss_c = score_strides[1]; p.ss_n = score_strides[2];
  p.B = B; p.C = C; p.N = N; p.gt = gt_boxes; p.gt_batch = gt_batch; p.gt_cls = gt_classes; p.G = G;
  p.per_image = per_image;
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(det_loss_kernel, dim3(B), dim3(256), 0, st, p);
  hipLaunchKernelGGL(det_loss_mean_kernel, dim3(1), dim3(64), 0, st, (const float*)per_image, B, loss);
  return launch_status();
}
