// K10 / K12 — full-rank eval tail on the device.
//   * gmr_mask_scores_f32:  scores[mask] = -1e10          (reference common/trainer.py:383-384)
//   * gmr_topk_rows_f32:    per-row top-K, score desc, ties -> lowest index
//                           (torch.topk at common/trainer.py:386 and the graph-rebuild
//                           top-k at :546/556).  Exact radix select on order-preserving
//                           uint32 keys (4 passes of 8 bits, LDS histograms), then a
//                           deterministic collection and a bitonic sort of <= 64 winners.
//   * gmr_eval_metrics:     hit matrix + Recall/NDCG/Precision/MAP sums over users
//                           (utils/topk_evaluator.py:107-120, utils/metrics.py:12-105).
#include "gmr_common.h"

namespace {

__device__ __forceinline__ uint32_t fkey(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void mask_kernel(int64_t n, const int* __restrict__ rows, const int* __restrict__ cols, float* __restrict__ s,
                            int64_t ld, float fill) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) s[(int64_t)rows[i] * ld + cols[i]] = fill;
}

constexpr int TK_THREADS = 256;

// STAGED: the row's order-preserving keys are staged in LDS once (n_cols <= TK_STAGE_COLS), so the
// four radix passes and the collection read LDS instead of re-reading the row from HBM / L2.  The
// histogram adds are run-length aggregated per thread: scores are close together, so the early
// passes put nearly every key in one bin and per-element LDS atomics would serialise on it.
constexpr int TK_STAGE_COLS = 36864;  // 144 KB of the 160 KB LDS

template <bool STAGED>
__global__ void __launch_bounds__(TK_THREADS) topk_rows_kernel(int64_t n_rows, int64_t n_cols, const float* __restrict__ S,
                                                               int64_t ld, int K, int* __restrict__ out_idx,
                                                               int64_t ld_idx, float* __restrict__ out_val) {
  extern __shared__ uint32_t s_key[];
  __shared__ int hist[256];
  __shared__ uint32_t s_prefix;
  __shared__ int s_need;
  __shared__ int scan_gt[TK_THREADS];
  __shared__ int scan_eq[TK_THREADS];
  __shared__ unsigned long long cand[64];
  const int64_t row = blockIdx.x;
  if (row >= n_rows) return;
  const float* p = S + row * ld;
  const int t = threadIdx.x;
  auto key = [&](int64_t j) -> uint32_t { return STAGED ? s_key[j] : fkey(p[j]); };
  if (STAGED) {
    for (int64_t j = t; j < n_cols; j += TK_THREADS) s_key[j] = fkey(p[j]);
  }

  uint32_t prefix = 0, pmask = 0;
  int need = K;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    hist[t] = 0;
    __syncthreads();
    int run_bin = 0, run_cnt = 0;
    for (int64_t j = t; j < n_cols; j += TK_THREADS) {
      const uint32_t k = key(j);
      if ((k & pmask) == prefix) {
        const int b = (k >> shift) & 255;
        if (b != run_bin && run_cnt) {
          atomicAdd(&hist[run_bin], run_cnt);
          run_cnt = 0;
        }
        run_bin = b;
        ++run_cnt;
      }
    }
    if (run_cnt) atomicAdd(&hist[run_bin], run_cnt);
    __syncthreads();
    if (t == 0) {
      int acc = 0, b = 255;
      for (; b > 0; --b) {
        if (acc + hist[b] >= need) break;
        acc += hist[b];
      }
      s_prefix = prefix | ((uint32_t)b << shift);
      s_need = need - acc;
    }
    __syncthreads();
    prefix = s_prefix;
    need = s_need;
    pmask |= 0xFFu << shift;
    __syncthreads();
  }
  // prefix = key of the K-th largest element; need = how many elements equal to it to take
  const uint32_t T = prefix;
  const int64_t chunk = (n_cols + TK_THREADS - 1) / TK_THREADS;
  const int64_t c0 = t * chunk, c1 = min(n_cols, c0 + chunk);
  int n_gt = 0, n_eq = 0;
  for (int64_t j = c0; j < c1; ++j) {
    const uint32_t k = key(j);
    n_gt += k > T;
    n_eq += k == T;
  }
  // exclusive scans of n_gt and n_eq over threads (thread order == column order)
  scan_gt[t] = n_gt;
  scan_eq[t] = n_eq;
  __syncthreads();
  for (int off = 1; off < TK_THREADS; off <<= 1) {
    int a = t >= off ? scan_gt[t - off] : 0;
    int b = t >= off ? scan_eq[t - off] : 0;
    __syncthreads();
    scan_gt[t] += a;
    scan_eq[t] += b;
    __syncthreads();
  }
  const int total_gt = scan_gt[TK_THREADS - 1];
  int gt_slot = scan_gt[t] - n_gt;
  int eq_ord = scan_eq[t] - n_eq;
  if (t < 64) cand[t] = ~0ull;
  __syncthreads();
  for (int64_t j = c0; j < c1; ++j) {
    const uint32_t k = key(j);
    int slot = -1;
    if (k > T) slot = gt_slot++;
    else if (k == T) {
      if (eq_ord < need) slot = total_gt + eq_ord;
      ++eq_ord;
    }
    // sort key: larger score first, then lower index -> ascending on (~key, idx)
    if (slot >= 0) cand[slot] = ((unsigned long long)(~k) << 32) | (uint32_t)j;
  }
  __syncthreads();
  // bitonic sort of 64 candidates ascending (padding = ~0 sorts last)
  for (int size = 2; size <= 64; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (t < 32) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        unsigned long long a = cand[lo], b = cand[hi];
        if ((a > b) == up) {
          cand[lo] = b;
          cand[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  if (t < K) {
    const unsigned long long e = cand[t];
    const int j = (int)(uint32_t)(e & 0xFFFFFFFFull);
    out_idx[row * ld_idx + t] = j;
    if (out_val) out_val[row * ld_idx + t] = p[j];
  }
}

// k == 1: single pass arg-max per row, ties -> lowest index
__global__ void __launch_bounds__(256) argmax_rows_kernel(int64_t n_rows, int64_t n_cols, const float* __restrict__ S,
                                                          int64_t ld, int* __restrict__ out_idx, int64_t ld_idx,
                                                          float* __restrict__ out_val) {
  __shared__ unsigned long long red[4];
  const int64_t row = blockIdx.x;
  const float* p = S + row * ld;
  unsigned long long best = ~0ull;  // ascending order on (~key, idx): a total order, so any visiting order
                                    // (and any reduction tree) returns the same entry
  auto take = [&](float v, int64_t j) {
    const unsigned long long e = ((unsigned long long)(~fkey(v)) << 32) | (uint32_t)j;
    best = e < best ? e : best;
  };
  int64_t j0 = 0;
  if ((((uintptr_t)p) & 15) == 0) {  // 16-byte rows (round 6: 4 columns per load, 240 -> ~120 us on the 19,445 x
                                     // 7,050 rebuild rows)
    const int64_t n4 = n_cols / 4;
    const float4* p4 = reinterpret_cast<const float4*>(p);
    for (int64_t q = threadIdx.x; q < n4; q += 256) {
      const float4 v = p4[q];
      take(v.x, 4 * q);
      take(v.y, 4 * q + 1);
      take(v.z, 4 * q + 2);
      take(v.w, 4 * q + 3);
    }
    j0 = 4 * n4;
  }
  for (int64_t j = j0 + threadIdx.x; j < n_cols; j += 256) take(p[j], j);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    unsigned long long o = __shfl_xor(best, m);
    best = o < best ? o : best;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = red[0];
    for (int i = 1; i < 4; ++i) b = red[i] < b ? red[i] : b;
    const int j = (int)(uint32_t)(b & 0xFFFFFFFFull);
    out_idx[row * ld_idx] = j;
    if (out_val) out_val[row * ld_idx] = p[j];
  }
}

// One thread per user.  ks = {5, 10, 20, 50} (any ascending list <= K, up to 8).
// sums layout: [metric][k] with metric 0 recall, 1 ndcg, 2 precision, 3 map; per-block partials.
// sel (optional): the eval-user rows to sum over (a user group of the test-time extras)
__global__ void __launch_bounds__(256) metrics_kernel(int64_t n_users, const int* __restrict__ sel,
                                                      const int* __restrict__ topk, int64_t ld_topk,
                                                      int K, const int64_t* __restrict__ pos_ptr,
                                                      const int* __restrict__ pos_items, int n_ks, const int* __restrict__ ks,
                                                      double* __restrict__ part) {
  __shared__ double red[4][8][4];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t u = (i < n_users && sel) ? (int64_t)sel[i] : i;
  double m[4][8];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) m[a][b] = 0.0;
  if (i < n_users) {
    const int64_t beg = pos_ptr[u], end = pos_ptr[u + 1];
    const int plen = (int)(end - beg);
    double cum = 0.0, dcg = 0.0, idcg = 0.0, sum_pre = 0.0;
    int ki = 0;
    for (int r = 0; r < K && ki < n_ks; ++r) {
      const int item = topk[u * ld_topk + r];
      int64_t lo = beg, hi = end;
      while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (pos_items[mid] < item) lo = mid + 1;
        else hi = mid;
      }
      const bool hit = lo < end && pos_items[lo] == item;
      const double rank = (double)(r + 1);
      const double disc = 1.0 / log2(rank + 1.0);
      if (hit) {
        cum += 1.0;
        dcg += disc;
        sum_pre += cum / rank;
      }
      if (r < plen) idcg += disc;
      while (ki < n_ks && ks[ki] == r + 1) {
        const double kk = (double)(r + 1);
        m[0][ki] = cum / (double)plen;
        m[1][ki] = dcg / idcg;
        m[2][ki] = cum / kk;
        m[3][ki] = sum_pre / (double)(plen < r + 1 ? plen : r + 1);
        ++ki;
      }
    }
  }
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      double v = gmr::wave_sum_d(m[a][b]);
      if ((threadIdx.x & 63) == 0) red[a][b][w] = v;
    }
  __syncthreads();
  if (threadIdx.x < 32) {
    const int a = threadIdx.x >> 3, b = threadIdx.x & 7;
    part[(int64_t)blockIdx.x * 32 + threadIdx.x] = (red[a][b][0] + red[a][b][1]) + (red[a][b][2] + red[a][b][3]);
  }
}

// per-item recommendation counts of the top-ks[j] columns (Coverage / Gini / Tail%, topk_evaluator.py:212-270);
// integer atomics, so the counts are exact whatever the order
__global__ void item_counts_kernel(int64_t n_users, const int* __restrict__ topk, int64_t ld_topk, int n_ks,
                                   const int* __restrict__ ks, int64_t n_items, int* __restrict__ counts) {
  const int kmax = ks[n_ks - 1];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_users * kmax) return;
  const int64_t u = i / kmax;
  const int r = (int)(i % kmax);
  const int item = topk[u * ld_topk + r];
  if (item < 0 || item >= n_items) return;
  for (int j = 0; j < n_ks; ++j)
    if (r < ks[j]) atomicAdd(&counts[(int64_t)j * n_items + item], 1);
}

__global__ void reduce_parts_kernel(int nparts, int width, const double* __restrict__ part, double* __restrict__ out) {
  const int c = threadIdx.x;
  if (c >= width) return;
  double s = 0.0;
  for (int i = 0; i < nparts; ++i) s += part[(int64_t)i * width + c];
  out[c] = s;
}

}  // namespace

extern "C" int gmr_mask_scores_f32(int64_t n, const int32_t* rows, const int32_t* cols, float* scores, int64_t ld,
                                   float fill, void* stream) {
  GMR_ARG(scores && (n == 0 || (rows && cols)), "bad args");
  if (n == 0) return GMR_OK;
  hipLaunchKernelGGL(mask_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, rows, cols, scores,
                     ld, fill);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_topk_rows_f32(int64_t n_rows, int64_t n_cols, const float* scores, int64_t ld, int32_t k,
                                 int32_t* out_idx, int64_t ld_idx, float* out_val, void* stream) {
  GMR_ARG(scores && out_idx && n_rows > 0 && n_cols > 0, "bad args");
  GMR_ARG(k >= 1 && k <= 64 && k <= n_cols, "k must be in [1, min(64, n_cols)]");
  GMR_ARG((n_cols + TK_THREADS - 1) / TK_THREADS < 32768, "n_cols too large");
  GMR_ARG(n_rows < (1ll << 31), "too many rows");
  if (k == 1)
    hipLaunchKernelGGL(argmax_rows_kernel, dim3((unsigned)n_rows), dim3(256), 0, (hipStream_t)stream, n_rows, n_cols,
                       scores, ld, out_idx, ld_idx, out_val);
  else if (n_cols <= TK_STAGE_COLS) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(topk_rows_kernel<true>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)sizeof(uint32_t) * TK_STAGE_COLS);
    if (attr != hipSuccess) return gmr::hip_status(__func__, attr);
    hipLaunchKernelGGL(topk_rows_kernel<true>, dim3((unsigned)n_rows), dim3(TK_THREADS), sizeof(uint32_t) * n_cols,
                       (hipStream_t)stream, n_rows, n_cols, scores, ld, k, out_idx, ld_idx, out_val);
  } else
    hipLaunchKernelGGL(topk_rows_kernel<false>, dim3((unsigned)n_rows), dim3(TK_THREADS), 0, (hipStream_t)stream,
                       n_rows, n_cols, scores, ld, k, out_idx, ld_idx, out_val);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int64_t gmr_eval_metrics_partials(int64_t n_users) { return 32 * (int64_t)gmr::grid_for(n_users, 256); }

extern "C" int gmr_eval_metrics(int64_t n_users, const int32_t* topk, int64_t ld_topk, int32_t K,
                                const int64_t* pos_ptr, const int32_t* pos_items, int32_t n_ks, const int32_t* ks,
                                double* partials, double* out_sums, void* stream) {
  GMR_ARG(topk && pos_ptr && pos_items && ks && partials && out_sums && n_users > 0, "bad args");
  GMR_ARG(n_ks >= 1 && n_ks <= 8 && K <= 64, "n_ks must be 1..8");
  const int g = gmr::grid_for(n_users, 256);
  hipLaunchKernelGGL(metrics_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, n_users, nullptr, topk, ld_topk, K,
                     pos_ptr, pos_items, n_ks, ks, partials);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(reduce_parts_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, g, 32, partials, out_sums);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_eval_metrics_sel(int64_t n_sel, const int32_t* sel, const int32_t* topk, int64_t ld_topk, int32_t K,
                                    const int64_t* pos_ptr, const int32_t* pos_items, int32_t n_ks, const int32_t* ks,
                                    double* partials, double* out_sums, void* stream) {
  GMR_ARG(sel && topk && pos_ptr && pos_items && ks && partials && out_sums && n_sel > 0, "bad args");
  GMR_ARG(n_ks >= 1 && n_ks <= 8 && K <= 64, "n_ks must be 1..8");
  const int g = gmr::grid_for(n_sel, 256);
  hipLaunchKernelGGL(metrics_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, n_sel, sel, topk, ld_topk, K, pos_ptr,
                     pos_items, n_ks, ks, partials);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(reduce_parts_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, g, 32, partials, out_sums);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_topk_item_counts(int64_t n_users, const int32_t* topk, int64_t ld_topk, int32_t n_ks,
                                    const int32_t* ks, int64_t n_items, int32_t* counts, void* stream) {
  GMR_ARG(topk && ks && counts && n_users > 0 && n_items > 0 && n_ks >= 1 && n_ks <= 8, "bad args");
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(counts, 0, sizeof(int32_t) * (size_t)n_ks * (size_t)n_items, st);
  if (e != hipSuccess) return gmr::hip_status(__func__, e);
  // ks sorted ascending, the last one <= the top-k width (callers pass the evaluator's sorted topk list)
  hipLaunchKernelGGL(item_counts_kernel, dim3(gmr::grid_for(n_users * 64, 256)), dim3(256), 0, st, n_users, topk, ld_topk,
                     n_ks, ks, n_items, counts);
  GMR_LAUNCHED();
  return GMR_OK;
}
