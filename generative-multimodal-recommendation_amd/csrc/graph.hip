// K11 — device construction of the symmetric-normalised bipartite adjacency in CSR.
//
//   rows 0..U-1      user u : [u (self loop, optional)] + [U + item for its items, ascending]
//   rows U..U+I-1    item i : [users that hold i, ascending] + [U + i (self loop, optional)]
//   val(r, c) = float( (deg_r + eps)^-1/2 * (deg_c + eps)^-1/2 )   computed in fp64
//
// Serves both reference builders:
//   DiffMM.get_norm_adj_mat   models/diffmm.py:88-107   (no self loops, eps = 1e-7)
//   DiffMMTrainer.buildUIMatrix + normalizeAdj   common/trainer.py:464-485  (self loops, eps = 0)
// Columns are sorted inside each row, so the CSR equals the reference's coalesced COO.
// Item rows are filled through atomically claimed slots, then each row is put in user order
// by its own workgroup (rank count / LDS bitmap), so the build is deterministic.
#include <algorithm>

#include "gmr_common.h"

namespace {

__global__ void count_items_kernel(int64_t nnz, const int* __restrict__ items, int* __restrict__ cnt) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nnz) atomicAdd(&cnt[items[e]], 1);
}

// rowptr for all N+1 rows (single block, chunked serial + LDS scan over 1024 chunk sums)
__global__ void __launch_bounds__(1024) rowptr_kernel(int U, int I, const int* __restrict__ uptr,
                                                      const int* __restrict__ cnt, int sl, int* __restrict__ rowptr) {
  __shared__ int s[1024];
  const int t = threadIdx.x;
  const int N = U + I;
  const int chunk = (N + 1023) / 1024;
  const int r0 = t * chunk, r1 = min(N, r0 + chunk);
  int sum = 0;
  for (int r = r0; r < r1; ++r) sum += (r < U ? uptr[r + 1] - uptr[r] : cnt[r - U]) + sl;
  s[t] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    int v = t >= off ? s[t - off] : 0;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  int o = s[t] - sum;
  for (int r = r0; r < r1; ++r) {
    rowptr[r] = o;
    o += (r < U ? uptr[r + 1] - uptr[r] : cnt[r - U]) + sl;
  }
  if (t == 1023) rowptr[N] = s[1023];
}

// user rows in place; every entry is also scattered into its item row at an atomically
// claimed slot (order fixed afterwards by item_sort_kernel)
__global__ void user_rows_kernel(int U, const int* __restrict__ uptr, const int* __restrict__ uitems, int sl,
                                 const int* __restrict__ rowptr, int* __restrict__ col, int* __restrict__ fill) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  int o = rowptr[u];
  if (sl) col[o++] = u;
  for (int e = uptr[u]; e < uptr[u + 1]; ++e) {
    const int it = uitems[e];
    col[o++] = U + it;
    col[rowptr[U + it] + atomicAdd(&fill[it], 1)] = u;
  }
}

// LDS-privatised variants for I <= kLdsItems: each block counts its users' items in LDS and
// touches every global counter once (the rebuilt graphs send most users to a few popular items,
// where one global atomic per entry serialises on the same address).
constexpr int kLdsItems = 8192;
constexpr int kPrivBlocks = 64;
__global__ void __launch_bounds__(1024) count_items_priv_kernel(int U, int I, const int* __restrict__ uptr,
                                                                const int* __restrict__ uitems, int* __restrict__ cnt) {
  __shared__ int hist[kLdsItems];
  const int t = threadIdx.x;
  for (int i = t; i < I; i += 1024) hist[i] = 0;
  __syncthreads();
  const int uc = (U + gridDim.x - 1) / gridDim.x;
  const int u0 = blockIdx.x * uc, u1 = min(U, u0 + uc);
  const int e0 = u0 < U ? uptr[u0] : 0, e1 = u0 < U ? uptr[u1] : 0;
  for (int e = e0 + t; e < e1; e += 1024) atomicAdd(&hist[uitems[e]], 1);
  __syncthreads();
  for (int i = t; i < I; i += 1024)
    if (hist[i]) atomicAdd(&cnt[i], hist[i]);
}

__global__ void __launch_bounds__(1024) user_rows_priv_kernel(int U, int I, const int* __restrict__ uptr,
                                                              const int* __restrict__ uitems, int sl,
                                                              const int* __restrict__ rowptr, int* __restrict__ col,
                                                              int* __restrict__ fill) {
  __shared__ int base[kLdsItems];
  __shared__ int loc[kLdsItems];
  const int t = threadIdx.x;
  for (int i = t; i < I; i += 1024) {
    base[i] = 0;
    loc[i] = 0;
  }
  __syncthreads();
  const int uc = (U + gridDim.x - 1) / gridDim.x;
  const int u0 = blockIdx.x * uc, u1 = min(U, u0 + uc);
  const int e0 = u0 < U ? uptr[u0] : 0, e1 = u0 < U ? uptr[u1] : 0;
  for (int e = e0 + t; e < e1; e += 1024) atomicAdd(&base[uitems[e]], 1);
  __syncthreads();
  for (int i = t; i < I; i += 1024)
    if (base[i]) base[i] = atomicAdd(&fill[i], base[i]);
  __syncthreads();
  // user rows (in place) + item-row slots claimed from the block's reserved ranges
  for (int u = u0 + t; u < u1; u += 1024) {
    int o = rowptr[u];
    if (sl) col[o++] = u;
    for (int e = uptr[u]; e < uptr[u + 1]; ++e) {
      const int it = uitems[e];
      col[o++] = U + it;
      col[rowptr[U + it] + base[it] + atomicAdd(&loc[it], 1)] = u;
    }
  }
}

// One workgroup per item row: put the row's users in ascending order (the reference's
// coalesced COO order).  Users of a row are distinct, so short rows rank each entry by a
// count of smaller entries in LDS and long rows go through an LDS bitmap over all U users
// with a popcount prefix — deterministic and independent of the atomic slot order.
constexpr int kSortThreads = 256;
__global__ void __launch_bounds__(kSortThreads) item_sort_kernel(int U, const int* __restrict__ rowptr,
                                                                 int* __restrict__ col, int sl) {
  extern __shared__ __attribute__((aligned(16))) uint32_t bits[];  // (U + 31) / 32 words
  __shared__ int s_val[kSortThreads];
  __shared__ int s_part[kSortThreads];
  const int i = blockIdx.x, t = threadIdx.x;
  const int beg = rowptr[U + i];
  const int L = rowptr[U + i + 1] - beg - sl;
  if (sl && t == 0) col[beg + L] = U + i;
  if (L <= 1) return;
  if (L <= kSortThreads) {
    const int v = t < L ? col[beg + t] : 0;
    s_val[t] = v;
    __syncthreads();
    if (t < L) {
      int r = 0;
      for (int j = 0; j < L; ++j) r += s_val[j] < v;
      col[beg + r] = v;
    }
    return;
  }
  const int W = (U + 31) >> 5;
  for (int w = t; w < W; w += kSortThreads) bits[w] = 0u;
  __syncthreads();
  for (int e = t; e < L; e += kSortThreads) {
    const int v = col[beg + e];
    atomicOr(&bits[v >> 5], 1u << (v & 31));
  }
  __syncthreads();
  // contiguous word range per thread, block-exclusive scan of the range popcounts
  const int per = (W + kSortThreads - 1) / kSortThreads;
  const int w0 = min(W, t * per), w1 = min(W, w0 + per);
  int cnt = 0;
  for (int w = w0; w < w1; ++w) cnt += __popc(bits[w]);
  s_part[t] = cnt;
  __syncthreads();
  for (int off = 1; off < kSortThreads; off <<= 1) {
    const int a = t >= off ? s_part[t - off] : 0;
    __syncthreads();
    s_part[t] += a;
    __syncthreads();
  }
  int o = beg + s_part[t] - cnt;
  for (int w = w0; w < w1; ++w) {
    uint32_t b = bits[w];
    while (b) {
      const int k = __ffs(b) - 1;
      col[o++] = (w << 5) + k;
      b &= b - 1;
    }
  }
}

// d[r] = (deg_r + eps)^-1/2 in fp64, once per node
__global__ void dis_kernel(int N, const int* __restrict__ rowptr, double eps, double* __restrict__ dis) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < N) dis[r] = pow((double)(rowptr[r + 1] - rowptr[r]) + eps, -0.5);
}

// one wave per row: values d_r * d_c in fp64, rounded once to fp32
__global__ void values_kernel(int N, const int* __restrict__ rowptr, const int* __restrict__ col,
                              const double* __restrict__ dis, float* __restrict__ val) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= N) return;
  const int lane = threadIdx.x & 63;
  const int beg = rowptr[r], end = rowptr[r + 1];
  const double dr = dis[r];
  for (int e = beg + lane; e < end; e += 64) val[e] = (float)(dr * dis[col[e]]);
}

// sort the k items of each user (insertion sort, k <= 64) and write uptr = u*k
__global__ void topk_to_user_csr_kernel(int U, int k, const int* __restrict__ topk, int64_t ld, int* __restrict__ uptr,
                                        int* __restrict__ uitems) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u > U) return;
  uptr[u] = u * k;
  if (u == U) return;
  int v[64];
  for (int j = 0; j < k; ++j) {
    int x = topk[(int64_t)u * ld + j];
    int p = j;
    while (p > 0 && v[p - 1] > x) {
      v[p] = v[p - 1];
      --p;
    }
    v[p] = x;
  }
  for (int j = 0; j < k; ++j) uitems[u * k + j] = v[j];
}

}  // namespace

extern "C" int64_t gmr_bipartite_nnz(int64_t n_users, int64_t n_items, int64_t n_user_items, int32_t self_loops) {
  return 2 * n_user_items + (self_loops ? n_users + n_items : 0);
}

extern "C" int64_t gmr_bipartite_workspace_ints(int64_t n_users, int64_t n_items) {
  return 2 * n_items + 2 * (n_users + n_items) + 2;  // counters | fp64 d (8-byte aligned)
}

extern "C" int gmr_bipartite_symnorm_build(int64_t n_users, int64_t n_items, const int32_t* user_ptr,
                                           const int32_t* user_items, int64_t n_user_items, int32_t self_loops,
                                           double deg_eps, int32_t* workspace, int32_t* rowptr, int32_t* col,
                                           float* val, void* stream) {
  GMR_ARG(user_ptr && user_items && workspace && rowptr && col && val, "null pointer");
  GMR_ARG(n_users > 0 && n_items > 0 && n_users + n_items < (1ll << 30), "bad size");
  GMR_ARG(2 * n_user_items + n_users + n_items < (1ll << 31), "too many entries");
  hipStream_t st = (hipStream_t)stream;
  const int U = (int)n_users, I = (int)n_items, N = U + I;
  const int sl = self_loops ? 1 : 0;
  GMR_ARG(n_users <= 1200000, "n_users above the LDS bitmap budget of the item-row sort");
  int* cnt = workspace;
  hipError_t e = hipMemsetAsync(workspace, 0, sizeof(int) * 2 * (size_t)I, st);
  if (e != hipSuccess) return gmr::hip_status(__func__, e);
  const bool priv = I <= kLdsItems;
  const int pblocks = (int)std::min<int64_t>(kPrivBlocks, std::max<int64_t>(1, n_user_items / 2048));
  if (n_user_items > 0) {
    if (priv)
      hipLaunchKernelGGL(count_items_priv_kernel, dim3(pblocks), dim3(1024), 0, st, U, I, user_ptr, user_items, cnt);
    else
      hipLaunchKernelGGL(count_items_kernel, dim3(gmr::grid_for(n_user_items, 256)), dim3(256), 0, st, n_user_items,
                         user_items, cnt);
    GMR_LAUNCHED();
  }
  hipLaunchKernelGGL(rowptr_kernel, dim3(1), dim3(1024), 0, st, U, I, user_ptr, cnt, sl, rowptr);
  GMR_LAUNCHED();
  if (priv)
    hipLaunchKernelGGL(user_rows_priv_kernel, dim3(pblocks), dim3(1024), 0, st, U, I, user_ptr, user_items, sl, rowptr,
                       col, workspace + I);
  else
    hipLaunchKernelGGL(user_rows_kernel, dim3(gmr::grid_for(U, 256)), dim3(256), 0, st, U, user_ptr, user_items, sl,
                       rowptr, col, workspace + I);
  GMR_LAUNCHED();
  const size_t dyn = sizeof(uint32_t) * (size_t)((U + 31) / 32);
  if (dyn > 65536) {
    e = hipFuncSetAttribute((const void*)item_sort_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
    if (e != hipSuccess) return gmr::hip_status(__func__, e);
  }
  hipLaunchKernelGGL(item_sort_kernel, dim3(I), dim3(kSortThreads), dyn, st, U, rowptr, col, sl);
  GMR_LAUNCHED();
  double* dis = reinterpret_cast<double*>(workspace + 2 * (int64_t)I + ((2 * (int64_t)I) & 1));
  hipLaunchKernelGGL(dis_kernel, dim3(gmr::grid_for(N, 256)), dim3(256), 0, st, N, rowptr, deg_eps, dis);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(values_kernel, dim3(gmr::grid_for(N, 4)), dim3(256), 0, st, N, rowptr, col, dis, val);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_topk_to_user_csr(int64_t n_users, int32_t k, const int32_t* topk, int64_t ld, int32_t* user_ptr,
                                    int32_t* user_items, void* stream) {
  GMR_ARG(topk && user_ptr && user_items && n_users > 0, "bad args");
  GMR_ARG(k >= 1 && k <= 64, "k must be 1..64");
  hipLaunchKernelGGL(topk_to_user_csr_kernel, dim3(gmr::grid_for(n_users + 1, 256)), dim3(256), 0, (hipStream_t)stream,
                     (int)n_users, k, topk, ld, user_ptr, user_items);
  GMR_LAUNCHED();
  return GMR_OK;
}
