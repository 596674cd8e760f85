// On-device BPR epoch sampler (replaces the host pandas shuffle + Python rejection sampler
// of utils/dataloader.py:218-275).  Semantics kept: every train interaction appears once
// per epoch in a uniformly random order; the negative is drawn uniformly from the items
// that occur in the training split (TrainDataLoader.all_items, :116) and redrawn while it
// is in the user's history (:267-275).  The random streams are our own (Philox), so the
// batches are statistically — not bitwise — equivalent to the reference's.  The reference redraws
// without bound (it would never return for a user holding every item); here a row gives up after
// kMaxDraws draws, keeps its last candidate and is counted in *n_fallback, so a caller can report it.
#include "gmr_common.h"

namespace {

constexpr int kMaxDraws = 4096;

// Balanced Feistel bijection on [0, 2^bits) (bits even), 4 rounds keyed by Philox output;
// cycle-walking maps it to a bijection on [0, n).
__device__ uint32_t feistel(uint32_t x, int bits, uint4 k) {
  const int hb = bits / 2;
  const uint32_t m = (1u << hb) - 1;
  uint32_t L = x >> hb, R = x & m;
  const uint32_t keys[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    uint32_t f = R * 0x9E3779B1u ^ keys[r];
    f ^= f >> 15;
    f *= 0x85EBCA77u;
    f ^= f >> 13;
    const uint32_t nr = (L ^ f) & m;
    L = R;
    R = nr;
  }
  return (L << hb) | R;
}

__device__ __forceinline__ uint32_t perm_index(uint32_t p, uint32_t n, int bits, uint4 k) {
  uint32_t x = p;
  // cycle-walking keeps a bijection on [0, n)
  for (int it = 0; it < 4096; ++it) {
    x = feistel(x, bits, k);
    if (x < n) return x;
  }
  return p;  // unreachable: each walk step lands in [0,n) with probability >= 1/4
}

__device__ bool has_item(const int* __restrict__ items, int beg, int end, int v) {
  int lo = beg, hi = end;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    int x = items[mid];
    if (x < v) lo = mid + 1;
    else hi = mid;
  }
  return lo < end && items[lo] == v;
}

__global__ void sample_epoch_kernel(int n, int bits, const int* __restrict__ iu, const int* __restrict__ ii,
                                    const int* __restrict__ rowptr, const int* __restrict__ items,
                                    const int* __restrict__ all_items, int n_all, uint64_t seed, uint64_t epoch,
                                    int* __restrict__ out_u, int* __restrict__ out_p, int* __restrict__ out_n,
                                    int* __restrict__ n_fallback) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint4 k = gmr::Philox::gen(seed, epoch, 0xFEED);
  const uint32_t j = perm_index((uint32_t)p, (uint32_t)n, bits, k);
  const int u = iu[j];
  out_u[p] = u;
  out_p[p] = ii[j];
  const int beg = rowptr[u], end = rowptr[u + 1];
  int cand = 0;
  bool found = false;
  for (int attempt = 0; attempt < kMaxDraws && !found; ++attempt) {
    const uint4 r = gmr::Philox::gen(seed ^ 0x5DEECE66Dull, (epoch << 32) | (uint32_t)attempt, (uint64_t)p);
    cand = all_items[(int)(((uint64_t)r.x * (uint64_t)n_all) >> 32)];
    found = !has_item(items, beg, end, cand);
  }
  out_n[p] = cand;
  if (!found && n_fallback) atomicAdd(n_fallback, 1);
}

}  // namespace

extern "C" int gmr_sample_epoch(int64_t n_inter, const int32_t* inter_user, const int32_t* inter_item,
                                const int32_t* user_rowptr, const int32_t* user_items, const int32_t* all_items,
                                int64_t n_all_items, uint64_t seed, uint64_t epoch, int32_t* out_users,
                                int32_t* out_pos, int32_t* out_neg, int32_t* n_fallback, void* stream) {
  GMR_ARG(inter_user && inter_item && user_rowptr && user_items && all_items && out_users && out_pos && out_neg,
          "null pointer");
  GMR_ARG(n_inter > 0 && n_inter < (1ll << 31) && n_all_items > 0, "bad size");
  int bits = 2;
  while ((1ll << bits) < n_inter) ++bits;
  if (bits & 1) ++bits;  // even width keeps both Feistel halves equal
  hipLaunchKernelGGL(sample_epoch_kernel, dim3(gmr::grid_for(n_inter, 256)), dim3(256), 0, (hipStream_t)stream,
                     (int)n_inter, bits, inter_user, inter_item, user_rowptr, user_items, all_items, (int)n_all_items,
                     seed, epoch, out_users, out_pos, out_neg, n_fallback);
  GMR_LAUNCHED();
  return GMR_OK;
}

namespace {
__global__ void permutation_kernel(int n, int bits, uint64_t seed, uint64_t epoch, int* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint4 k = gmr::Philox::gen(seed, epoch, 0xBEEF);
  out[p] = (int)perm_index((uint32_t)p, (uint32_t)n, bits, k);
}
}  // namespace

extern "C" int gmr_permutation(int64_t n, uint64_t seed, uint64_t epoch, int32_t* out, void* stream) {
  GMR_ARG(out && n > 0 && n < (1ll << 31), "bad args");
  int bits = 2;
  while ((1ll << bits) < n) ++bits;
  if (bits & 1) ++bits;
  hipLaunchKernelGGL(permutation_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, (int)n, bits,
                     seed, epoch, out);
  GMR_LAUNCHED();
  return GMR_OK;
}
