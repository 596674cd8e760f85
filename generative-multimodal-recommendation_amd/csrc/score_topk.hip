// K9 + K10 fused — full-rank eval in one kernel, no E x I score matrix:
//   scores = U[users] . I^T            (models/diffmm.py:276-277, genrecv1.py:426, vbpr.py full_sort_predict)
//   scores[train positives] = -1e10    (common/trainer.py:383-384)
//   top-k per row, score desc, ties -> lowest index   (torch.topk, common/trainer.py:386)
//
// One wave owns 16 user rows and streams the whole item table past them in 64-item steps:
//   * scores on the fp32 matrix cores (v_mfma_f32_16x16x4_f32, exact fp32 products, fp32 sums): the k
//     order is permuted so each lane reads 16 CONSECUTIVE k of one user row (A, loaded once) and of one
//     item row (B, four float4 per 16-item tile, straight from L2: the table is 1.8 MB at baby);
//   * the mask: each row's train positives are sorted, so a lane only compares the row's next masked
//     item with the step's range (a load only when one falls inside);
//   * selection: per row a candidate buffer of 128 (score key, item) pairs in LDS and a threshold tau =
//     the k-th best score among the items seen so far.  An item enters only if its score beats tau
//     STRICTLY (items arrive in increasing index order, so an equal score loses the tie); when a buffer
//     passes 112 entries (checked per 16-item tile) the wave selects its k smallest 64-bit keys ((~okey(score)) << 32 | item: unique,
//     so there are no ties to break) by a bitwise radix select on ballots, keeps exactly those and raises
//     tau.  After the last step the k survivors are sorted by a 64-lane bitonic network.
// The selection is exact (the same k items, in the same order, as a full radix top-k over the masked
// row); the scores are fp32 MFMA dot products like the unfused GEMM's (summation order may differ).
#include "gmr_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int ST_WAVES = 4;     // waves per workgroup (independent: no block barrier)
constexpr int ST_ROWS = 16;     // rows per wave (one 16 x 16 MFMA tile height)
constexpr int ST_CAP = 128;     // candidate slots per row (two 4-wave workgroups per CU fit the LDS)
constexpr int ST_TILES = 4;     // 16-item tiles per step
constexpr int ST_STEP = 16 * ST_TILES;
constexpr int ST_MSTAGE = 512;   // masked items of a wave's 16 rows staged in LDS

__device__ __forceinline__ uint32_t okey(float f) {  // order-preserving uint32 key
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float okey_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Keep the K smallest of the row's n (<= ST_CAP) unique 64-bit entries in slots [0, K) (any order);
// returns tau = okey of the K-th best score.  Wave-uniform call.
__device__ uint32_t st_compact(unsigned long long* buf, int n, int K, int lane) {
  constexpr int NE = ST_CAP / 64;
  unsigned long long e[NE];
  bool v[NE];
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int i = lane + 64 * j;
    v[j] = i < n;
    e[j] = v[j] ? buf[i] : ~0ull;
  }
  // high word (~okey): its K-th smallest value H, and how many entries equal to H are among the K
  uint32_t H = 0;
  int need = K;
#pragma unroll 1
  for (int b = 31; b >= 0; --b) {
    const uint32_t m = ~0u << b;
    int c = 0;
#pragma unroll
    for (int j = 0; j < NE; ++j) c += __popcll(__ballot(v[j] && ((((uint32_t)(e[j] >> 32)) ^ H) & m) == 0));
    if (c < need) {
      need -= c;
      H |= 1u << b;
    }
  }
  int eq = 0;
#pragma unroll
  for (int j = 0; j < NE; ++j) eq += __popcll(__ballot(v[j] && (uint32_t)(e[j] >> 32) == H));
  uint32_t L = 0xffffffffu;
  if (eq > need) {  // equal scores straddle the cut: the lowest items among them stay
    L = 0;
#pragma unroll 1
    for (int b = 31; b >= 0; --b) {
      const uint32_t m = ~0u << b;
      int c = 0;
#pragma unroll
      for (int j = 0; j < NE; ++j)
        c += __popcll(__ballot(v[j] && (uint32_t)(e[j] >> 32) == H && ((((uint32_t)e[j]) ^ L) & m) == 0));
      if (c < need) {
        need -= c;
        L |= 1u << b;
      }
    }
  }
  const unsigned long long T = ((unsigned long long)H << 32) | L;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int pos = 0;
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const bool keep = v[j] && e[j] <= T;
    const unsigned long long bal = __ballot(keep);
    if (keep) buf[pos + __popcll(bal & lt)] = e[j];
    pos += __popcll(bal);
  }
  return ~H;
}

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long x, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)x, m), hi = __shfl_xor((uint32_t)(x >> 32), m);
  return ((unsigned long long)hi << 32) | lo;
}

// One wave's 16 rows (DK = D / 64: embedding width 64 or 128).  STAGED: the rows' masked items sit in
// the wave's LDS slice (a mask lookup is an LDS read); otherwise (more than ST_MSTAGE masked items in
// the 16 rows) they are read from global memory, which also waits for the item prefetch in flight.
template <int DK, bool STAGED>
__device__ __forceinline__ void score_topk_wave(int64_t n_rows, int64_t row0, int lane, const float (&a)[16 * DK],
                                                int64_t n_items, const float* __restrict__ I, int64_t ldi,
                                                const int64_t* __restrict__ mptr, const int* __restrict__ mcols,
                                                const int* ms, int64_t mbase, float fill, int K,
                                                unsigned long long (*cb)[ST_CAP], int* cn,
                                                unsigned long long* trash) {
  constexpr int KS = 16 * DK;
  const int col = lane & 15, grp = lane >> 4;
  auto mask_at = [&](int64_t i) -> int { return STAGED ? ms[i - mbase] : mcols[i]; };
  // the lane's output rows are row0 + 4 grp + e (MFMA C/D map: row = 4 (lane >> 4) + reg, col = lane & 15)
  int64_t mc[4], me[4];
  int nm[4];
  uint32_t tau[4];
  int cnt[4];  // entries in the buffers of the lane's rows (the same in the 16 lanes of a row group)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t r = row0 + 4 * grp + e;
    mc[e] = r < n_rows ? mptr[r] : 0;
    me[e] = r < n_rows ? mptr[r + 1] : 0;
    nm[e] = mc[e] < me[e] ? mask_at(mc[e]) : 0x7fffffff;
    tau[e] = 0;
    cnt[e] = 0;
  }
  // items [c0, c0 + 64): this lane's 16 consecutive k of item c0 + 16 t + col (clamped: the loads of
  // a step past the end are issued anyway, so no branch splits the prefetch from its use; 32-bit
  // offsets, n_items * ldi < 2^31 is checked by the host)
  const int nlast = (int)n_items - 1, ld32 = (int)ldi;
  const float* __restrict__ ig = I + KS * grp;
  auto load_b = [&](int c0, float (&bb)[ST_TILES][KS]) {
#pragma unroll
    for (int t = 0; t < ST_TILES; ++t) {
      const float4* p = reinterpret_cast<const float4*>(ig + min(c0 + 16 * t + col, nlast) * ld32);
#pragma unroll
      for (int q = 0; q < KS / 4; ++q) {
        const float4 x = p[q];
        bb[t][4 * q] = x.x;
        bb[t][4 * q + 1] = x.y;
        bb[t][4 * q + 2] = x.z;
        bb[t][4 * q + 3] = x.w;
      }
    }
  };
  auto mfma = [&](const float (&b)[ST_TILES][KS], f32x4 (&acc)[ST_TILES]) {
#pragma unroll
    for (int t = 0; t < ST_TILES; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int t = 0; t < ST_TILES; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[t][s], acc[t], 0, 0, 0);
  };
  // train positives of the lane's rows inside [c0, c0 + 64) -> fill (a wave-uniform test; the loop
  // runs only in the rare steps that hold one)
  auto mask_fix = [&](int c0, f32x4 (&acc)[ST_TILES]) {
    bool hit = false;
#pragma unroll
    for (int e = 0; e < 4; ++e) hit |= nm[e] < c0 + ST_STEP;
    if (!__ballot(hit)) return;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      while (nm[e] < c0 + ST_STEP) {
        const int d = nm[e] - c0;
        if (d >= 0 && (d & 15) == col) {
#pragma unroll
          for (int t = 0; t < ST_TILES; ++t)
            if (t == (d >> 4)) acc[t][e] = fill;
        }
        ++mc[e];
        nm[e] = mc[e] < me[e] ? mask_at(mc[e]) : 0x7fffffff;
      }
    }
  };
  // candidates of one step, branch-free: a row's slots come from a ballot over the 16 lanes of its group
  // (tile by tile); a lane with nothing to insert writes its own trash slot
  const uint32_t below = (1u << col) - 1u;
  // a row near its capacity (one tile adds at most 16): keep its k best, raise its tau
  auto compact_check = [&]() {
    bool near = false;
#pragma unroll
    for (int e = 0; e < 4; ++e) near |= cnt[e] > ST_CAP - 16;
    if (!__ballot(near)) return;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      unsigned long long full = __ballot(col == 0 && cnt[e] > ST_CAP - 16);  // one bit per row group
      while (full) {
        const int g = (__ffsll((long long)full) - 1) >> 4;
        full &= full - 1;
        const int r = 4 * g + e;
        const int n = __shfl(cnt[e], 16 * g);
        const uint32_t nt = st_compact(cb[r], n, K, lane);
        if (grp == g) {
          tau[e] = nt;
          cnt[e] = K;
        }
      }
    }
  };
  auto filter = [&](int c0, const f32x4 (&acc)[ST_TILES]) {
#pragma unroll
    for (int t = 0; t < ST_TILES; ++t) {
      const int c = c0 + 16 * t + col;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t k = okey(acc[t][e]);
        const bool in = c < n_items && k > tau[e];
        const uint32_t g = (uint32_t)(__ballot(in) >> (16 * grp)) & 0xffffu;
        unsigned long long* dst = in ? &cb[4 * grp + e][cnt[e] + __popc(g & below)] : trash;
        *dst = ((unsigned long long)(~k) << 32) | (uint32_t)c;
        cnt[e] += __popc(g);
      }
      compact_check();
    }
  };
  // software pipeline: the MFMAs of step j + 1 are issued before the filter of step j (independent
  // registers: the matrix pipe runs while the vector pipe filters); two item register sets and two
  // accumulator sets, the loads of step j + 2 in flight meanwhile
  float b0[ST_TILES][KS], b1[ST_TILES][KS];
  f32x4 acc0[ST_TILES], acc1[ST_TILES];
  load_b(0, b0);
  load_b(ST_STEP, b1);
  mfma(b0, acc0);
  const int ni = (int)n_items;
#pragma unroll 1
  for (int c0 = 0;; c0 += 2 * ST_STEP) {
    mask_fix(c0, acc0);
    load_b(c0 + 2 * ST_STEP, b0);
    __builtin_amdgcn_sched_barrier(0);
    mfma(b1, acc1);
    filter(c0, acc0);
    if (c0 + ST_STEP >= ni) break;
    mask_fix(c0 + ST_STEP, acc1);
    load_b(c0 + 3 * ST_STEP, b1);
    __builtin_amdgcn_sched_barrier(0);
    mfma(b0, acc0);
    filter(c0 + ST_STEP, acc1);
    if (c0 + 2 * ST_STEP >= ni) break;
  }
  if (col == 0) {  // the final pass reads the counts from LDS
#pragma unroll
    for (int e = 0; e < 4; ++e) cn[4 * grp + e] = cnt[e];
  }
}

template <int DK>
__global__ void __launch_bounds__(64 * ST_WAVES, DK == 1 ? 2 : 1) score_topk_kernel(
    int64_t n_rows, const int* __restrict__ users, const float* __restrict__ U, int64_t ldu, int64_t n_items,
    const float* __restrict__ I, int64_t ldi, const int64_t* __restrict__ mptr, const int* __restrict__ mcols,
    float fill, int K, int* __restrict__ out_idx, int64_t ld_idx, float* __restrict__ out_val) {
  __shared__ unsigned long long cand[ST_WAVES][ST_ROWS][ST_CAP];
  __shared__ int cnt[ST_WAVES][ST_ROWS];
  __shared__ int mstage[ST_WAVES][ST_MSTAGE];
  __shared__ unsigned long long trash[ST_WAVES][64];  // per-lane sink of the branch-free candidate writes
  constexpr int KS = 16 * DK;  // k values per lane: lane group g holds k in [KS g, KS (g + 1))
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, col = lane & 15, grp = lane >> 4;
  const int64_t row0 = ((int64_t)blockIdx.x * ST_WAVES + w) * ST_ROWS;
  if (row0 >= n_rows) return;
  unsigned long long(*cb)[ST_CAP] = cand[w];
  int* cn = cnt[w];

  float a[KS];  // A[row col][k = KS grp + s]
  {
    const int64_t r = min(row0 + col, n_rows - 1);
    const int64_t u = users ? (int64_t)users[r] : r;
    const float4* p = reinterpret_cast<const float4*>(U + u * ldu + KS * grp);
#pragma unroll
    for (int q = 0; q < KS / 4; ++q) {
      const float4 x = p[q];
      a[4 * q] = x.x;
      a[4 * q + 1] = x.y;
      a[4 * q + 2] = x.z;
      a[4 * q + 3] = x.w;
    }
  }
  if (lane < ST_ROWS) cn[lane] = 0;
  const int64_t mbase = mptr[row0], mend = mptr[min(row0 + ST_ROWS, n_rows)];
  if (mend - mbase <= ST_MSTAGE) {
    for (int64_t i = mbase + lane; i < mend; i += 64) mstage[w][i - mbase] = mcols[i];
    // other lanes of this wave read the staged entries: order the LDS writes before those reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    score_topk_wave<DK, true>(n_rows, row0, lane, a, n_items, I, ldi, mptr, mcols, mstage[w], mbase, fill, K, cb, cn,
                              &trash[w][lane]);
  } else {
    score_topk_wave<DK, false>(n_rows, row0, lane, a, n_items, I, ldi, mptr, mcols, mstage[w], mbase, fill, K, cb, cn,
                              &trash[w][lane]);
  }
  // final: the k best of each row, sorted ascending on the 64-bit key (score desc, item asc)
#pragma unroll 1
  for (int r = 0; r < ST_ROWS; ++r) {
    const int64_t row = row0 + r;
    if (row >= n_rows) break;
    int n = cn[r];
    if (n > K) {
      st_compact(cb[r], n, K, lane);
      n = K;
    }
    unsigned long long x = lane < n ? cb[r][lane] : ~0ull;
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const unsigned long long o = shfl_xor_u64(x, stride);
        const bool keep_min = ((lane & stride) == 0) == ((lane & size) == 0 || size == 64);
        x = keep_min ? (o < x ? o : x) : (o < x ? x : o);
      }
    if (lane < K) {
      out_idx[row * ld_idx + lane] = (int)(uint32_t)x;
      if (out_val) out_val[row * ld_idx + lane] = okey_inv(~(uint32_t)(x >> 32));
    }
  }
}

}  // namespace

extern "C" int gmr_score_topk_f32(int64_t n_rows, const int32_t* users, const float* user_table, int64_t ld_user,
                                  int64_t n_items, const float* item_table, int64_t ld_item, int64_t dim,
                                  const int64_t* mask_ptr, const int32_t* mask_cols, float fill, int32_t k,
                                  int32_t* out_idx, int64_t ld_idx, float* out_val, void* stream) {
  GMR_ARG(user_table && item_table && out_idx && n_rows > 0 && n_items > 0, "bad args");
  GMR_ARG(mask_ptr && mask_cols, "mask_ptr / mask_cols required (an empty mask: mask_ptr all zero)");
  GMR_ARG(dim == 64 || dim == 128, "embedding width must be 64 or 128");
  GMR_ARG(k >= 1 && k <= 64 && k <= n_items, "k must be in [1, min(64, n_items)]");
  GMR_ARG(n_items < (1ll << 31) - ST_STEP && ld_idx >= k, "bad sizes");
  GMR_ARG(n_items * ld_item < (1ll << 31), "item table too large for 32-bit offsets");
  GMR_ARG(ld_user % 4 == 0 && ld_item % 4 == 0 && ld_user >= dim && ld_item >= dim, "leading dims: multiples of 4, >= dim");
  GMR_ARG(((uintptr_t)user_table | (uintptr_t)item_table) % 16 == 0, "tables must be 16-byte aligned");
  const int64_t waves = (n_rows + ST_ROWS - 1) / ST_ROWS;
  const dim3 grid((unsigned)((waves + ST_WAVES - 1) / ST_WAVES));
  if (dim == 64)
    hipLaunchKernelGGL(score_topk_kernel<1>, grid, dim3(64 * ST_WAVES), 0, (hipStream_t)stream, n_rows, users,
                       user_table, ld_user, n_items, item_table, ld_item, mask_ptr, mask_cols, fill, k, out_idx, ld_idx,
                       out_val);
  else
    hipLaunchKernelGGL(score_topk_kernel<2>, grid, dim3(64 * ST_WAVES), 0, (hipStream_t)stream, n_rows, users,
                       user_table, ld_user, n_items, item_table, ld_item, mask_ptr, mask_cols, fill, k, out_idx, ld_idx,
                       out_val);
  GMR_LAUNCHED();
  return GMR_OK;
}
