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
//     STRICTLY (items arrive in increasing index order, so an equal score loses the tie); a 16-item
//     tile whose scores all stay at or below their rows' thresholds costs four compares and a scalar
//     branch.  When a buffer passes 112 entries the wave keeps its k smallest 64-bit keys ((~okey(score))
//     << 32 | item: unique, so there are no ties to break), found by a radix walk on ballots that stops
//     once the k are decided (about log2(128) + a few rounds), and raises tau.  After the last step the
//     k survivors are sorted by a 64-lane bitonic network.
//   * split-bf16 scores (gmr_score_topk_x6, d = 64): the item table as three bf16 planes, the six-product
//     split of gemm_x6.hip on v_mfma_f32_16x16x32_bf16 (2.7x the fp32 MFMA rate, fp32-accurate sums).
// The selection is exact (the same k items, in the same order, as a full radix top-k over the masked
// row); the scores are fp32 MFMA dot products like the unfused GEMM's (summation order may differ).
#include <type_traits>

#include "gmr_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int ST_WAVES = 4;     // waves per workgroup (independent: no block barrier)
constexpr int ST_ROWS = 16;     // rows per wave (one 16 x 16 MFMA tile height)
constexpr int ST_CAP = 128;     // candidate slots per row (two 4-wave workgroups per CU fit the LDS)
constexpr int ST_TILES = 4;     // 16-item tiles per step (fp32 scores)
constexpr int ST_TILES_X6 = 2;  // 16-item tiles per step (split-bf16 scores: three bf16 planes per tile)
constexpr int ST_MSTAGE = 512;   // masked items of a wave's 16 rows staged in LDS

__device__ __forceinline__ uint32_t okey(float f) {  // order-preserving uint32 key
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float okey_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// exact three-way bf16 split x = hi + mid + lo (gemm_x6.hip's split3, same clamp into bf16's range)
__device__ __forceinline__ void st_split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)__builtin_amdgcn_fmed3f(x, -0x1.fep127f, 0x1.fep127f);
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

// Keep the K smallest of the row's n (K < n <= ST_CAP) unique 64-bit entries in slots [0, K) (any order);
// returns tau = okey of the K-th best score.  Wave-uniform call.  A radix walk down the 64-bit keys,
// one ballot count per bit, that stops as soon as the K are decided: after round b every entry whose
// top bits lie below the prefix P is in, every entry above it is out, and `need` of the `cnt` entries
// sharing the prefix are still to be taken; the walk ends when need == cnt (all of them) or need == 0
// (none).  Unique keys separate after about log2(n) + a few rounds instead of the fixed 32 or 64.
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
  unsigned long long P = 0;  // decided top bits (64 - s of them)
  int need = K, cnt = n, s = 64;
#pragma unroll 1
  while (need != cnt && need != 0) {
    --s;
    const unsigned long long half = P << 1;  // prefix with bit s = 0
    int c0 = 0;
#pragma unroll
    for (int j = 0; j < NE; ++j) c0 += __popcll(__ballot(v[j] && (e[j] >> s) == half));
    if (c0 >= need) {
      P = half;
      cnt = c0;
    } else {
      P = half | 1ull;
      need -= c0;
      cnt -= c0;
    }
  }
  // kept: top bits below P, and those equal to P when all of the shared group is taken
  const unsigned long long lim = need ? P + 1ull : P;  // keep (e >> s) < lim  (s < 64: one round ran)
  const unsigned long long lt = (1ull << lane) - 1ull;
  int pos = 0;
  uint32_t worst = 0;  // largest kept high word (~okey): the K-th best score
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const bool keep = v[j] && (e[j] >> s) < lim;
    const unsigned long long bal = __ballot(keep);
    if (keep) {
      buf[pos + __popcll(bal & lt)] = e[j];
      worst = max(worst, (uint32_t)(e[j] >> 32));
    }
    pos += __popcll(bal);
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) worst = max(worst, (uint32_t)__shfl_xor((int)worst, m));
  return ~worst;
}

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long x, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)x, m), hi = __shfl_xor((uint32_t)(x >> 32), m);
  return ((unsigned long long)hi << 32) | lo;
}

// One wave's 16 rows (DK = D / 64: embedding width 64 or 128).  STAGED: the rows' masked items sit in
// the wave's LDS slice (a mask lookup is an LDS read); otherwise (more than ST_MSTAGE masked items in
// the 16 rows) they are read from global memory, which also waits for the item prefetch in flight.
// X6: scores on the bf16 matrix cores from exact three-way splits (v_mfma_f32_16x16x32_bf16, the six
// products hi*hi + hi*mid + mid*hi + hi*lo + lo*hi + mid*mid of gemm_x6.hip: fp32-accurate sums, 2.7x
// the fp32 MFMA rate); the item table arrives as three bf16 planes (gmr_split3_planes), the user rows
// are split in registers once (fa).  I / ldi then address plane 0 in bf16 elements, ps = plane stride.
template <int DK, bool STAGED, bool X6>
__device__ __forceinline__ void score_topk_wave(int64_t n_rows, int64_t row0, int lane, const float (&a)[16 * DK],
                                                const bf16x8 (&fa)[3][2 * DK], int ps,
                                                int64_t n_items, const void* __restrict__ I, int64_t ldi,
                                                const int64_t* __restrict__ mptr, const int* __restrict__ mcols,
                                                const int* ms, int64_t mbase, float fill, int K,
                                                unsigned long long (*cb)[ST_CAP], int* cn) {
  constexpr int KS = 16 * DK;
  constexpr int ST_T = X6 ? ST_TILES_X6 : ST_TILES, ST_STEP = 16 * ST_T;
  const int col = lane & 15, grp = lane >> 4;
  auto mask_at = [&](int64_t i) -> int { return STAGED ? ms[i - mbase] : mcols[i]; };
  // the lane's output rows are row0 + 4 grp + e (MFMA C/D map: row = 4 (lane >> 4) + reg, col = lane & 15)
  int64_t mc[4], me[4];
  int nm[4];
  float tau[4];  // per row: the k-th best score so far (NaN until the first compaction: every item enters)
  int cnt[4];  // entries in the buffers of the lane's rows (the same in the 16 lanes of a row group)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t r = row0 + 4 * grp + e;
    mc[e] = r < n_rows ? mptr[r] : 0;
    me[e] = r < n_rows ? mptr[r + 1] : 0;
    nm[e] = mc[e] < me[e] ? mask_at(mc[e]) : 0x7fffffff;
    // NaN, not -inf: !(s <= NaN) admits every item, a -inf score (a caller's -inf fill) included, until
    // the first compaction has k entries and sets tau to the k-th of them
    tau[e] = __builtin_nanf("");
    cnt[e] = 0;
  }
  // items [c0, c0 + 64): this lane's 16 consecutive k of item c0 + 16 t + col (clamped: the loads of
  // a step past the end are issued anyway, so no branch splits the prefetch from its use; 32-bit
  // offsets, n_items * ldi < 2^31 is checked by the host)
  const int nlast = (int)n_items - 1, ld32 = (int)ldi;
  // B registers of one step: fp32 [tile][KS] or bf16 [tile][plane][KS / 8 chunks of 8]
  using BRegs = std::conditional_t<X6, bf16x8[ST_T][3][KS / 8], float[ST_T][KS]>;
  auto load_b = [&](int c0, BRegs& bb) {
#pragma unroll
    for (int t = 0; t < ST_T; ++t) {
      const int item = min(c0 + 16 * t + col, nlast);
      if constexpr (X6) {
        const __bf16* p = reinterpret_cast<const __bf16*>(I) + item * ld32 + KS * grp;
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
          for (int c = 0; c < KS / 8; ++c) bb[t][q][c] = *reinterpret_cast<const bf16x8*>(p + q * ps + 8 * c);
      } else {
        const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(I) + KS * grp + item * ld32);
#pragma unroll
        for (int q = 0; q < KS / 4; ++q) {
          const float4 x = p[q];
          bb[t][4 * q] = x.x;
          bb[t][4 * q + 1] = x.y;
          bb[t][4 * q + 2] = x.z;
          bb[t][4 * q + 3] = x.w;
        }
      }
    }
  };
  auto mfma = [&](const BRegs& b, f32x4 (&acc)[ST_T]) {
#pragma unroll
    for (int t = 0; t < ST_T; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (X6) {
#pragma unroll
      for (int c = 0; c < KS / 8; ++c)
#pragma unroll
        for (int t = 0; t < ST_T; ++t) {  // small terms first (gemm_x6.hip's order)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1][c], b[t][1][c], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][c], b[t][2][c], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2][c], b[t][0][c], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][c], b[t][1][c], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1][c], b[t][0][c], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][c], b[t][0][c], acc[t], 0, 0, 0);
        }
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int t = 0; t < ST_T; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[t][s], acc[t], 0, 0, 0);
    }
  };
  // train positives of the lane's rows inside [c0, c0 + 64) -> fill (a wave-uniform test; the loop
  // runs only in the rare steps that hold one)
  auto mask_fix = [&](int c0, f32x4 (&acc)[ST_T]) {
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
          for (int t = 0; t < ST_T; ++t)
            if (t == (d >> 4)) acc[t][e] = fill;
        }
        ++mc[e];
        nm[e] = mc[e] < me[e] ? mask_at(mc[e]) : 0x7fffffff;
      }
    }
  };
  // candidates of one tile: per row a ballot of the lanes whose score beats the row's threshold
  // (!(s <= tau): a NaN score enters, as torch.topk ranks NaN first); a tile none of whose 64 scores
  // beats its row's threshold costs four compares and a scalar branch, the common case once the
  // thresholds have risen.  A row's entrants get consecutive slots from the ballot over the 16 lanes of
  // its group.  Keys are built from s + 0 (-0 -> +0: equal scores compare equal, ties -> lowest item).
  const uint32_t below = (1u << col) - 1u;
  // a row near its capacity (one tile adds at most 16): keep its k best, raise its threshold
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
          tau[e] = okey_inv(nt);
          cnt[e] = K;
        }
      }
    }
  };
  auto filter = [&](int c0, const f32x4 (&acc)[ST_T]) {
#pragma unroll
    for (int t = 0; t < ST_T; ++t) {
      const int c = c0 + 16 * t + col;
      const bool valid = c < n_items;
      unsigned long long m[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = __ballot(valid && !(acc[t][e] <= tau[e]));
      if ((m[0] | m[1] | m[2] | m[3]) == 0) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (m[e] == 0) continue;
        const uint32_t g = (uint32_t)(m[e] >> (16 * grp)) & 0xffffu;
        if ((g >> col) & 1u)
          cb[4 * grp + e][cnt[e] + __popc(g & below)] =
              ((unsigned long long)(~okey(acc[t][e] + 0.0f)) << 32) | (uint32_t)c;
        cnt[e] += __popc(g);
      }
      compact_check();
    }
  };
  // software pipeline: the MFMAs of step j + 1 are issued before the filter of step j (independent
  // registers: the matrix pipe runs while the vector pipe filters); two item register sets and two
  // accumulator sets, the loads of step j + 2 in flight meanwhile
  BRegs b0, b1;
  f32x4 acc0[ST_T], acc1[ST_T];
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

template <int DK, bool X6>
__global__ void __launch_bounds__(64 * ST_WAVES, DK == 1 ? 2 : 1) score_topk_kernel(
    int64_t n_rows, const int* __restrict__ users, const float* __restrict__ U, int64_t ldu, int64_t n_items,
    const void* __restrict__ I, int64_t ldi, int ps, const int64_t* __restrict__ mptr, const int* __restrict__ mcols,
    float fill, int K, int* __restrict__ out_idx, int64_t ld_idx, float* __restrict__ out_val) {
  __shared__ unsigned long long cand[ST_WAVES][ST_ROWS][ST_CAP];
  __shared__ int cnt[ST_WAVES][ST_ROWS];
  __shared__ int mstage[ST_WAVES][ST_MSTAGE];
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
  bf16x8 fa[3][2 * DK];  // X6: the three planes of a, 8 k per chunk
  if constexpr (X6) {
#pragma unroll
    for (int c = 0; c < 2 * DK; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        __bf16 h, m, l;
        st_split3(a[8 * c + e], h, m, l);
        fa[0][c][e] = h;
        fa[1][c][e] = m;
        fa[2][c][e] = l;
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
    score_topk_wave<DK, true, X6>(n_rows, row0, lane, a, fa, ps, n_items, I, ldi, mptr, mcols, mstage[w], mbase, fill,
                                  K, cb, cn);
  } else {
    score_topk_wave<DK, false, X6>(n_rows, row0, lane, a, fa, ps, n_items, I, ldi, mptr, mcols, mstage[w], mbase,
                                   fill, K, cb, cn);
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

static int score_topk_check(int64_t n_rows, const void* user_table, int64_t ld_user, int64_t n_items,
                            const void* item_table, int64_t dim, const int64_t* mask_ptr, const int32_t* mask_cols,
                            int32_t k, const int32_t* out_idx, int64_t ld_idx) {
  GMR_ARG(user_table && item_table && out_idx && n_rows > 0 && n_items > 0, "bad args");
  GMR_ARG(mask_ptr && mask_cols, "mask_ptr / mask_cols required (an empty mask: mask_ptr all zero)");
  GMR_ARG(k >= 1 && k <= 64 && k <= n_items, "k must be in [1, min(64, n_items)]");
  GMR_ARG(n_items < (1ll << 31) - 64 && ld_idx >= k, "bad sizes");
  GMR_ARG(ld_user % 4 == 0 && ld_user >= dim, "user leading dim: a multiple of 4, >= dim");
  GMR_ARG(((uintptr_t)user_table | (uintptr_t)item_table) % 16 == 0, "tables must be 16-byte aligned");
  return GMR_OK;
}

extern "C" int gmr_score_topk_f32(int64_t n_rows, const int32_t* users, const float* user_table, int64_t ld_user,
                                  int64_t n_items, const float* item_table, int64_t ld_item, int64_t dim,
                                  const int64_t* mask_ptr, const int32_t* mask_cols, float fill, int32_t k,
                                  int32_t* out_idx, int64_t ld_idx, float* out_val, void* stream) {
  GMR_ARG(dim == 64 || dim == 128, "embedding width must be 64 or 128");
  if (score_topk_check(n_rows, user_table, ld_user, n_items, item_table, dim, mask_ptr, mask_cols, k, out_idx,
                       ld_idx) != GMR_OK)
    return GMR_ERR_ARG;
  GMR_ARG(n_items * ld_item < (1ll << 31), "item table too large for 32-bit offsets");
  GMR_ARG(ld_item % 4 == 0 && ld_item >= dim, "item leading dim: a multiple of 4, >= dim");
  const int64_t waves = (n_rows + ST_ROWS - 1) / ST_ROWS;
  const dim3 grid((unsigned)((waves + ST_WAVES - 1) / ST_WAVES));
  if (dim == 64)
    hipLaunchKernelGGL((score_topk_kernel<1, false>), grid, dim3(64 * ST_WAVES), 0, (hipStream_t)stream, n_rows, users,
                       user_table, ld_user, n_items, item_table, ld_item, 0, mask_ptr, mask_cols, fill, k, out_idx,
                       ld_idx, out_val);
  else
    hipLaunchKernelGGL((score_topk_kernel<2, false>), grid, dim3(64 * ST_WAVES), 0, (hipStream_t)stream, n_rows, users,
                       user_table, ld_user, n_items, item_table, ld_item, 0, mask_ptr, mask_cols, fill, k, out_idx,
                       ld_idx, out_val);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_score_topk_x6(int64_t n_rows, const int32_t* users, const float* user_table, int64_t ld_user,
                                 int64_t n_items, const uint16_t* item_planes, int64_t ld_plane, int64_t plane_stride,
                                 int64_t dim, const int64_t* mask_ptr, const int32_t* mask_cols, float fill, int32_t k,
                                 int32_t* out_idx, int64_t ld_idx, float* out_val, void* stream) {
  GMR_ARG(dim == 64, "split-bf16 scoring: embedding width 64");
  if (score_topk_check(n_rows, user_table, ld_user, n_items, item_planes, dim, mask_ptr, mask_cols, k, out_idx,
                       ld_idx) != GMR_OK)
    return GMR_ERR_ARG;
  GMR_ARG(ld_plane % 8 == 0 && ld_plane >= dim && plane_stride % 8 == 0 && plane_stride >= n_items * ld_plane,
          "planes: leading dim a multiple of 8 and >= dim, plane stride a multiple of 8 holding every row");
  GMR_ARG(3 * plane_stride < (1ll << 31), "item planes too large for 32-bit offsets");
  const int64_t waves = (n_rows + ST_ROWS - 1) / ST_ROWS;
  const dim3 grid((unsigned)((waves + ST_WAVES - 1) / ST_WAVES));
  hipLaunchKernelGGL((score_topk_kernel<1, true>), grid, dim3(64 * ST_WAVES), 0, (hipStream_t)stream, n_rows, users,
                     user_table, ld_user, n_items, item_planes, ld_plane, (int)plane_stride, mask_ptr, mask_cols, fill,
                     k, out_idx, ld_idx, out_val);
  GMR_LAUNCHED();
  return GMR_OK;
}
