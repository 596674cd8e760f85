// GenRecV1 graph builders and host-stage replacements:
//   * CSR transpose (backward of the non-symmetric SpMMs: the dropped UI graph, kNN II graphs, R)
//   * SpAdjDropEdge (models/genrecv1.py:443-457) as a CSR compaction
//   * kNN item-item graph with 'sym' normalisation (common/trainer.py:682-687, utils/utils.py:152-197)
//   * InterestDebiase (common/interest_cluster.py:157-383): exact-n uniform picks + cluster rules
//   * K-means (common/interest_cluster.py:60-79, sklearn KMeans): StandardScaler, k-means++ seeding,
//     Lloyd steps whose distance and centroid products run on the MFMA GEMM.
// All outputs are deterministic functions of the inputs and the Philox (seed, step) stream.
#include "gmr_common.h"

namespace {

// exclusive scan of n ints (single workgroup: chunked serial sums + LDS Hillis-Steele)
__global__ void __launch_bounds__(1024) scan_kernel(int64_t n, const int* __restrict__ cnt, int* __restrict__ out) {
  __shared__ int s[1024];
  const int t = threadIdx.x;
  const int64_t chunk = (n + 1023) / 1024;
  const int64_t r0 = t * chunk, r1 = r0 + chunk < n ? r0 + chunk : n;
  int sum = 0;
  for (int64_t r = r0; r < r1; ++r) sum += cnt[r];
  s[t] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = t >= off ? s[t - off] : 0;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  int o = s[t] - sum;
  for (int64_t r = r0; r < r1; ++r) {
    out[r] = o;
    o += cnt[r];
  }
  if (t == 1023) out[n] = s[1023];
}

// ----------------------------------------------------------------- CSR transpose
__global__ void count_cols_kernel(int64_t nnz, const int* __restrict__ col, int* __restrict__ cnt) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nnz) atomicAdd(&cnt[col[e]], 1);
}

__global__ void scatter_t_kernel(int n_rows, const int* __restrict__ rowptr, const int* __restrict__ col,
                                 const float* __restrict__ val, const int* __restrict__ trp, int* __restrict__ fill,
                                 int* __restrict__ tcol, float* __restrict__ tval) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  for (int e = rowptr[r]; e < rowptr[r + 1]; ++e) {
    const int c = col[e];
    const int o = trp[c] + atomicAdd(&fill[c], 1);
    tcol[o] = r;
    tval[o] = val[e];
  }
}

constexpr int kT = 256;

// one workgroup per transposed row: order entries by source row (distinct keys, values carried);
// long rows: rank by bitmap prefix into a staging copy, then copy back (two passes, no aliasing)
__global__ void __launch_bounds__(kT) place_t_rows_kernel(int n_src, const int* __restrict__ trp,
                                                          const int* __restrict__ tcol_in,
                                                          const float* __restrict__ tval_in, int* __restrict__ tcol,
                                                          float* __restrict__ tval) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ int s_part[kT];
  const int i = blockIdx.x, t = threadIdx.x;
  const int beg = trp[i], L = trp[i + 1] - beg;
  if (L <= kT) {
    if (L == 1 && t == 0) {
      tcol[beg] = tcol_in[beg];
      tval[beg] = tval_in[beg];
    }
    if (L <= 1) return;
    int k = 0;
    float v = 0.f;
    __shared__ int s_key[kT];
    if (t < L) {
      k = tcol_in[beg + t];
      v = tval_in[beg + t];
    }
    s_key[t] = t < L ? k : 0x7fffffff;
    __syncthreads();
    if (t < L) {
      int r = 0;
      for (int j = 0; j < L; ++j) r += s_key[j] < k;
      tcol[beg + r] = k;
      tval[beg + r] = v;
    }
    return;
  }
  const int W = (n_src + 31) >> 5;
  uint32_t* bits = lds;
  int* pre = reinterpret_cast<int*>(lds + W);
  for (int w = t; w < W; w += kT) bits[w] = 0u;
  __syncthreads();
  for (int e = t; e < L; e += kT) {
    const int k = tcol_in[beg + e];
    atomicOr(&bits[k >> 5], 1u << (k & 31));
  }
  __syncthreads();
  const int per = (W + kT - 1) / kT;
  const int w0 = min(W, t * per), w1 = min(W, w0 + per);
  int cnt = 0;
  for (int w = w0; w < w1; ++w) cnt += __popc(bits[w]);
  s_part[t] = cnt;
  __syncthreads();
  for (int off = 1; off < kT; off <<= 1) {
    const int a = t >= off ? s_part[t - off] : 0;
    __syncthreads();
    s_part[t] += a;
    __syncthreads();
  }
  int o = s_part[t] - cnt;
  for (int w = w0; w < w1; ++w) {
    pre[w] = o;
    o += __popc(bits[w]);
  }
  __syncthreads();
  for (int e = t; e < L; e += kT) {
    const int k = tcol_in[beg + e];
    const int rank = pre[k >> 5] + __popc(bits[k >> 5] & ((1u << (k & 31)) - 1u));
    tcol[beg + rank] = k;
    tval[beg + rank] = tval_in[beg + e];
  }
}

// ----------------------------------------------------------------- SpAdjDropEdge
// keep entry e iff floor(u + keep_rate) >= 1 (u = uniform draw) — or keep[e] when given
__device__ __forceinline__ bool edge_kept(int64_t e, const uint8_t* keep, float keep_rate, uint64_t seed,
                                          uint64_t step) {
  if (keep) return keep[e] != 0;
  const uint4 r = gmr::Philox::gen(seed, step, (uint64_t)e);
  const float u = (float)(r.x >> 8) * (1.0f / 16777216.0f);  // [0, 1)
  return floorf(u + keep_rate) >= 1.f;
}

// position of column c in row r (columns ascending; present by symmetry)
__device__ __forceinline__ int find_in_row(const int* __restrict__ rowptr, const int* __restrict__ col, int r, int c) {
  int lo = rowptr[r], hi = rowptr[r + 1] - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (col[mid] < c) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// keep flag of entry e = (r, c); transposed: the flag of (c, r) of a structurally symmetric matrix,
// so the result is (A with its entries dropped)^T built directly from A
__device__ __forceinline__ bool kept_entry(int r, int e, const int* __restrict__ rowptr, const int* __restrict__ col,
                                           int transposed, const uint8_t* keep, float keep_rate, uint64_t seed,
                                           uint64_t step) {
  const int src = transposed ? find_in_row(rowptr, col, col[e], r) : e;
  return edge_kept(src, keep, keep_rate, seed, step);
}

// one wave per row: ballot of the kept entries
__global__ void __launch_bounds__(256) drop_count_kernel(int n_rows, const int* __restrict__ rowptr,
                                                         const int* __restrict__ col, int transposed,
                                                         const uint8_t* __restrict__ keep, float keep_rate,
                                                         uint64_t seed, uint64_t step, int* __restrict__ cnt) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n_rows) return;
  const int lane = threadIdx.x & 63;
  int c = 0;
  for (int e0 = rowptr[r]; e0 < rowptr[r + 1]; e0 += 64) {
    const int e = e0 + lane;
    const bool k = e < rowptr[r + 1] && kept_entry(r, e, rowptr, col, transposed, keep, keep_rate, seed, step);
    c += __popcll(__ballot(k));
  }
  if (lane == 0) cnt[r] = c;
}

__global__ void __launch_bounds__(256) drop_write_kernel(int n_rows, const int* __restrict__ rowptr,
                                                         const int* __restrict__ col, const float* __restrict__ val,
                                                         int transposed, const uint8_t* __restrict__ keep,
                                                         float keep_rate, uint64_t seed, uint64_t step,
                                                         const int* __restrict__ orp, int* __restrict__ ocol,
                                                         float* __restrict__ oval) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n_rows) return;
  const int lane = threadIdx.x & 63;
  int o = orp[r];
  for (int e0 = rowptr[r]; e0 < rowptr[r + 1]; e0 += 64) {
    const int e = e0 + lane;
    const bool k = e < rowptr[r + 1] && kept_entry(r, e, rowptr, col, transposed, keep, keep_rate, seed, step);
    const unsigned long long m = __ballot(k);
    if (k) {
      const int pos = o + __popcll(m & ((1ull << lane) - 1ull));
      const int src = transposed ? find_in_row(rowptr, col, col[e], r) : e;
      ocol[pos] = col[e];
      oval[pos] = val[src] / keep_rate;
    }
    o += __popcll(m);
  }
}

// ----------------------------------------------------------------- kNN graph ('sym')
// deg[r] = sum of the row's k kept similarities in top-k order (fp32, like index_add_)
__global__ void knn_deg_kernel(int n, int k, const float* __restrict__ tv, int64_t ldv, float* __restrict__ dis) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  float d = 0.f;
  for (int j = 0; j < k; ++j) d = __fadd_rn(d, tv[(int64_t)r * ldv + j]);
  float x = powf(d, -0.5f);
  if (isinf(x)) x = 0.f;
  dis[r] = x;
}

// row r: columns ascending (insertion sort of the k picks), w = d_r * v * d_c
__global__ void knn_csr_kernel(int n, int k, const int* __restrict__ ti, int64_t ldi, const float* __restrict__ tv,
                               int64_t ldv, const float* __restrict__ dis, int* __restrict__ rowptr,
                               int* __restrict__ col, float* __restrict__ val) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > n) return;
  rowptr[r] = r * k;
  if (r == n) return;
  int cs[64];
  float vs[64];
  for (int j = 0; j < k; ++j) {
    const int c = ti[(int64_t)r * ldi + j];
    const float v = tv[(int64_t)r * ldv + j];
    int p = j;
    while (p > 0 && cs[p - 1] > c) {
      cs[p] = cs[p - 1];
      vs[p] = vs[p - 1];
      --p;
    }
    cs[p] = c;
    vs[p] = v;
  }
  const float dr = dis[r];
  for (int j = 0; j < k; ++j) {
    col[(int64_t)r * k + j] = cs[j];
    val[(int64_t)r * k + j] = __fmul_rn(__fmul_rn(dr, vs[j]), dis[cs[j]]);
  }
}

// ----------------------------------------------------------------- InterestDebiase
// Candidates: the gen_topk positions of each row where p_sample flipped the history bit
// (only those positions of `denoised` can differ from x0, trainer.py:752-754).  type 0 = 0->1
// ("dislike_to_like"), 1 = 1->0.  Exactly n_t = int(count_t * ratio) of each type are picked
// uniformly (random.sample, interest_cluster.py:234-243): smallest n_t of a Philox key per
// candidate (64-bit: 32 random bits << 32 | candidate index, so keys are distinct), by an 8-pass
// LDS radix select in one workgroup.
constexpr int kSel = 1024;
__device__ __forceinline__ int cand_type(const float* x0, const float* xs, int64_t ld, int b, int i) {
  const float a = x0[(int64_t)b * ld + i], g = xs[(int64_t)b * ld + i];
  if (a == 0.f && g == 1.f) return 0;
  if (a == 1.f && g == 0.f) return 1;
  return -1;
}

// candidate keys: UINT64_MAX unless position j (row j / k, pick j % k) flipped with the given type
__global__ void debias_keys_kernel(int B, int k, const int* __restrict__ topi, int64_t ldt, const float* __restrict__ x0,
                                   const float* __restrict__ xs, int64_t ld, uint64_t seed, uint64_t step,
                                   unsigned long long* __restrict__ keys) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B * k) return;
  const int b = j / k, i = topi[(int64_t)b * ldt + j % k];
  const int ty = cand_type(x0, xs, ld, b, i);
  for (int type = 0; type < 2; ++type) {
    unsigned long long key = ~0ull;
    if (ty == type) {
      const uint4 r = gmr::Philox::gen(seed, step * 2 + type, (uint64_t)j);
      key = ((unsigned long long)r.x << 32) | (unsigned)j;
    }
    keys[(int64_t)type * B * k + j] = key;
  }
}

__global__ void __launch_bounds__(kSel) debias_select_kernel(int B, int k, const int* __restrict__ topi, int64_t ldt,
                                                             const unsigned long long* __restrict__ keys, float ratio,
                                                             int* __restrict__ picks, int max_picks,
                                                             int* __restrict__ n_picks) {
  __shared__ int hist[256];
  __shared__ int s_cnt;
  __shared__ int s_out;
  __shared__ unsigned long long s_prefix;
  __shared__ int s_need;
  const int t = threadIdx.x;
  const int n = B * k;
  for (int type = 0; type < 2; ++type) {
    const unsigned long long* kk = keys + (int64_t)type * n;
    if (t == 0) s_cnt = 0;
    __syncthreads();
    int c = 0;
    for (int j = t; j < n; j += kSel) c += kk[j] != ~0ull;
    atomicAdd(&s_cnt, c);
    __syncthreads();
    const int total = s_cnt;
    const int need = (int)((float)total * ratio);
    // radix select of the need-th smallest key among this type's candidates (keys are distinct)
    unsigned long long prefix = 0ull;
    int remaining = need;
    if (need > 0) {
      for (int pass = 7; pass >= 0; --pass) {
        for (int h = t; h < 256; h += kSel) hist[h] = 0;
        __syncthreads();
        const unsigned long long hi_mask = pass == 7 ? 0ull : (~0ull << (8 * (pass + 1)));
        for (int j = t; j < n; j += kSel) {
          const unsigned long long key = kk[j];
          if (key == ~0ull || (key & hi_mask) != prefix) continue;
          atomicAdd(&hist[(key >> (8 * pass)) & 255], 1);
        }
        __syncthreads();
        if (t == 0) {
          int acc = 0, d = 0;
          for (; d < 256; ++d) {
            if (acc + hist[d] >= remaining) break;
            acc += hist[d];
          }
          s_prefix = prefix | ((unsigned long long)d << (8 * pass));
          s_need = remaining - acc;
        }
        __syncthreads();
        prefix = s_prefix;
        remaining = s_need;
        __syncthreads();
      }
    }
    if (t == 0) s_out = 0;
    __syncthreads();
    if (need > 0)
      for (int j = t; j < n; j += kSel) {
        const unsigned long long key = kk[j];
        if (key != ~0ull && key <= prefix) {
          const int o = atomicAdd(&s_out, 1);
          if (o < max_picks) {
            picks[(type * max_picks + o) * 2] = j / k;
            picks[(type * max_picks + o) * 2 + 1] = topi[(int64_t)(j / k) * ldt + j % k];
          }
        }
      }
    __syncthreads();
    if (t == 0) n_picks[type] = min(s_out, max_picks);
    __syncthreads();
  }
}

// One wave per pick: the row's history cluster counts (labels < 64) decide the new bit.
// type 0 (0->1): 1 iff count[label[i]] > 0.  type 1 (1->0): 0 iff count[label[i]] <= min + 1,
// min over the clusters present in the history (interest_cluster.py:256-331; the image labels
// serve every modality, :258-267).
__global__ void __launch_bounds__(256) debias_apply_kernel(int type, const int* __restrict__ picks,
                                                           const int* __restrict__ n_picks, int npick_const,
                                                           const float* __restrict__ x0, int64_t ld0, int I,
                                                           const int* __restrict__ labels, float* __restrict__ den,
                                                           int64_t ldd) {
  __shared__ int cnt[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int np = n_picks ? n_picks[type] : npick_const;
  const int p = blockIdx.x * 4 + w;
  cnt[w][lane] = 0;
  __syncthreads();
  if (p >= np) return;
  const int b = picks[2 * p], i = picks[2 * p + 1];
  for (int j = lane; j < I; j += 64)
    if (x0[(int64_t)b * ld0 + j] > 0.f) atomicAdd(&cnt[w][labels[j]], 1);
  __syncthreads();
  if (lane != 0) return;
  const int cur = cnt[w][labels[i]];
  float v;
  if (type == 0) {
    v = cur > 0 ? 1.f : 0.f;
  } else {
    int mn = 0x7fffffff;
    for (int c = 0; c < 64; ++c)
      if (cnt[w][c] > 0 && cnt[w][c] < mn) mn = cnt[w][c];
    if (mn == 0x7fffffff) mn = 0;
    v = cur <= mn + 1 ? 0.f : 1.f;
  }
  den[(int64_t)b * ldd + i] = v;
}

// den = x0 except at the row's gen_topk positions, where it takes the p_sample outcome; score = den * probs
__global__ void gen_mask_kernel(int B, int I, int k, const int* __restrict__ topi, int64_t ldt,
                                const float* __restrict__ x0, const float* __restrict__ xs, int64_t ld,
                                float* __restrict__ den) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)B * I) return;
  const int b = (int)(gid / I), i = (int)(gid % I);
  bool m = false;
  for (int j = 0; j < k; ++j) m |= topi[(int64_t)b * ldt + j] == i;
  den[(int64_t)b * ld + i] = m ? xs[(int64_t)b * ld + i] : x0[(int64_t)b * ld + i];
}

// ----------------------------------------------------------------- K-means
// column mean / population std of X (n x d) -> scaled copy (sklearn StandardScaler; std 0 -> 1)
__global__ void __launch_bounds__(256) colstats_kernel(int64_t n, int d, const float* __restrict__ X, int64_t ldx,
                                                       float* __restrict__ mean, float* __restrict__ scale) {
  const int c = blockIdx.x;
  __shared__ double rs[4], rq[4];
  double s = 0.0, q = 0.0;
  for (int64_t r = threadIdx.x; r < n; r += 256) {
    const double v = X[r * ldx + c];
    s += v;
    q += v * v;
  }
  s = gmr::wave_sum_d(s);
  q = gmr::wave_sum_d(q);
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rq[threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double S = (rs[0] + rs[1]) + (rs[2] + rs[3]), Q = (rq[0] + rq[1]) + (rq[2] + rq[3]);
    const double mu = S / (double)n;
    double var = Q / (double)n - mu * mu;
    if (var < 0) var = 0;
    const double sd = sqrt(var);
    mean[c] = (float)mu;
    scale[c] = sd < 1e-300 ? 1.f : (float)sd;
  }
}

__global__ void standardize_kernel(int64_t n, int d, const float* __restrict__ X, int64_t ldx,
                                   const float* __restrict__ mean, const float* __restrict__ scale,
                                   float* __restrict__ Y, int64_t ldy, float* __restrict__ sq) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  float s = 0.f;
  for (int c = threadIdx.x; c < d; c += 256) {
    const float v = (X[r * ldx + c] - mean[c]) / scale[c];
    Y[r * ldy + c] = v;
    s += v * v;
  }
  __shared__ float red[4];
  s = gmr::wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) sq[r] = (red[0] + red[1]) + (red[2] + red[3]);
}

// squared distance of every point to centroid j (given the point norms and the dot column)
__global__ void min_dist_update_kernel(int64_t n, const float* __restrict__ xsq, const float* __restrict__ dots,
                                       int64_t ldd, const float* __restrict__ csq, int j, float* __restrict__ mind,
                                       int first) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const float d = fmaxf(xsq[r] - 2.f * dots[r * ldd] + csq[j], 0.f);
  mind[r] = first ? d : fminf(mind[r], d);
}

// sum of the 1,024 per-thread partials, by wave 0 in a fixed order (16 consecutive partials per lane, then a
// shuffle tree): the result in lane 0 (the serial 1,024-step sum of one thread was most of the launch)
__device__ __forceinline__ double kpp_wave_total(const double* part, int lane) {
  double v = 0.0;
#pragma unroll
  for (int q = 0; q < 16; ++q) v += part[lane * 16 + q];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
  return v;
}

// k-means++ pick: one workgroup; point chosen with probability mind[r] / sum (Philox draw).  Wave 0 scans the
// 64 group sums of 16 partials (shuffle scan, fixed order), a ballot finds the group holding u, one lane walks
// its <= 16 partials and then the <= chunk points of the partial
__global__ void __launch_bounds__(1024) kpp_pick_kernel(int64_t n, const float* __restrict__ mind, uint64_t seed,
                                                        uint64_t step, int* __restrict__ out) {
  __shared__ double part[1024];
  const int t = threadIdx.x;
  const int64_t chunk = (n + 1023) / 1024;
  const int64_t r0 = t * chunk, r1 = r0 + chunk < n ? r0 + chunk : n;
  double s = 0.0;
  for (int64_t r = r0; r < r1; ++r) s += mind ? (double)mind[r] : 1.0;
  part[t] = s;
  __syncthreads();
  if (t >= 64) return;
  double g = 0.0;
#pragma unroll
  for (int q = 0; q < 16; ++q) g += part[t * 16 + q];
  double inc = g;  // inclusive scan over the 64 groups
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const double o = __shfl_up(inc, off);
    if (t >= off) inc += o;
  }
  const double tot = __shfl(inc, 63);
  const uint4 rr = gmr::Philox::gen(seed, step, 0);
  const double u = ((double)rr.x + (double)rr.y * 4294967296.0) / 18446744073709551616.0 * tot;
  const unsigned long long bal = __ballot(inc > u);
  const int grp = bal ? __ffsll(bal) - 1 : 63;  // no group above u (rounding, or every mind 0): the last
  if (t != grp) return;
  double acc = inc - g;
  int j = grp * 16;
  for (; j < grp * 16 + 15 && acc + part[j] <= u; ++j) acc += part[j];
  const int64_t a = j * chunk, e = a + chunk < n ? a + chunk : n;
  int64_t pick = a < n ? a : n - 1;
  for (int64_t r = a; r < e; ++r) {
    const double m = mind ? (double)mind[r] : 1.0;
    pick = r;
    if (acc + m > u && m > 0) break;
    acc += m;
  }
  out[0] = (int)pick;
}

// greedy k-means++ step (sklearn's _kmeans_plusplus with n_local_trials candidates, KMeans' default seeding):
// the potential sum_r min(mind[r], |x_r - c_t|^2) of each candidate t (dots = X . Cc^T, fixed-order sums),
// the candidate of the lowest potential (ties -> lowest t) becomes center j and updates mind
__global__ void __launch_bounds__(1024) kpp_greedy_kernel(int64_t n, int L, const float* __restrict__ xsq,
                                                          const float* __restrict__ dots, int64_t ldd,
                                                          const float* __restrict__ ccsq, float* __restrict__ mind,
                                                          const float* __restrict__ Cc, int64_t ldcc, int d,
                                                          float* __restrict__ C, int64_t ldc, int j,
                                                          float* __restrict__ csq) {
  __shared__ double part[1024];
  __shared__ double pot[16];
  __shared__ int best_s;
  const int t0 = threadIdx.x;
  const int64_t chunk = (n + 1023) / 1024;
  const int64_t r0 = t0 * chunk, r1 = r0 + chunk < n ? r0 + chunk : n;
  for (int t = 0; t < L; ++t) {
    double s = 0.0;
    for (int64_t r = r0; r < r1; ++r) {
      const float dd = fmaxf(xsq[r] - 2.f * dots[r * ldd + t] + ccsq[t], 0.f);
      s += (double)fminf(mind[r], dd);
    }
    part[t0] = s;
    __syncthreads();
    if (t0 < 64) {
      const double tot = kpp_wave_total(part, t0);
      if (t0 == 0) pot[t] = tot;
    }
    __syncthreads();
  }
  if (t0 == 0) {
    int b = 0;
    for (int t = 1; t < L; ++t)
      if (pot[t] < pot[b]) b = t;
    best_s = b;
  }
  __syncthreads();
  const int b = best_s;
  for (int64_t r = t0; r < n; r += 1024) {
    const float dd = fmaxf(xsq[r] - 2.f * dots[r * ldd + b] + ccsq[b], 0.f);
    mind[r] = fminf(mind[r], dd);
  }
  for (int c = t0; c < d; c += 1024) C[(int64_t)j * ldc + c] = Cc[(int64_t)b * ldcc + c];
  if (t0 == 0) csq[j] = ccsq[b];
}

__global__ void copy_row_kernel(int d, const float* __restrict__ X, int64_t ldx, const int* __restrict__ idx,
                                float* __restrict__ C, int64_t ldc, int j, const float* __restrict__ xsq,
                                float* __restrict__ csq) {
  const int r = idx[0];
  for (int c = threadIdx.x; c < d; c += blockDim.x) C[(int64_t)j * ldc + c] = X[(int64_t)r * ldx + c];
  if (threadIdx.x == 0) csq[j] = xsq[r];
}

// label[r] = argmin_j (csq[j] - 2 dots[r, j]) (ties -> lowest j); one-hot^T rows; changed count
__global__ void assign_kernel(int64_t n, int k, const float* __restrict__ dots, int64_t ldd,
                              const float* __restrict__ csq, const float* __restrict__ xsq, int* __restrict__ label,
                              float* __restrict__ onehot_t, int64_t ldo, int* __restrict__ changed,
                              double* __restrict__ inertia_parts) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double in = 0.0;
  if (r < n) {
    int best = 0;
    float bd = csq[0] - 2.f * dots[r * ldd];
    for (int j = 1; j < k; ++j) {
      const float d = csq[j] - 2.f * dots[r * ldd + j];
      if (d < bd) {
        bd = d;
        best = j;
      }
    }
    if (label[r] != best) atomicAdd(changed, 1);
    label[r] = best;
    for (int j = 0; j < k; ++j) onehot_t[(int64_t)j * ldo + r] = j == best ? 1.f : 0.f;
    in = fmax(0.0, (double)xsq[r] + (double)bd);
  }
  in = gmr::wave_sum_d(in);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = in;
  __syncthreads();
  if (threadIdx.x == 0) inertia_parts[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// centroids = sums / counts (empty clusters keep their previous centroid); csq refreshed
__global__ void centroid_kernel(int k, int d, const float* __restrict__ sums, int64_t lds,
                                const float* __restrict__ onehot_t, int64_t ldo, int64_t n, float* __restrict__ C,
                                int64_t ldc, float* __restrict__ csq) {
  const int j = blockIdx.x;
  __shared__ float s_cnt;
  __shared__ float red[4];
  float c = 0.f;
  for (int64_t r = threadIdx.x; r < n; r += 256) c += onehot_t[(int64_t)j * ldo + r];
  c = gmr::wave_sum(c);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) s_cnt = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  const float cnt = s_cnt;
  float q = 0.f;
  for (int cc = threadIdx.x; cc < d; cc += 256) {
    float v = cnt > 0.f ? sums[(int64_t)j * lds + cc] / cnt : C[(int64_t)j * ldc + cc];
    C[(int64_t)j * ldc + cc] = v;
    q += v * v;
  }
  __syncthreads();
  q = gmr::wave_sum(q);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) csq[j] = (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace

extern "C" int gmr_csr_transpose(int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t* rowptr,
                                 const int32_t* col, const float* val, int32_t* workspace, int32_t* t_rowptr,
                                 int32_t* t_col, float* t_val, int32_t* stage_col, float* stage_val, void* stream) {
  GMR_ARG(rowptr && col && val && workspace && t_rowptr && t_col && t_val && stage_col && stage_val, "null pointer");
  GMR_ARG(n_rows > 0 && n_cols > 0 && nnz >= 0 && nnz < (1ll << 31), "bad size");
  GMR_ARG(n_rows <= 262144, "n_rows above the LDS budget of the transpose row sort");
  hipStream_t st = (hipStream_t)stream;
  int* cnt = workspace;
  int* fill = workspace + n_cols;
  hipError_t e = hipMemsetAsync(workspace, 0, sizeof(int) * 2 * (size_t)n_cols, st);
  if (e != hipSuccess) return gmr::hip_status(__func__, e);
  if (nnz > 0) {
    hipLaunchKernelGGL(count_cols_kernel, dim3(gmr::grid_for(nnz, 256)), dim3(256), 0, st, nnz, col, cnt);
    GMR_LAUNCHED();
  }
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, n_cols, cnt, t_rowptr);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(scatter_t_kernel, dim3(gmr::grid_for(n_rows, 256)), dim3(256), 0, st, (int)n_rows, rowptr, col,
                     val, t_rowptr, fill, stage_col, stage_val);
  GMR_LAUNCHED();
  const int W = (int)((n_rows + 31) / 32);
  const size_t dyn = sizeof(uint32_t) * 2 * (size_t)W;
  if (dyn > 65536) {
    e = hipFuncSetAttribute((const void*)place_t_rows_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
    if (e != hipSuccess) return gmr::hip_status(__func__, e);
  }
  hipLaunchKernelGGL(place_t_rows_kernel, dim3((unsigned)n_cols), dim3(kT), dyn, st, (int)n_rows, t_rowptr, stage_col,
                     stage_val, t_col, t_val);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_csr_drop_count(int64_t n_rows, const int32_t* rowptr, const int32_t* col, int32_t transposed,
                                  const uint8_t* keep, float keep_rate, uint64_t seed, uint64_t step,
                                  int32_t* workspace, int32_t* out_rowptr, void* stream) {
  GMR_ARG(rowptr && col && workspace && out_rowptr && n_rows > 0, "bad args");
  GMR_ARG(keep_rate > 0.f && keep_rate <= 1.f, "keep_rate in (0, 1]");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(drop_count_kernel, dim3(gmr::grid_for(n_rows, 4)), dim3(256), 0, st, (int)n_rows, rowptr, col,
                     (int)transposed, keep, keep_rate, seed, step, workspace);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, st, n_rows, workspace, out_rowptr);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_csr_drop_write(int64_t n_rows, const int32_t* rowptr, const int32_t* col, const float* val,
                                  int32_t transposed, const uint8_t* keep, float keep_rate, uint64_t seed,
                                  uint64_t step, const int32_t* out_rowptr, int32_t* out_col, float* out_val,
                                  void* stream) {
  GMR_ARG(rowptr && col && val && out_rowptr && out_col && out_val && n_rows > 0, "bad args");
  hipLaunchKernelGGL(drop_write_kernel, dim3(gmr::grid_for(n_rows, 4)), dim3(256), 0, (hipStream_t)stream,
                     (int)n_rows, rowptr, col, val, (int)transposed, keep, keep_rate, seed, step, out_rowptr, out_col,
                     out_val);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_knn_symnorm_csr(int64_t n, int32_t k, const int32_t* topi, int64_t ldi, const float* topv,
                                   int64_t ldv, float* dis_ws, int32_t* rowptr, int32_t* col, float* val,
                                   void* stream) {
  GMR_ARG(topi && topv && dis_ws && rowptr && col && val && n > 0, "bad args");
  GMR_ARG(k >= 1 && k <= 64, "k must be 1..64");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(knn_deg_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, st, (int)n, k, topv, ldv, dis_ws);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(knn_csr_kernel, dim3(gmr::grid_for(n + 1, 256)), dim3(256), 0, st, (int)n, k, topi, ldi, topv,
                     ldv, dis_ws, rowptr, col, val);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_gen_mask(int32_t B, int32_t I, int32_t k, const int32_t* topi, int64_t ldt, const float* x0,
                            const float* xs, int64_t ld, float* den, void* stream) {
  GMR_ARG(topi && x0 && xs && den && B > 0 && I > 0 && k > 0, "bad args");
  hipLaunchKernelGGL(gen_mask_kernel, dim3(gmr::grid_for((int64_t)B * I, 256)), dim3(256), 0, (hipStream_t)stream, B, I,
                     k, topi, ldt, x0, xs, ld, den);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_debias_select(int32_t B, int32_t k, const int32_t* topi, int64_t ldt, const float* x0,
                                 const float* xs, int64_t ld, float ratio, uint64_t seed, uint64_t step,
                                 uint64_t* keys_ws, int32_t* picks, int32_t max_picks, int32_t* n_picks,
                                 void* stream) {
  GMR_ARG(topi && x0 && xs && keys_ws && picks && n_picks && B > 0 && k > 0 && max_picks > 0, "bad args");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(debias_keys_kernel, dim3(gmr::grid_for((int64_t)B * k, 256)), dim3(256), 0, st, B, k, topi, ldt,
                     x0, xs, ld, seed, step, (unsigned long long*)keys_ws);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(debias_select_kernel, dim3(1), dim3(kSel), 0, st, B, k, topi, ldt,
                     (const unsigned long long*)keys_ws, ratio, picks, max_picks, n_picks);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_debias_apply(int32_t type, const int32_t* picks, const int32_t* n_picks, int32_t max_picks,
                                const float* x0, int64_t ld0, int32_t I, const int32_t* labels, float* den,
                                int64_t ldd, void* stream) {
  GMR_ARG(picks && x0 && labels && den && (type == 0 || type == 1) && max_picks >= 0, "bad args");
  if (max_picks == 0) return GMR_OK;
  hipLaunchKernelGGL(debias_apply_kernel, dim3(gmr::grid_for(max_picks, 4)), dim3(256), 0, (hipStream_t)stream, type,
                     picks, n_picks, max_picks, x0, ld0, I, labels, den, ldd);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_kmeans_standardize(int64_t n, int32_t d, const float* X, int64_t ldx, float* mean, float* scale,
                                      float* Y, int64_t ldy, float* sq, void* stream) {
  GMR_ARG(X && mean && scale && Y && sq && n > 0 && d > 0, "bad args");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(colstats_kernel, dim3(d), dim3(256), 0, st, n, d, X, ldx, mean, scale);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(standardize_kernel, dim3((unsigned)n), dim3(256), 0, st, n, d, X, ldx, mean, scale, Y, ldy, sq);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_kmeans_pp_pick(int64_t n, const float* mind, uint64_t seed, uint64_t step, int32_t* out,
                                  void* stream) {
  GMR_ARG(out && n > 0, "bad args");
  hipLaunchKernelGGL(kpp_pick_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, n, mind, seed, step, out);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_kmeans_pp_greedy(int64_t n, int32_t L, const float* xsq, const float* dots, int64_t ldd,
                                    const float* ccsq, float* mind, const float* Cc, int64_t ldcc, int32_t d, float* C,
                                    int64_t ldc, int32_t j, float* csq, void* stream) {
  GMR_ARG(xsq && dots && ccsq && mind && Cc && C && csq && n > 0 && L >= 1 && L <= 16 && d > 0 && j >= 0 && ldd >= L,
          "bad args");
  hipLaunchKernelGGL(kpp_greedy_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, n, L, xsq, dots, ldd, ccsq, mind,
                     Cc, ldcc, d, C, ldc, j, csq);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_kmeans_take_center(int32_t d, const float* X, int64_t ldx, const int32_t* idx, float* C,
                                      int64_t ldc, int32_t j, const float* xsq, float* csq, void* stream) {
  GMR_ARG(X && idx && C && xsq && csq, "bad args");
  hipLaunchKernelGGL(copy_row_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, d, X, ldx, idx, C, ldc, j, xsq, csq);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_kmeans_min_dist(int64_t n, const float* xsq, const float* dots, int64_t ld_dots, const float* csq,
                                   int32_t j, float* mind, int32_t first, void* stream) {
  GMR_ARG(xsq && dots && csq && mind && n > 0 && j >= 0 && ld_dots >= 1, "bad args");
  hipLaunchKernelGGL(min_dist_update_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, xsq,
                     dots, ld_dots, csq, (int)j, mind, first);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int64_t gmr_kmeans_parts(int64_t n) { return gmr::grid_for(n, 256); }

extern "C" int gmr_kmeans_assign(int64_t n, int32_t k, const float* dots, int64_t ldd, const float* csq,
                                 const float* xsq, int32_t* label, float* onehot_t, int64_t ldo, int32_t* changed,
                                 double* inertia_parts, void* stream) {
  GMR_ARG(dots && csq && xsq && label && onehot_t && changed && inertia_parts && n > 0 && k > 0, "bad args");
  hipLaunchKernelGGL(assign_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, k, dots, ldd,
                     csq, xsq, label, onehot_t, ldo, changed, inertia_parts);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_kmeans_centroids(int32_t k, int32_t d, const float* sums, int64_t lds, const float* onehot_t,
                                    int64_t ldo, int64_t n, float* C, int64_t ldc, float* csq, void* stream) {
  GMR_ARG(sums && onehot_t && C && csq && k > 0 && d > 0, "bad args");
  hipLaunchKernelGGL(centroid_kernel, dim3(k), dim3(256), 0, (hipStream_t)stream, k, d, sums, lds, onehot_t, ldo, n, C,
                     ldc, csq);
  GMR_LAUNCHED();
  return GMR_OK;
}
