// K1 — CSR SpMM for the LightGCN-style graph convolution (gfx950).
//
// Replaces torch.spmm / torch.sparse.mm on the normalised user-item adjacency
// (reference models/diffmm.py:136-191, 285).  Y = alpha * A * X + beta * Y with
//   * X given as up to 4 column blocks of 64 floats, each block a "split source":
//     source row s < split reads lo[b] + s*ld_lo[b], else hi[b] + (s-split)*ld_hi[b]
//     (this removes the torch.concat([uEmbeds, feats]) copies of the reference);
//   * nnz-balanced work: a plan cuts every row into segments of <= seg_nnz entries.
//     One wave64 owns one segment; a 64-float row block is 16 lanes x float4, so a
//     wave gathers 64/(16*nb) neighbour rows per instruction.  Single-segment rows
//     are written directly; hub rows (popular items) write per-segment partials that
//     a second pass adds in segment order, so results are deterministic.
#include <algorithm>
#include <cstdlib>

#include "gmr_common.h"

namespace {

constexpr int kPlanHdr = 4;  // n_seg, n_fix, n_partial, pad

struct PlanView {
  int* hdr;
  int* seg_row;
  int* seg_beg;
  int* seg_end;
  int* seg_slot;
  int* fix_row;
  int* fix_first;
  int* fix_cnt;
};

__host__ __device__ inline int64_t plan_max_seg(int64_t n_rows, int64_t nnz, int seg_nnz) {
  return n_rows + (nnz + seg_nnz - 1) / seg_nnz + 1;
}
__host__ __device__ inline int64_t plan_max_fix(int64_t n_rows, int64_t nnz, int seg_nnz) {
  int64_t f = (nnz + seg_nnz - 1) / seg_nnz + 1;
  return f < n_rows ? f : n_rows;
}

__host__ __device__ inline PlanView plan_view(int32_t* p, int64_t n_rows, int64_t nnz, int seg_nnz) {
  int64_t ms = plan_max_seg(n_rows, nnz, seg_nnz), mf = plan_max_fix(n_rows, nnz, seg_nnz);
  PlanView v;
  v.hdr = p;
  v.seg_row = p + kPlanHdr;
  v.seg_beg = v.seg_row + ms;
  v.seg_end = v.seg_beg + ms;
  v.seg_slot = v.seg_end + ms;
  v.fix_row = v.seg_slot + ms;
  v.fix_first = v.fix_row + mf;
  v.fix_cnt = v.fix_first + mf;
  return v;
}

// Single-workgroup plan builder: three exclusive scans over rows (segments, fix rows,
// partial slots) done as chunked serial sums + an LDS scan of the 1024 chunk totals.
__global__ void __launch_bounds__(1024) plan_build_kernel(const int* __restrict__ rowptr, int n_rows, int seg_nnz,
                                                          PlanView pv) {
  __shared__ int s_seg[1024], s_fix[1024], s_part[1024];
  const int t = threadIdx.x;
  const int chunk = (n_rows + 1023) / 1024;
  const int r0 = t * chunk, r1 = min(n_rows, r0 + chunk);
  int ns = 0, nf = 0, np_ = 0;
  for (int r = r0; r < r1; ++r) {
    int deg = rowptr[r + 1] - rowptr[r];
    int k = deg <= seg_nnz ? 1 : (deg + seg_nnz - 1) / seg_nnz;
    ns += k;
    if (k > 1) {
      nf += 1;
      np_ += k;
    }
  }
  s_seg[t] = ns;
  s_fix[t] = nf;
  s_part[t] = np_;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    int a = t >= off ? s_seg[t - off] : 0;
    int b = t >= off ? s_fix[t - off] : 0;
    int c = t >= off ? s_part[t - off] : 0;
    __syncthreads();
    s_seg[t] += a;
    s_fix[t] += b;
    s_part[t] += c;
    __syncthreads();
  }
  int so = s_seg[t] - ns, fo = s_fix[t] - nf, po = s_part[t] - np_;
  for (int r = r0; r < r1; ++r) {
    int beg = rowptr[r], end = rowptr[r + 1];
    int deg = end - beg;
    int k = deg <= seg_nnz ? 1 : (deg + seg_nnz - 1) / seg_nnz;
    if (k == 1) {
      pv.seg_row[so] = r;
      pv.seg_beg[so] = beg;
      pv.seg_end[so] = end;
      pv.seg_slot[so] = -1;
      ++so;
    } else {
      pv.fix_row[fo] = r;
      pv.fix_first[fo] = po;
      pv.fix_cnt[fo] = k;
      ++fo;
      for (int j = 0; j < k; ++j) {
        pv.seg_row[so] = r;
        pv.seg_beg[so] = beg + j * seg_nnz;
        pv.seg_end[so] = min(end, beg + (j + 1) * seg_nnz);
        pv.seg_slot[so] = po++;
        ++so;
      }
    }
  }
  if (t == 1023) {
    pv.hdr[0] = s_seg[1023];
    pv.hdr[1] = s_fix[1023];
    pv.hdr[2] = s_part[1023];
    pv.hdr[3] = 0;
  }
}

struct Src {
  const float* lo[4];
  const float* hi[4];
  int64_t ld_lo[4];
  int64_t ld_hi[4];
  int64_t split;
  int64_t panel_rows;  // lane plans: > 0 = X in column-panel layout (gmr_spmm_panel_f32), lo[0] = base
};

// lane plans: output block b (64 columns) goes to y[b] with row stride ld[b] (gmr_spmm_multi_f32)
struct Dst {
  float* y[4];
  int64_t ld[4];
};

// NB = number of 64-column blocks (d = 64 * NB).  LPR = lanes per neighbour row.
template <int NB>
__global__ void __launch_bounds__(256) spmm_seg_kernel(const int* __restrict__ col, const float* __restrict__ val,
                                                       PlanView pv, Src src, float alpha, float beta,
                                                       float* __restrict__ y, int64_t ldy,
                                                       float* __restrict__ partial) {
  constexpr int LPR = 16 * NB;
  constexpr int G = 64 / LPR;  // neighbour rows gathered per wave instruction
  const int lane = threadIdx.x & 63;
  const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n_seg = pv.hdr[0];
  if (seg >= n_seg) return;
  const int row = pv.seg_row[seg];
  const int beg = pv.seg_beg[seg], end = pv.seg_end[seg];
  const int slot = pv.seg_slot[seg];
  const int g = lane / LPR;
  const int sub = lane % LPR;
  const int blk = sub >> 4;
  const int c4 = (sub & 15) * 4;
  const float* lo = src.lo[blk];
  const float* hi = src.hi[blk];
  const int64_t ldl = src.ld_lo[blk], ldh = src.ld_hi[blk];
  const int64_t split = src.split;

  // UNR neighbour rows per lane group in flight: the loads of one batch are independent and
  // issued back to back (masked entries read row 0 with weight 0: always a valid address).
  constexpr int UNR = 8;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int base = beg; base < end; base += 64) {
    const int e = base + lane;
    int my_c = 0;
    float my_v = 0.f;
    if (e < end) {
      my_c = col[e];
      my_v = val[e];
    }
    const int cnt = min(64, end - base);
    for (int j = 0; j < cnt; j += UNR * G) {
      float4 xs[UNR];
      float vs[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int k = j + u * G + g;
        const int c = __shfl(my_c, k & 63);
        const float v = __shfl(my_v, k & 63);
        const bool ok = k < cnt;
        const int cc = ok ? c : 0;
        const float* p = cc < split ? lo + (int64_t)cc * ldl : hi + (int64_t)(cc - split) * ldh;
        xs[u] = *reinterpret_cast<const float4*>(p + c4);
        vs[u] = ok ? v : 0.f;
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) acc = gmr::f4_fma(vs[u], xs[u], acc);
    }
  }
#pragma unroll
  for (int m = LPR; m < 64; m <<= 1) acc = gmr::f4_add(acc, gmr::shfl_xor_f4(acc, m));
  if (g != 0) return;
  const int cc = blk * 64 + c4;
  if (slot < 0) {
    float* yp = y + (int64_t)row * ldy + cc;
    float4 o = gmr::f4_scale(alpha, acc);
    if (beta != 0.f) {
      float4 old = *reinterpret_cast<const float4*>(yp);
      o = gmr::f4_fma(beta, old, o);
    }
    *reinterpret_cast<float4*>(yp) = o;
  } else {
    *reinterpret_cast<float4*>(partial + (int64_t)slot * (64 * NB) + cc) = acc;
  }
}

template <int NB>
__global__ void __launch_bounds__(256) spmm_fix_kernel(PlanView pv, float alpha, float beta, float* __restrict__ y,
                                                       int64_t ldy, const float* __restrict__ partial) {
  constexpr int D = 64 * NB;
  constexpr int TPR = D / 4;  // threads per fix row
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t f = gid / TPR;
  if (f >= pv.hdr[1]) return;
  const int c = (int)(gid % TPR) * 4;
  const int row = pv.fix_row[f], first = pv.fix_first[f], cnt = pv.fix_cnt[f];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int j = 0;
  for (; j + 8 <= cnt; j += 8) {  // 8 independent partial rows in flight, summed in segment order
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(partial + (int64_t)(first + j + u) * D + c);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = gmr::f4_add(acc, v[u]);
  }
  for (; j < cnt; ++j) acc = gmr::f4_add(acc, *reinterpret_cast<const float4*>(partial + (int64_t)(first + j) * D + c));
  float* yp = y + (int64_t)row * ldy + c;
  float4 o = gmr::f4_scale(alpha, acc);
  if (beta != 0.f) o = gmr::f4_fma(beta, *reinterpret_cast<const float4*>(yp), o);
  *reinterpret_cast<float4*>(yp) = o;
}

// ----------------------------------------------------------------------------------------
// Blocked variant (plans with seg_nnz >= 512 = T): rows are packed into blocks of whole rows,
// a new block starting at row 0, every T-th row, and at each row that contains an nnz index
// that is a positive multiple of T, so a block holds <= ~T nnz plus at most one long row.
// One 1024-thread workgroup (128 lane groups of 8) owns one block and one 32-float column
// slice (XCD-pinned as in the group variant): it stages the block's rowptr in LDS, splits
// the block's nnz range evenly over its 128 groups (merge-path), and each group walks its
// range 16 neighbours at a time with all 16 gathers in flight, emitting rows as it crosses
// row ends.  Rows cut by group boundaries are summed in LDS in group order, so results are
// deterministic and no second pass (or partial buffer) is needed; hub rows get the whole
// workgroup.  Few, long-lived waves: the short-wave variants are bound by the wave launch
// rate on this graph shape (SQ counters, profiles/).
constexpr int kBlkThreads = 1024;
constexpr int kBlkGroups = kBlkThreads / 8;

__host__ __device__ inline int64_t blk_max_blocks(int64_t n_rows, int64_t nnz, int T) {
  return (nnz + T - 1) / T + (n_rows + T - 1) / T + 2;
}

__global__ void __launch_bounds__(1024) blk_plan_kernel(const int* __restrict__ rowptr, int n_rows, int T,
                                                        int max_blocks, int* __restrict__ plan) {
  __shared__ int s_cnt[1024];
  const int t = threadIdx.x;
  const int chunk = (n_rows + 1023) / 1024;
  const int r0 = t * chunk, r1 = min(n_rows, r0 + chunk);
  auto starts = [&](int r) -> bool {
    if (r == 0 || r % T == 0) return true;
    const int a = rowptr[r], b = rowptr[r + 1];
    const int first_mult = ((a + T - 1) / T) * T;  // smallest multiple of T >= a
    return first_mult > 0 && first_mult < b;
  };
  int n = 0;
  for (int r = r0; r < r1; ++r) n += starts(r) ? 1 : 0;
  s_cnt[t] = n;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    int v = t >= off ? s_cnt[t - off] : 0;
    __syncthreads();
    s_cnt[t] += v;
    __syncthreads();
  }
  int o = s_cnt[t] - n;
  int* blk_row = plan + kPlanHdr;
  int* blk_nnz = blk_row + max_blocks + 1;
  for (int r = r0; r < r1; ++r)
    if (starts(r)) {
      blk_row[o] = r;
      blk_nnz[o] = rowptr[r];
      ++o;
    }
  if (t == 1023) {
    plan[0] = s_cnt[1023];
    plan[1] = plan[2] = 0;
    plan[3] = T;
    blk_row[s_cnt[1023]] = n_rows;
    blk_nnz[s_cnt[1023]] = rowptr[n_rows];
  }
}

template <int NB>
__global__ void __launch_bounds__(kBlkThreads) spmm_blk_kernel(const int* __restrict__ rowptr,
                                                               const int* __restrict__ col,
                                                               const float* __restrict__ val,
                                                               const int* __restrict__ plan, int T, int max_blocks,
                                                               Src src, float alpha, float beta,
                                                               float* __restrict__ y, int64_t ldy) {
  constexpr int NS = 2 * NB, RP = 8 / NS;
  extern __shared__ __attribute__((aligned(16))) int s_rp[];  // T + 1 entries
  __shared__ float4 s_part[kBlkGroups][2][8];
  __shared__ int s_prow[kBlkGroups][2];
  const int xcd = blockIdx.x & 7;
  const int slice = xcd % NS, rpart = xcd / NS;
  const int nblk = plan[0];
  const int b_lo = (int)((int64_t)nblk * rpart / RP), b_hi = (int)((int64_t)nblk * (rpart + 1) / RP);
  const int bi = b_lo + (int)(blockIdx.x >> 3);
  if (bi >= b_hi) return;
  const int* blk_row = plan + kPlanHdr;
  const int* blk_nnz = blk_row + max_blocks + 1;
  // the block's row and nnz ranges come from the plan, so the rowptr staging and the first
  // col/val loads are issued together (one dependent round trip instead of two)
  const int row0 = blk_row[bi], nrows = blk_row[bi + 1] - row0;
  const int E0 = blk_nnz[bi], E1 = blk_nnz[bi + 1];
  const int grp = threadIdx.x >> 3, sub = threadIdx.x & 7;
  const int wg = (threadIdx.x & 63) >> 3;  // group index inside the wave (shuffle base)
  const int L = (E1 - E0 + kBlkGroups - 1) / kBlkGroups;
  const int a = min(E1, E0 + grp * L), b = min(E1, a + L);
  int ca = 0, cb = 0;
  float va = 0.f, vb = 0.f;
  if (a + sub < b) {
    ca = col[a + sub];
    va = val[a + sub];
  }
  if (a + 8 + sub < b) {
    cb = col[a + 8 + sub];
    vb = val[a + 8 + sub];
  }
  for (int i = threadIdx.x; i <= nrows; i += kBlkThreads) s_rp[i] = rowptr[row0 + i];
  s_prow[grp][0] = s_prow[grp][1] = -1;
  const int blk = slice >> 1;
  const int c4 = (slice & 1) * 32 + sub * 4;
  const float* lo = src.lo[blk] + c4;
  const float* hi = src.hi[blk] + c4;
  const int64_t ldl = src.ld_lo[blk], ldh = src.ld_hi[blk];
  const int64_t split = src.split;
  const int ycol = slice * 32 + sub * 4;
  // first 16 gathers go out before the barrier (they do not need the row table)
  float4 xs[16];
  float vs[16];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = __shfl(ca, (wg << 3) + u);
    vs[u] = __shfl(va, (wg << 3) + u);
    xs[u] = *reinterpret_cast<const float4*>(c < split ? lo + (int64_t)c * ldl : hi + (int64_t)(c - split) * ldh);
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = __shfl(cb, (wg << 3) + u);
    vs[8 + u] = __shfl(vb, (wg << 3) + u);
    xs[8 + u] = *reinterpret_cast<const float4*>(c < split ? lo + (int64_t)c * ldl : hi + (int64_t)(c - split) * ldh);
  }
  __syncthreads();
  if (a < b) {
    int lo_r = 0, hi_r = nrows - 1;  // largest r with s_rp[r] <= a
    while (lo_r < hi_r) {
      const int mid = (lo_r + hi_r + 1) >> 1;
      if (s_rp[mid] <= a) lo_r = mid; else hi_r = mid - 1;
    }
    int r = lo_r;
    int rend = s_rp[r + 1];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    auto emit = [&](int rr, float4 v) {
      const int rb = s_rp[rr], re = s_rp[rr + 1];
      if (rb >= a && re <= b) {
        float* yp = y + (int64_t)(row0 + rr) * ldy + ycol;
        float4 o = gmr::f4_scale(alpha, v);
        if (beta != 0.f) o = gmr::f4_fma(beta, *reinterpret_cast<const float4*>(yp), o);
        *reinterpret_cast<float4*>(yp) = o;
      } else {
        const int k = rb < a ? 0 : 1;  // 0: continues a row begun by an earlier group; 1: row owner
        s_part[grp][k][sub] = v;
        if (sub == 0) s_prow[grp][k] = rr;
      }
    };
    for (int e = a;;) {
      const int cnt = min(16, b - e);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        if (u < cnt) {
          while (e + u >= rend) {  // leave finished rows (empty ones are written by the pass below)
            if (s_rp[r] != rend) emit(r, acc);
            acc = make_float4(0.f, 0.f, 0.f, 0.f);
            ++r;
            rend = s_rp[r + 1];
          }
          acc = gmr::f4_fma(vs[u], xs[u], acc);
        }
      }
      e += 16;
      if (e >= b) break;
      // long ranges (hub blocks): next 16 neighbours
      const int ea = e + sub, eb = e + 8 + sub;
      ca = cb = 0;
      va = vb = 0.f;
      if (ea < b) {
        ca = col[ea];
        va = val[ea];
      }
      if (eb < b) {
        cb = col[eb];
        vb = val[eb];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = __shfl(ca, (wg << 3) + u);
        vs[u] = __shfl(va, (wg << 3) + u);
        xs[u] = *reinterpret_cast<const float4*>(c < split ? lo + (int64_t)c * ldl : hi + (int64_t)(c - split) * ldh);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = __shfl(cb, (wg << 3) + u);
        vs[8 + u] = __shfl(vb, (wg << 3) + u);
        xs[8 + u] =
            *reinterpret_cast<const float4*>(c < split ? lo + (int64_t)c * ldl : hi + (int64_t)(c - split) * ldh);
      }
    }
    emit(r, acc);
  }
  // empty rows: Y = beta * Y
  for (int i = grp; i < nrows; i += kBlkGroups) {
    if (s_rp[i] == s_rp[i + 1]) {
      float* yp = y + (int64_t)(row0 + i) * ldy + ycol;
      float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
      if (beta != 0.f) o = gmr::f4_scale(beta, *reinterpret_cast<const float4*>(yp));
      *reinterpret_cast<float4*>(yp) = o;
    }
  }
  __syncthreads();
  // rows cut by group boundaries: the owner adds the continuations in group order
  if (s_prow[grp][1] >= 0) {
    const int rr = s_prow[grp][1];
    float4 v = s_part[grp][1][sub];
    for (int k = grp + 1; k < kBlkGroups && s_prow[k][0] == rr; ++k) v = gmr::f4_add(v, s_part[k][0][sub]);
    float* yp = y + (int64_t)(row0 + rr) * ldy + ycol;
    float4 o = gmr::f4_scale(alpha, v);
    if (beta != 0.f) o = gmr::f4_fma(beta, *reinterpret_cast<const float4*>(yp), o);
    *reinterpret_cast<float4*>(yp) = o;
  }
}

// ----------------------------------------------------------------------------------------
// Lane plan (seg_nnz = GMR_SPMM_LANE_PLAN | L, L = 32, 64 or 128).  The graph-conv adjacencies
// average ~9 nnz per row with Zipf hub rows of thousands.  The wave-per-segment kernel above
// launches one wave per row and gathers whole 64*NB-float rows of X, which at d = 128 (13.6 MB at
// baby) do not fit one XCD's 4 MB L2, so most gathers are served by the Infinity Cache
// (DESIGN.md 5.1).  Here
//   * X is cut into S column slices of W = 4*LPR floats (W = 16 for d = 64 and 128, 32 for
//     d = 256); slice s is served by XCD s (S = 8) or by XCDs s and s + 4 (S = 4, each taking
//     every other work item): an XCD gathers only its slice, which stays in its L2 (1.7 MB at
//     baby), and one gather instruction fetches 64/LPR neighbour rows;
//   * a lane group of LPR lanes owns one row of degree <= L and walks it 8 entries at a time,
//     the col/val words of the next 8 in flight while the current gathers land; the plan orders
//     rows by descending degree, so the groups of a wave make (nearly) equal trip counts;
//   * a row of degree > L (a hub) takes a whole 256-thread workgroup: its lane groups stride
//     over 8-entry batches and their sums meet in a fixed butterfly + LDS order;
//   * the grid is a bounded number of workgroups per XCD that loop over the work, so few waves
//     are launched.  One launch, no partial buffer; every row is summed in a fixed order
//     wherever it lands, so results are deterministic.
// Plan: hdr {n_hub_desc, n_short, packed | n_split << 1, L}, then int4 {row, beg, end, slot}
// descriptors: hub segments (rows longest first by power of two), then the short rows by
// descending degree (rows of one class in any order).  A hub row longer than kHubSeg entries is
// cut into kHubSeg-entry segments, each its own workgroup (the rebuilt UI graphs can have one
// item row holding most users: a single workgroup walking it was the launch's whole tail); the
// segments write partial sums to partial[slot] and a fixup pass adds them in segment order
// (lane_fix list {row, first slot, n_segments, 0}), so the sum order stays fixed.
constexpr int kLaneThreads = 256;
constexpr int kPackTab = 34;  // packed lane plan: bucket-table entries per column (see below)
constexpr int kLaneMaxBuckets = 320;
constexpr int kHubSeg = 1024;  // entries per hub segment

__host__ __device__ inline int64_t lane_desc_cap(int64_t n_rows, int64_t nnz) { return n_rows + nnz / kHubSeg + 1; }
__host__ __device__ inline int64_t lane_fix_cap(int64_t nnz) { return nnz / kHubSeg + 1; }
__host__ __device__ inline int64_t lane_fix_off(int64_t n_rows, int64_t nnz) {
  return kPlanHdr + 4 * lane_desc_cap(n_rows, nnz);
}
__host__ __device__ inline int64_t lane_tab_off(int64_t n_rows, int64_t nnz) {
  return lane_fix_off(n_rows, nnz) + 4 * lane_fix_cap(nnz);
}

__device__ __forceinline__ int lane_bucket(int deg, int L, int HB) {
  return deg > L ? 30 - (31 - __clz(deg)) : HB + (L - deg);
}

// rows up to kHubSplit entries stay whole (one workgroup, ≤ 16 passes): norm_adj's Zipf hubs
// (≤ 4.4k at baby) then need no fixup launch; longer rows (a collapsed rebuilt UI graph's item
// row of most users) are cut into kHubSeg-entry segments
constexpr int kHubSplit = 8192;
__host__ __device__ inline int hub_segs(int deg) { return deg > kHubSplit ? (deg + kHubSeg - 1) / kHubSeg : 1; }

// Row classes (csplit > 0, non-packed plans): the short rows >= csplit (the item rows of a
// bipartite graph) are listed before the rows < csplit (users), each class by descending degree,
// so each phase of the launch gathers from ONE side's X rows (users' or items' slice): a smaller
// live footprint per XCD L2 than the interleaved degree order.
__device__ __forceinline__ int lane_bucket_c(int r, int deg, int L, int HB, int csplit) {
  return deg > L ? lane_bucket(deg, L, HB) : lane_bucket(deg, L, HB) + (csplit > 0 && r < csplit ? L + 1 : 0);
}

__global__ void __launch_bounds__(1024) lane_plan_kernel(const int* __restrict__ rowptr, int n_rows, int64_t nnz, int L,
                                                         int HB, int packed, int csplit, int* __restrict__ plan) {
  __shared__ int s_cnt[kLaneMaxBuckets], s_off[kLaneMaxBuckets];
  __shared__ int s_slot, s_nfix;
  const int t = threadIdx.x, nbk = HB + (csplit > 0 ? 2 : 1) * (L + 1);
  for (int i = t; i < nbk; i += 1024) s_cnt[i] = 0;
  if (t == 0) s_slot = s_nfix = 0;
  __syncthreads();
  for (int r = t; r < n_rows; r += 1024) {
    const int deg = rowptr[r + 1] - rowptr[r];
    atomicAdd(&s_cnt[lane_bucket_c(r, deg, L, HB, csplit)], deg > L ? hub_segs(deg) : 1);  // one per hub segment
  }
  __syncthreads();
  if (t == 0) {
    int o = 0, n_hub = 0;
    for (int b = 0; b < nbk; ++b) {
      s_off[b] = o;
      o += s_cnt[b];
      if (b == HB - 1) n_hub = o;
    }
    plan[0] = n_hub;
    plan[1] = o - n_hub;
    plan[3] = L;
    if (packed) {  // bucket j = degree L - j: first plan index and first packed entry
      int* tb = plan + lane_tab_off(n_rows, nnz);
      int e = 0;
      for (int j = 0; j <= L; ++j) {
        tb[j] = s_off[HB + j];
        tb[kPackTab + j] = e;
        e += s_cnt[HB + j] * (L - j);
      }
      tb[L + 1] = o;
      tb[kPackTab + L + 1] = e;
    }
  }
  __syncthreads();
  int4* desc = reinterpret_cast<int4*>(plan + kPlanHdr);
  int4* fix = reinterpret_cast<int4*>(plan + lane_fix_off(n_rows, nnz));
  for (int r = t; r < n_rows; r += 1024) {
    const int beg = rowptr[r], end = rowptr[r + 1], deg = end - beg;
    const int ns = deg > L ? hub_segs(deg) : 1;
    const int d0 = atomicAdd(&s_off[lane_bucket_c(r, deg, L, HB, csplit)], ns);
    if (ns == 1) {
      desc[d0] = make_int4(r, beg, end, -1);
    } else {  // segments j of the row write partial[slot0 + j]; the fixup adds them in j order
      const int slot0 = atomicAdd(&s_slot, ns);
      fix[atomicAdd(&s_nfix, 1)] = make_int4(r, slot0, ns, 0);
      for (int j = 0; j < ns; ++j)
        desc[d0 + j] = make_int4(r, beg + j * kHubSeg, min(end, beg + (j + 1) * kHubSeg), slot0 + j);
    }
  }
  __syncthreads();
  if (t == 0) plan[2] = packed | (s_nfix << 1);
}

// hub-segment fixup: y[row] = alpha * sum_j partial[slot0 + j] + beta * y[row], j in order
__device__ __forceinline__ void lane_fix_body(const int* __restrict__ plan, int64_t n_rows, int64_t nnz, int ncols,
                                              const float* __restrict__ part, float alpha, float beta, const Dst& dst,
                                              int i0, int step) {
  const int n_fix = plan[2] >> 1;
  const int4* fix = reinterpret_cast<const int4*>(plan + lane_fix_off(n_rows, nnz));
  const int c4n = ncols / 4;
  for (int i = i0; i < n_fix * c4n; i += step) {
    const int f = i / c4n, c = (i % c4n) * 4;
    const int4 fx = fix[f];
    float4 s = *reinterpret_cast<const float4*>(part + (int64_t)fx.y * 256 + c);
    for (int j = 1; j < fx.z; ++j) s = gmr::f4_add(s, *reinterpret_cast<const float4*>(part + (int64_t)(fx.y + j) * 256 + c));
    float* yp = dst.y[c >> 6] + (int64_t)fx.x * dst.ld[c >> 6] + (c & 63);
    float4 o = gmr::f4_scale(alpha, s);
    if (beta != 0.f) o = gmr::f4_fma(beta, *reinterpret_cast<const float4*>(yp), o);
    *reinterpret_cast<float4*>(yp) = o;
  }
}
__global__ void __launch_bounds__(256) lane_fix_kernel(const int* __restrict__ plan, int64_t n_rows, int64_t nnz,
                                                       int ncols, const float* __restrict__ part, float alpha,
                                                       float beta, Dst dst) {
  lane_fix_body(plan, n_rows, nnz, ncols, part, alpha, beta, dst, blockIdx.x * blockDim.x + threadIdx.x,
                gridDim.x * blockDim.x);
}

// Packed lane plan (GMR_SPMM_LANE_PLAN | GMR_SPMM_PACKED | 32).  The short rows' col/val are
// copied into plan order, so the rows of one degree bucket sit back to back with a fixed stride:
// a lane group finds its row's entries from a 34-entry bucket table in LDS (no descriptor load on
// the critical path), and the next pass's col/val are in flight while the current gathers land.
// Plan words after the descriptors: table {first plan index}[34] {first entry}[34], then
// pcol[nnz], pval[nnz].  Entries keep their CSR order, so sums are bit-identical to the lane plan.
__host__ __device__ inline int64_t pack_off(int64_t n_rows, int64_t nnz) {
  return lane_tab_off(n_rows, nnz) + 2 * kPackTab;
}

__global__ void __launch_bounds__(256) lane_pack_kernel(const int* __restrict__ col, const float* __restrict__ val,
                                                        int n_rows, int64_t nnz, int* __restrict__ plan) {
  const int n_hub = plan[0], L = plan[3], n_desc = plan[0] + plan[1];
  const int* tb = plan + lane_tab_off(n_rows, nnz);
  const int4* desc = reinterpret_cast<const int4*>(plan + kPlanHdr);
  int* pcol = plan + pack_off(n_rows, nnz);
  float* pval = reinterpret_cast<float*>(pcol + nnz);
  for (int k = n_hub + blockIdx.x * blockDim.x + threadIdx.x; k < n_desc; k += gridDim.x * blockDim.x) {
    const int4 d = desc[k];
    const int deg = d.z - d.y, j = L - deg;
    const int e0 = tb[kPackTab + j] + (k - tb[j]) * deg;
    for (int q = 0; q < deg; ++q) {
      pcol[e0 + q] = col[d.y + q];
      pval[e0 + q] = val[d.y + q];
    }
  }
}

// One lane-plan product for workgroup `bid` of its launch (bid & 7 = the XCD: launches and the
// job ranges of a multi-job launch are multiples of 8 workgroups).
template <int LPR, bool PACKED, int EB>
__device__ __forceinline__ void lane_body(const int* __restrict__ col, const float* __restrict__ val,
                                          const int* __restrict__ plan, int S, int wpx, const Src& src, float alpha,
                                          float beta, const Dst& dst, int n_rows, int64_t nnz,
                                          float* __restrict__ hub_part, int bid, int nt) {
  constexpr int NW = kLaneThreads / 64;  // waves per workgroup
  constexpr int NG = 64 / LPR;           // lane groups per wave
  constexpr int EPL = EB / LPR;          // col/val words per lane per batch
  __shared__ float4 s_red[NW][LPR];
  const int xcd = bid & 7, k = bid >> 3;
  const int slice = xcd % S, part = xcd / S, P = 8 / S;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane / LPR, sub = lane % LPR, gbase = grp * LPR;
  const int n_hub = plan[0], n_short = plan[1];
  const int4* __restrict__ desc = reinterpret_cast<const int4*>(plan + kPlanHdr);
  const int c0 = slice * 4 * LPR;  // first column of the slice
  const int blk = c0 >> 6, cin = (c0 & 63) + sub * 4;
  // column-panel X: slice s is a contiguous panel_rows x W block, so an XCD's slice fills whole lines
  const bool panel = src.panel_rows > 0;
  const float* lo = panel ? src.lo[0] + (int64_t)slice * src.panel_rows * (4 * LPR) + sub * 4 : src.lo[blk] + cin;
  const float* hi = panel ? lo : src.hi[blk] + cin;
  const int64_t ldl = panel ? 4 * LPR : src.ld_lo[blk], ldh = panel ? 4 * LPR : src.ld_hi[blk];
  const int64_t split = panel ? src.panel_rows : src.split;
  float* yc = dst.y[blk] + (c0 & 63) + sub * 4;
  const int64_t ldy = dst.ld[blk];

  // nt & 2: the streamed-once index words (col/val, packed entries) are read non-temporally, so they
  // do not evict the X slice from L2; nt & 1: Y is stored non-temporally for the same reason
  auto ldi = [&](const int* p) -> int { return (nt & 2) ? __builtin_nontemporal_load(p) : *p; };
  auto ldf = [&](const float* p) -> float { return (nt & 2) ? __builtin_nontemporal_load(p) : *p; };
  // sum over the batches at e0, e0 + step, ... below end (e0, end and step are uniform in the group)
  auto walk = [&](int e0, int end, int step) -> float4 {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int cc[EPL];
    float vv[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
      const int i = e0 + q * LPR + sub;
      cc[q] = i < end ? ldi(col + i) : 0;
      vv[q] = i < end ? ldf(val + i) : 0.f;
    }
    for (int e = e0; e < end; e += step) {
      float4 xs[EB];
      float vs[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int c = __shfl(cc[u / LPR], gbase + u % LPR);
        vs[u] = __shfl(vv[u / LPR], gbase + u % LPR);
        xs[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e + u < end)
          xs[u] = *reinterpret_cast<const float4*>(c < split ? lo + (int64_t)c * ldl : hi + (int64_t)(c - split) * ldh);
      }
      const int en = e + step;
#pragma unroll
      for (int q = 0; q < EPL; ++q) {  // the next batch's indices travel while the gathers land
        const int i = en + q * LPR + sub;
        cc[q] = i < end ? ldi(col + i) : 0;
        vv[q] = i < end ? ldf(val + i) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < EB; ++u) acc = gmr::f4_fma(vs[u], xs[u], acc);
    }
    return acc;
  };
  auto store = [&](int row, float4 acc) {
    float* yp = yc + (int64_t)row * ldy;
    float4 o = gmr::f4_scale(alpha, acc);
    if (beta != 0.f) o = gmr::f4_fma(beta, *reinterpret_cast<const float4*>(yp), o);
    if (nt & 1) {
      typedef float v4 __attribute__((ext_vector_type(4)));
      v4 ov = {o.x, o.y, o.z, o.w};
      __builtin_nontemporal_store(ov, reinterpret_cast<v4*>(yp));
    } else {
      *reinterpret_cast<float4*>(yp) = o;
    }
  };

  const int wg = part * wpx + k, n_wg = P * wpx;
  __shared__ int s_tb[2 * kPackTab];
  if (PACKED) {
    if (threadIdx.x < 2 * kPackTab) s_tb[threadIdx.x] = plan[lane_tab_off(n_rows, nnz) + threadIdx.x];
    __syncthreads();
  }
  // hub rows: one workgroup each; group partials meet in a fixed butterfly + LDS order
  for (int hb = wg; hb < n_hub; hb += n_wg) {
    const int4 d = desc[hb];
    float4 acc = walk(d.y + (wid * NG + grp) * EB, d.z, NW * NG * EB);
#pragma unroll
    for (int m = LPR; m < 64; m <<= 1) acc = gmr::f4_add(acc, gmr::shfl_xor_f4(acc, m));
    if (grp == 0) s_red[wid][sub] = acc;
    __syncthreads();
    if (threadIdx.x < LPR) {
      float4 s = s_red[0][sub];
#pragma unroll
      for (int q = 1; q < NW; ++q) s = gmr::f4_add(s, s_red[q][sub]);
      if (d.w < 0)
        store(d.x, s);
      else  // a segment of a split hub row: partial row d.w, full-width columns (lane_fix_kernel adds them)
        *reinterpret_cast<float4*>(hub_part + (int64_t)d.w * 256 + c0 + sub * 4) = s;
    }
    __syncthreads();
  }
  // short rows: NG consecutive (equal-degree) rows per wave and pass; the next descriptor is in
  // flight while the current row is walked
  const int stride = n_wg * NW * NG;
  int base = (wg * NW + wid) * NG;
  if constexpr (PACKED) {
    constexpr int EM = 32 / LPR;  // col/val words per lane of a degree-32 row
    const int* __restrict__ pcol = plan + pack_off(n_rows, nnz);
    const float* __restrict__ pval = reinterpret_cast<const float*>(pcol + nnz);
    const int* __restrict__ drow = plan + kPlanHdr;  // desc[k].x = plan + kPlanHdr + 4k
    // row, degree and entries of short row `base + grp` (bucket j: largest j with s_tb[j] <= k)
    auto fetch = [&](int b, int& row, int& deg, int* cc, float* vv) {
      const int k = n_hub + b + grp;
      deg = 0;
      row = -1;
      if (b + grp < n_short) {
        int j = 0;
#pragma unroll
        for (int st = 32; st >= 1; st >>= 1)
          if (j + st <= 32 && s_tb[j + st] <= k) j += st;
        deg = 32 - j;
        const int e0 = s_tb[kPackTab + j] + (k - s_tb[j]) * deg;
        row = drow[4 * k];
#pragma unroll
        for (int q = 0; q < EM; ++q) {
          const int i = q * LPR + sub;
          cc[q] = i < deg ? ldi(pcol + e0 + i) : 0;
          vv[q] = i < deg ? ldf(pval + e0 + i) : 0.f;
        }
      } else {
#pragma unroll
        for (int q = 0; q < EM; ++q) {
          cc[q] = 0;
          vv[q] = 0.f;
        }
      }
    };
    int row, deg, cc[EM];
    float vv[EM];
    fetch(base, row, deg, cc, vv);
    for (; base < n_short; base += stride) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      float4 xs[EB];
      float vs[EB];
      // batch 0 gathers first, then the next pass's indices, then the rest of this row
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int c = __shfl(cc[u / LPR], gbase + u % LPR);
        vs[u] = __shfl(vv[u / LPR], gbase + u % LPR);
        xs[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (u < deg)
          xs[u] = *reinterpret_cast<const float4*>(c < split ? lo + (int64_t)c * ldl : hi + (int64_t)(c - split) * ldh);
      }
      int rown, degn, cn[EM];
      float vn[EM];
      fetch(base + stride, rown, degn, cn, vn);
#pragma unroll
      for (int u = 0; u < EB; ++u) acc = gmr::f4_fma(vs[u], xs[u], acc);
#pragma unroll
      for (int bt = 1; bt < 32 / EB; ++bt) {
        if (bt * EB < deg) {
#pragma unroll
          for (int u = 0; u < EB; ++u) {
            const int e = bt * EB + u;
            const int c = __shfl(cc[e / LPR], gbase + e % LPR);
            vs[u] = __shfl(vv[e / LPR], gbase + e % LPR);
            xs[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e < deg)
              xs[u] =
                  *reinterpret_cast<const float4*>(c < split ? lo + (int64_t)c * ldl : hi + (int64_t)(c - split) * ldh);
          }
#pragma unroll
          for (int u = 0; u < EB; ++u) acc = gmr::f4_fma(vs[u], xs[u], acc);
        }
      }
      if (row >= 0) store(row, acc);
      row = rown;
      deg = degn;
#pragma unroll
      for (int q = 0; q < EM; ++q) {
        cc[q] = cn[q];
        vv[q] = vn[q];
      }
    }
    return;
  }
  int4 d = base + grp < n_short ? desc[n_hub + base + grp] : make_int4(-1, 0, 0, 0);
  for (; base < n_short; base += stride) {
    const int nb = base + stride + grp;
    const int4 dn = nb < n_short ? desc[n_hub + nb] : make_int4(-1, 0, 0, 0);
    const float4 acc = walk(d.y, d.z, EB);
    if (d.x >= 0) store(d.x, acc);
    d = dn;
  }
}

template <int LPR, bool PACKED, int EB>
__global__ void __launch_bounds__(kLaneThreads) spmm_lane_kernel(const int* __restrict__ col,
                                                                  const float* __restrict__ val,
                                                                  const int* __restrict__ plan, int S, int wpx, Src src,
                                                                  float alpha, float beta, Dst dst, int n_rows,
                                                                  int64_t nnz, float* __restrict__ hub_part, int nt) {
  lane_body<LPR, PACKED, EB>(col, val, plan, S, wpx, src, alpha, beta, dst, n_rows, nnz, hub_part, blockIdx.x, nt);
}

// Multi-job lane launch (gmr_spmm_jobs_f32): independent products, possibly of different
// matrices, in one grid; job q owns workgroups [off[q], off[q+1]) (multiples of 8, so each keeps
// its XCD-slice mapping) and runs exactly the single-job body.
constexpr int kMaxJobs = 4;
struct LaneJob {
  const int* col;
  const float* val;
  const int* plan;
  float* part;
  Src src;
  Dst dst;
  int64_t nnz;
  float alpha, beta;
  int S, wpx, n_rows, packed, fix, ncols, nt;
};
struct LaneJobs {
  LaneJob j[kMaxJobs];
  int off[kMaxJobs + 1];
  int n;
};

// hub-segment fixups of every job whose plan split hub rows (jobs write disjoint outputs)
__global__ void __launch_bounds__(256) lane_fix_jobs_kernel(LaneJobs J) {
  for (int q = 0; q < J.n; ++q) {
    const LaneJob& jb = J.j[q];
    if (jb.fix)
      lane_fix_body(jb.plan, jb.n_rows, jb.nnz, jb.ncols, jb.part, jb.alpha, jb.beta, jb.dst,
                    blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
  }
}

template <int LPR, int EB>
__global__ void __launch_bounds__(kLaneThreads) spmm_lane_jobs_kernel(LaneJobs J) {
  const int b = blockIdx.x;
  int q = 0;
#pragma unroll
  for (int t = 1; t < kMaxJobs; ++t) q += (t < J.n && b >= J.off[t]) ? 1 : 0;
  const LaneJob& jb = J.j[q];
  const int bid = b - J.off[q];
  if (jb.packed)
    lane_body<LPR, true, EB>(jb.col, jb.val, jb.plan, jb.S, jb.wpx, jb.src, jb.alpha, jb.beta, jb.dst, jb.n_rows,
                             jb.nnz, jb.part, bid, jb.nt);
  else
    lane_body<LPR, false, EB>(jb.col, jb.val, jb.plan, jb.S, jb.wpx, jb.src, jb.alpha, jb.beta, jb.dst, jb.n_rows,
                              jb.nnz, jb.part, bid, jb.nt);
}


// ----------------------------------------------------------------------------------------
// Chunk plan (seg_nnz = GMR_SPMM_CHUNK_PLAN).  The lane plan gives each lane group one row per
// pass, so a row of degree 2 (every user row of a rebuilt UI graph) leaves 6 of the group's 8
// gather slots idle and a row of degree 9 (a typical norm_adj row) takes two dependent rounds.
// Here the rows of degree 1..128 are cut, in row order, into tasks of whole rows holding at most
// 128 entries; a wave owns a task and its lane groups each take 128 / NG consecutive entries,
// whatever rows they belong to, so every gather slot is used and a task is ONE round of gathers.
// Row sums that cross lane groups meet in LDS in group order (the group where the row starts adds
// the continuations), so each row is summed in a fixed order: deterministic.  Rows of degree
// > 128 (hubs) take a whole 1024-thread workgroup as in the lane plan; empty rows are listed.
// The X slicing (one column slice per XCD, kept in its L2) is the lane plan's.
// Plan: hdr {n_hub, n_task, n_empty, n_packed}, hub int4 {row, beg, end, 0}[HC],
//       task int2 {first packed entry, entries}[TC], empty rows [n_rows], row start in the
//       packed arrays [n_rows], then pcol[nnz], pval[nnz], prow[nnz] (rows of degree 1..128).
constexpr int kChunkThreads = 1024;
constexpr int kChunkTask = 128;  // entries per task = hub threshold

__host__ __device__ inline int64_t r4(int64_t w) { return (w + 3) / 4 * 4; }
__host__ __device__ inline int64_t chunk_hub_cap(int64_t n_rows, int64_t nnz) {
  const int64_t h = nnz / (kChunkTask + 1) + 1;
  return h < n_rows ? h : n_rows;
}
struct ChunkView {
  int* hdr;
  int4* hub;
  int2* task;
  int* empty;
  int* vstart;
  int* pcol;
  float* pval;
  int* prow;
};
__host__ __device__ inline ChunkView chunk_view(int32_t* p, int64_t n_rows, int64_t nnz) {
  ChunkView v;
  v.hdr = p;
  int64_t o = kPlanHdr;
  v.hub = reinterpret_cast<int4*>(p + o);
  o += 4 * chunk_hub_cap(n_rows, nnz);
  v.task = reinterpret_cast<int2*>(p + o);
  o += r4(2 * n_rows);
  v.empty = p + o;
  o += r4(n_rows);
  v.vstart = p + o;
  o += r4(n_rows);
  v.pcol = p + o;
  o += r4(nnz);
  v.pval = reinterpret_cast<float*>(p + o);
  o += r4(nnz);
  v.prow = p + o;
  return v;
}
__host__ __device__ inline int64_t chunk_plan_words(int64_t n_rows, int64_t nnz) {
  return kPlanHdr + 4 * chunk_hub_cap(n_rows, nnz) + r4(2 * n_rows) + 2 * r4(n_rows) + 3 * r4(nnz);
}

// exclusive scan of one int per thread of a 1024-thread block (Hillis-Steele in LDS)
__device__ int block_excl_scan(int v, int* s, int* total) {
  const int t = threadIdx.x;
  s[t] = v;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int a = t >= o ? s[t - o] : 0;
    __syncthreads();
    s[t] += a;
    __syncthreads();
  }
  const int incl = s[t];
  *total = s[1023];
  __syncthreads();
  return incl - v;
}

// One workgroup: thread t owns rows [t R, (t+1) R) and packs its short rows greedily into tasks of
// <= 128 entries (tasks never cross thread ranges); counts, scans, then writes the descriptors.
__global__ void __launch_bounds__(1024) chunk_plan_kernel(const int* __restrict__ rowptr, int n_rows, int64_t nnz,
                                                          int* __restrict__ plan) {
  __shared__ int s_scan[1024];
  ChunkView pv = chunk_view(plan, n_rows, nnz);
  const int t = threadIdx.x;
  const int R = (n_rows + 1023) / 1024;
  const int r0 = min(n_rows, t * R), r1 = min(n_rows, r0 + R);
  int nh = 0, ne = 0, nt = 0, nv = 0, run = 0;
  for (int r = r0; r < r1; ++r) {
    const int d = rowptr[r + 1] - rowptr[r];
    if (d == 0) {
      ++ne;
    } else if (d > kChunkTask) {
      ++nh;
    } else {
      nv += d;
      if (run == 0 || run + d > kChunkTask) {
        ++nt;
        run = d;
      } else {
        run += d;
      }
    }
  }
  int th, te, tt, tv;
  int oh = block_excl_scan(nh, s_scan, &th);
  int oe = block_excl_scan(ne, s_scan, &te);
  int ot = block_excl_scan(nt, s_scan, &tt);
  int ov = block_excl_scan(nv, s_scan, &tv);
  int tb = -1;  // first packed entry of the open task
  run = 0;
  for (int r = r0; r < r1; ++r) {
    const int beg = rowptr[r], end = rowptr[r + 1], d = end - beg;
    if (d == 0) {
      pv.empty[oe++] = r;
      pv.vstart[r] = -1;
    } else if (d > kChunkTask) {
      pv.hub[oh++] = make_int4(r, beg, end, 0);
      pv.vstart[r] = -1;
    } else {
      if (run == 0 || run + d > kChunkTask) {
        if (run > 0) pv.task[ot++] = make_int2(tb, run);
        tb = ov;
        run = d;
      } else {
        run += d;
      }
      pv.vstart[r] = ov;
      ov += d;
    }
  }
  if (run > 0) pv.task[ot++] = make_int2(tb, run);
  if (t == 0) {
    pv.hdr[0] = th;
    pv.hdr[1] = tt;
    pv.hdr[2] = te;
    pv.hdr[3] = tv;
  }
}

// copies the short rows' col / val (and their row ids) into the packed arrays
__global__ void __launch_bounds__(256) chunk_pack_kernel(const int* __restrict__ rowptr, const int* __restrict__ col,
                                                         const float* __restrict__ val, int n_rows, int64_t nnz,
                                                         int* __restrict__ plan) {
  ChunkView pv = chunk_view(plan, n_rows, nnz);
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n_rows; r += gridDim.x * blockDim.x) {
    const int v = pv.vstart[r];
    if (v < 0) continue;
    const int beg = rowptr[r], d = rowptr[r + 1] - beg;
    for (int q = 0; q < d; ++q) {
      pv.pcol[v + q] = col[beg + q];
      pv.pval[v + q] = val[beg + q];
      pv.prow[v + q] = r;
    }
  }
}

template <int LPR>
__global__ void __launch_bounds__(kChunkThreads) spmm_chunk_kernel(const int* __restrict__ col,
                                                                   const float* __restrict__ val,
                                                                   const int* __restrict__ plan, int n_rows,
                                                                   int64_t nnz, int S, int wpx, Src src, float alpha,
                                                                   float beta, Dst dst) {
  constexpr int NW = kChunkThreads / 64;  // waves per workgroup
  constexpr int NG = 64 / LPR;            // lane groups per wave
  constexpr int EB = kChunkTask / NG;     // entries per lane group and task (8 or 16)
  constexpr int EPL = EB / LPR;           // entry words per lane (2)
  __shared__ float4 s_red[NW][LPR];
  __shared__ float4 s_cacc[NW][NG][LPR];  // continuation partial of each lane group's first row
  __shared__ int s_crow[NW][NG];          // that row, or -1 when the group's first row starts in it
  __shared__ int s_cend[NW][NG];          // 1 when that continuation ends inside the group
  const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
  const int slice = xcd % S, part = xcd / S, P = 8 / S;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane / LPR, sub = lane % LPR, gbase = grp * LPR;
  const ChunkView pv = chunk_view(const_cast<int*>(plan), n_rows, nnz);
  const int n_hub = plan[0], n_task = plan[1], n_empty = plan[2];
  const int c0 = slice * 4 * LPR;  // first column of the slice
  const int blk = c0 >> 6, cin = (c0 & 63) + sub * 4;
  const bool panel = src.panel_rows > 0;
  const float* lo = panel ? src.lo[0] + (int64_t)slice * src.panel_rows * (4 * LPR) + sub * 4 : src.lo[blk] + cin;
  const float* hi = panel ? lo : src.hi[blk] + cin;
  const int64_t ldl = panel ? 4 * LPR : src.ld_lo[blk], ldh = panel ? 4 * LPR : src.ld_hi[blk];
  const int64_t split = panel ? src.panel_rows : src.split;
  float* yc = dst.y[blk] + (c0 & 63) + sub * 4;
  const int64_t ldy = dst.ld[blk];
  auto gather = [&](int c) -> float4 {
    return *reinterpret_cast<const float4*>(c < split ? lo + (int64_t)c * ldl : hi + (int64_t)(c - split) * ldh);
  };
  auto store = [&](int row, float4 acc) {
    float* yp = yc + (int64_t)row * ldy;
    float4 o = gmr::f4_scale(alpha, acc);
    if (beta != 0.f) o = gmr::f4_fma(beta, *reinterpret_cast<const float4*>(yp), o);
    *reinterpret_cast<float4*>(yp) = o;
  };
  const int wg = part * wpx + k, n_wg = P * wpx;

  // hub rows: one workgroup each, every lane group strides over EB-entry batches
  for (int hb = wg; hb < n_hub; hb += n_wg) {
    const int4 d = pv.hub[hb];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e0 = d.y + (wid * NG + grp) * EB; e0 < d.z; e0 += NW * NG * EB) {
      int cc[EPL];
      float vv[EPL];
#pragma unroll
      for (int q = 0; q < EPL; ++q) {
        const int i = e0 + q * LPR + sub;
        cc[q] = i < d.z ? col[i] : 0;
        vv[q] = i < d.z ? val[i] : 0.f;
      }
      float4 xs[EB];
      float vs[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int c = __shfl(cc[u / LPR], gbase + u % LPR);
        vs[u] = __shfl(vv[u / LPR], gbase + u % LPR);
        xs[u] = e0 + u < d.z ? gather(c) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < EB; ++u) acc = gmr::f4_fma(vs[u], xs[u], acc);
    }
#pragma unroll
    for (int m = LPR; m < 64; m <<= 1) acc = gmr::f4_add(acc, gmr::shfl_xor_f4(acc, m));
    if (grp == 0) s_red[wid][sub] = acc;
    __syncthreads();
    if (threadIdx.x < LPR) {
      float4 s = s_red[0][sub];
#pragma unroll
      for (int q = 1; q < NW; ++q) s = gmr::f4_add(s, s_red[q][sub]);
      store(d.x, s);
    }
    __syncthreads();
  }
  // empty rows: Y = beta * Y
  for (int i = wg * (kChunkThreads / LPR) + threadIdx.x / LPR; i < n_empty; i += n_wg * (kChunkThreads / LPR))
    store(pv.empty[i], make_float4(0.f, 0.f, 0.f, 0.f));

  // tasks: one per wave and pass
  const int* __restrict__ pcol = pv.pcol;
  const float* __restrict__ pval = pv.pval;
  const int* __restrict__ prow = pv.prow;
  for (int t = wg * NW + wid; t < n_task; t += n_wg * NW) {
    const int2 td = pv.task[t];
    const int tend = td.x + td.y;
    const int g0 = td.x + grp * EB, g1 = min(tend, g0 + EB);
    int cc[EPL], rr[EPL];
    float vv[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
      const int i = g0 + q * LPR + sub;
      const bool ok = i < g1;
      cc[q] = ok ? pcol[i] : 0;
      vv[q] = ok ? pval[i] : 0.f;
      rr[q] = ok ? prow[i] : -1;
    }
    // does the group's first row start before it / its last row continue after it?
    const int prev_row = (g0 > td.x && g0 < g1) ? prow[g0 - 1] : -1;
    const int next_row = (g1 < tend && g0 < g1) ? prow[g1] : -1;
    float4 xs[EB];
    float vs[EB];
    int rs[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int c = __shfl(cc[u / LPR], gbase + u % LPR);
      vs[u] = __shfl(vv[u / LPR], gbase + u % LPR);
      rs[u] = __shfl(rr[u / LPR], gbase + u % LPR);
      xs[u] = g0 + u < g1 ? gather(c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int first = rs[0];
    const bool cont = first >= 0 && first == prev_row;  // first row began in an earlier group
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 cacc = acc;
    int cur = first, cend = 0;
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      if (rs[u] < 0) break;
      if (rs[u] != cur) {  // cur ends inside this group
        if (cont && cur == first) {
          cacc = acc;
          cend = 1;
        } else {
          store(cur, acc);
        }
        acc = make_float4(0.f, 0.f, 0.f, 0.f);
        cur = rs[u];
      }
      acc = gmr::f4_fma(vs[u], xs[u], acc);
    }
    // cur = last row of the group (or -1 if empty)
    const bool last_open = cur >= 0 && cur == next_row;  // continues into the next group
    if (cur >= 0 && !last_open) {
      if (cont && cur == first) {  // the whole group is the tail of a row begun earlier
        cacc = acc;
        cend = 1;
      } else {
        store(cur, acc);
      }
    }
    const bool whole = cont && cur == first && last_open;  // group inside one spanning row
    if (whole) cacc = acc;
    if (sub == 0) {
      s_crow[wid][grp] = cont ? first : -1;
      s_cend[wid][grp] = cend;
    }
    s_cacc[wid][grp][sub] = cacc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the group where a spanning row starts adds the continuations of the next groups, in order
    if (last_open && !(cont && cur == first)) {
      float4 s = acc;
      for (int j = grp + 1; j < NG; ++j) {
        if (s_crow[wid][j] != cur) break;
        s = gmr::f4_add(s, s_cacc[wid][j][sub]);
        if (s_cend[wid][j]) break;
      }
      store(cur, s);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

}  // namespace

static inline int lane_l(int32_t seg_nnz) {  // longest short row of a lane plan, 0 if seg_nnz is invalid
  const int L = seg_nnz & 0xFFFF;
  if ((seg_nnz & ~0xFFFF) == (GMR_SPMM_LANE_PLAN | GMR_SPMM_PACKED)) return L == 32 ? L : 0;
  return (seg_nnz & ~0xFFFF) == GMR_SPMM_LANE_PLAN && (L == 32 || L == 64 || L == 128) ? L : 0;
}
static inline bool lane_packed(int32_t seg_nnz) { return (seg_nnz & GMR_SPMM_PACKED) != 0; }
static inline int lane_hb(int L) { return L == 32 ? 26 : L == 64 ? 25 : 24; }  // hub buckets = 31 - log2(L)

static int lane_wpx_cap() {  // workgroups per XCD of a lane-plan launch (GMR_SPMM_WPX overrides, for tuning)
  static const int cap = [] {
    const char* s = getenv("GMR_SPMM_WPX");
    const int v = s ? atoi(s) : 0;
    return v > 0 && v <= 1024 ? v : 512;
  }();
  return cap;
}

static int lane_lpr(int n_blocks) {  // GMR_SPMM_LPR = 4 / 8 overrides (tuning); row-major X only
  static const int ov = [] {
    const char* s = getenv("GMR_SPMM_LPR");
    const int v = s ? atoi(s) : 0;
    return v == 4 || v == 8 ? v : 0;
  }();
  // 16-column slices below d = 256: 32-column ones (full 128-byte lines, 2 XCDs per slice) win
  // 5-10 % at d = 128 in isolation (profiles/r01h_spmm_lpr_bench.txt) but lose 20-45 % inside the
  // DiffMM step, next to the side-stream products (rocprof r01j); d = 256 takes 32 columns (S <= 8)
  return n_blocks == 4 ? 8 : ov ? ov : 4;
}

// GMR_SPMM_NT: 1 = non-temporal Y stores (default: the output rows stream past L2 instead of
// evicting the XCD's X slice; -5..-16 % on the baby graphs, profiles/r02i_spmm_nt.txt),
// 2 = non-temporal index loads as well (no gain measured), 0 = plain stores
static int lane_nt() {
  static const int nt = [] {
    const char* s = getenv("GMR_SPMM_NT");
    const int v = s ? atoi(s) : 1;
    return v >= 0 && v <= 3 ? v : 1;
  }();
  return nt;
}

static int lane_eb() {  // GMR_SPMM_EB = 16: 16 gathers in flight per lane group and batch (tuning)
  static const int eb = [] {
    const char* s = getenv("GMR_SPMM_EB");
    return s && atoi(s) == 16 ? 16 : 8;
  }();
  return eb;
}

static int lane_wpx_cap_packed() {  // the packed kernel pipelines passes, so it wants fewer, longer waves
  static const int cap = [] {
    const char* s = getenv("GMR_SPMM_WPX_PACKED");
    const int v = s ? atoi(s) : 0;
    return v > 0 && v <= 1024 ? v : 512;
  }();
  return cap;
}

static inline bool is_chunk(int32_t seg_nnz) { return seg_nnz == GMR_SPMM_CHUNK_PLAN; }

extern "C" int64_t gmr_spmm_plan_words(int64_t n_rows, int64_t nnz, int32_t seg_nnz) {
  if (is_chunk(seg_nnz)) return chunk_plan_words(n_rows, nnz);
  if (seg_nnz & GMR_SPMM_LANE_PLAN) {
    if (!lane_l(seg_nnz)) return -1;
    return lane_packed(seg_nnz) ? pack_off(n_rows, nnz) + 2 * nnz : lane_tab_off(n_rows, nnz);
  }
  if (seg_nnz <= 0) return -1;
  if (seg_nnz >= 512) return kPlanHdr + 2 * (blk_max_blocks(n_rows, nnz, seg_nnz) + 1);
  return kPlanHdr + 4 * plan_max_seg(n_rows, nnz, seg_nnz) + 3 * plan_max_fix(n_rows, nnz, seg_nnz);
}

extern "C" int64_t gmr_spmm_partial_rows(int64_t n_rows, int64_t nnz, int32_t seg_nnz) {
  if (is_chunk(seg_nnz)) return 1;  // spanning rows meet in LDS
  // split hub rows: one 256-float partial row per segment (lane_fix_kernel)
  if (seg_nnz & GMR_SPMM_LANE_PLAN) return lane_l(seg_nnz) ? 2 * (nnz / kHubSeg) + 2 : -1;
  if (seg_nnz <= 0) return -1;
  if (seg_nnz >= 512) return 1;  // the blocked variant combines in LDS
  return 2 * ((nnz + seg_nnz - 1) / seg_nnz) + 2;
}

extern "C" int gmr_spmm_plan_build_split(const int32_t* rowptr, int64_t n_rows, int64_t nnz, int32_t seg_nnz,
                                         int64_t class_split, int32_t* plan, void* stream);
extern "C" int gmr_spmm_plan_build(const int32_t* rowptr, int64_t n_rows, int64_t nnz, int32_t seg_nnz,
                                   int32_t* plan, void* stream) {
  return gmr_spmm_plan_build_split(rowptr, n_rows, nnz, seg_nnz, 0, plan, stream);
}

extern "C" int gmr_spmm_plan_build_split(const int32_t* rowptr, int64_t n_rows, int64_t nnz, int32_t seg_nnz,
                                         int64_t class_split, int32_t* plan, void* stream) {
  GMR_ARG(rowptr && plan, "null pointer");
  GMR_ARG(class_split >= 0 && class_split <= n_rows, "class_split must be in [0, n_rows]");
  GMR_ARG(class_split == 0 || ((seg_nnz & GMR_SPMM_LANE_PLAN) && !lane_packed(seg_nnz)),
          "row classes need a non-packed lane plan");
  GMR_ARG(n_rows > 0 && n_rows < (1ll << 31) && nnz >= 0 && nnz < (1ll << 31), "bad size");
  if (is_chunk(seg_nnz)) {
    GMR_ARG(((uintptr_t)plan & 15) == 0, "plan must be 16-byte aligned");
    hipLaunchKernelGGL(chunk_plan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, rowptr, (int)n_rows, nnz, plan);
    GMR_LAUNCHED();
    return GMR_OK;
  }
  if (seg_nnz & GMR_SPMM_LANE_PLAN) {
    const int L = lane_l(seg_nnz);
    GMR_ARG(L, "lane plans take seg_nnz = GMR_SPMM_LANE_PLAN | 32, 64 or 128 (packed: 32)");
    GMR_ARG(((uintptr_t)plan & 15) == 0, "plan must be 16-byte aligned");
    hipLaunchKernelGGL(lane_plan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, rowptr, (int)n_rows, nnz, L,
                       lane_hb(L), (int)lane_packed(seg_nnz), (int)class_split, plan);
    GMR_LAUNCHED();
    return GMR_OK;
  }
  GMR_ARG((seg_nnz >= 64 && seg_nnz < 512 && seg_nnz % 64 == 0) || (seg_nnz >= 512 && seg_nnz <= 8192),
          "seg_nnz: a multiple of 64 below 512 (segment plan) or 512..8192 (blocked plan)");
  GMR_ARG(n_rows < (1 << 30), "n_rows too large");
  if (seg_nnz >= 512) {
    GMR_ARG(seg_nnz <= 8192, "blocked plans take seg_nnz <= 8192");
    hipLaunchKernelGGL(blk_plan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, rowptr, (int)n_rows, seg_nnz,
                       (int)blk_max_blocks(n_rows, nnz, seg_nnz), plan);
    GMR_LAUNCHED();
    return GMR_OK;
  }
  PlanView pv = plan_view(plan, n_rows, nnz, seg_nnz);
  hipLaunchKernelGGL(plan_build_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, rowptr, (int)n_rows, seg_nnz,
                     pv);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_spmm_plan_pack(const int32_t* rowptr, const int32_t* col, const float* val, int64_t n_rows,
                                  int64_t nnz, int32_t seg_nnz, int32_t* plan, void* stream) {
  GMR_ARG(plan && (nnz == 0 || (col && val)), "null pointer");
  GMR_ARG(n_rows > 0 && n_rows < (1ll << 29) && nnz >= 0 && nnz < (1ll << 31), "bad size");
  if (is_chunk(seg_nnz)) {
    GMR_ARG(rowptr, "chunk plans are packed from the CSR: rowptr needed");
    const int grid = (int)std::min<int64_t>((n_rows + 255) / 256, 2048);
    hipLaunchKernelGGL(chunk_pack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, rowptr, col, val, (int)n_rows,
                       nnz, plan);
    GMR_LAUNCHED();
    return GMR_OK;
  }
  GMR_ARG(lane_l(seg_nnz) && lane_packed(seg_nnz), "not a packed lane plan");
  const int grid = (int)std::min<int64_t>((n_rows + 255) / 256, 2048);
  hipLaunchKernelGGL(lane_pack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, col, val, (int)n_rows, nnz, plan);
  GMR_LAUNCHED();
  return GMR_OK;
}

static int lane_launch(const int32_t* col, const float* val, int64_t n_rows, int64_t nnz, const int32_t* plan,
                       int32_t seg_nnz, int32_t n_blocks, const Src& s, float alpha, float beta, const Dst& d,
                       float* partial, int32_t flags, hipStream_t st0);
static Dst dst_rowmajor(float* y, int64_t ldy, int n_blocks) {
  Dst d;
  for (int b = 0; b < 4; ++b) {
    d.y[b] = y + 64 * (b < n_blocks ? b : 0);
    d.ld[b] = ldy;
  }
  return d;
}

extern "C" int gmr_spmm_panel_f32(const int32_t* col, const float* val, int64_t n_rows, int64_t nnz,
                                  const int32_t* plan, int32_t seg_nnz, int32_t n_blocks, const float* x_panel,
                                  int64_t panel_rows, float alpha, float beta, float* y, int64_t ldy, float* partial,
                                  int32_t flags, void* stream) {
  GMR_ARG(plan && y && x_panel && (nnz == 0 || (col && val)), "null pointer");
  GMR_ARG(lane_l(seg_nnz) || is_chunk(seg_nnz), "column-panel sources need a lane or chunk plan");
  GMR_ARG(n_blocks == 1 || n_blocks == 2 || n_blocks == 4, "n_blocks must be 1, 2 or 4");
  GMR_ARG(n_rows > 0 && panel_rows > 0 && ldy >= 64 * n_blocks && ldy % 4 == 0, "bad shape");
  GMR_ARG((((uintptr_t)y | (uintptr_t)x_panel | (uintptr_t)plan) & 15) == 0, "pointers must be 16-byte aligned");
  Src s;
  for (int b = 0; b < 4; ++b) {
    s.lo[b] = s.hi[b] = x_panel;
    s.ld_lo[b] = s.ld_hi[b] = 0;
  }
  s.split = panel_rows;
  s.panel_rows = panel_rows;
  return lane_launch(col, val, n_rows, nnz, plan, seg_nnz, n_blocks, s, alpha, beta, dst_rowmajor(y, ldy, n_blocks),
                     partial, flags, (hipStream_t)stream);
}

extern "C" int gmr_spmm_plan_info(const int32_t* plan, int32_t* host_hdr, void* stream) {
  GMR_ARG(plan && host_hdr, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemcpyAsync(host_hdr, plan, sizeof(int32_t) * kPlanHdr, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return gmr::hip_status(__func__, e);
  return GMR_OK;
}

static int chunk_wpx_cap() {  // workgroups per XCD of a chunk-plan launch (GMR_SPMM_CHUNK_WPX: tuning)
  static const int cap = [] {
    const char* s = getenv("GMR_SPMM_CHUNK_WPX");
    const int v = s ? atoi(s) : 0;
    return v > 0 && v <= 1024 ? v : 32;
  }();
  return cap;
}

static int chunk_launch(const int32_t* col, const float* val, int64_t n_rows, int64_t nnz, const int32_t* plan,
                        int32_t n_blocks, const Src& s, float alpha, float beta, const Dst& d, hipStream_t st0) {
  const int lpr = n_blocks == 4 ? 8 : 4;  // slices of 16 (d = 64, 128) or 32 (d = 256) columns
  const int S = 16 * n_blocks / lpr;
  const int64_t tasks = nnz / kChunkTask + 1;  // about one wave-task per 128 entries
  const int64_t waves = (tasks + (8 / S) - 1) / (8 / S);
  const int wpx = (int)std::max<int64_t>(1, std::min<int64_t>((waves + kChunkThreads / 64 - 1) / (kChunkThreads / 64),
                                                              chunk_wpx_cap()));
  const dim3 grid((unsigned)(8 * wpx));
  if (lpr == 8)
    hipLaunchKernelGGL(spmm_chunk_kernel<8>, grid, dim3(kChunkThreads), 0, st0, col, val, plan, (int)n_rows, nnz, S, wpx,
                       s, alpha, beta, d);
  else
    hipLaunchKernelGGL(spmm_chunk_kernel<4>, grid, dim3(kChunkThreads), 0, st0, col, val, plan, (int)n_rows, nnz, S, wpx,
                       s, alpha, beta, d);
  GMR_LAUNCHED();
  return GMR_OK;
}

// column slices S and workgroups per XCD of a lane-plan product
static void lane_grid(int64_t n_rows, int32_t n_blocks, int lpr, bool packed, int& S, int& wpx) {
  S = 16 * n_blocks / lpr;  // column slices: 4 (d = 64), 8 (d = 128, 256)
  const int64_t waves = (n_rows + 64 / lpr - 1) / (64 / lpr) / (8 / S) + 1;  // one pass over the rows
  const int cap = packed ? lane_wpx_cap_packed() : lane_wpx_cap();
  wpx = (int)std::max<int64_t>(1, std::min<int64_t>((waves + 3) / 4, cap));
}

static int lane_launch(const int32_t* col, const float* val, int64_t n_rows, int64_t nnz, const int32_t* plan,
                       int32_t seg_nnz, int32_t n_blocks, const Src& s, float alpha, float beta, const Dst& d,
                       float* partial, int32_t flags, hipStream_t st0) {
  if (is_chunk(seg_nnz)) return chunk_launch(col, val, n_rows, nnz, plan, n_blocks, s, alpha, beta, d, st0);
  // lanes per row: a slice is 4 * lpr columns (column panels are 16 wide below d = 256)
  const int lpr = s.panel_rows > 0 ? (n_blocks == 4 ? 8 : 4) : lane_lpr(n_blocks);
  const bool packed = lane_packed(seg_nnz);
  int S, wpx;
  lane_grid(n_rows, n_blocks, lpr, packed, S, wpx);
  const dim3 grid((unsigned)(8 * wpx));
#define GMR_LANE_LAUNCH(LPRV, PK, EBV)                                                                      \
  hipLaunchKernelGGL((spmm_lane_kernel<LPRV, PK, EBV>), grid, dim3(kLaneThreads), 0, st0, col, val, plan, S, wpx, \
                   s, alpha, beta, d, (int)n_rows, nnz, partial, lane_nt())
  const bool wide = lane_eb() == 16;  // entries gathered per lane group and batch
  if (lpr == 8) {
    if (packed) { if (wide) GMR_LANE_LAUNCH(8, true, 16); else GMR_LANE_LAUNCH(8, true, 8); }
    else { if (wide) GMR_LANE_LAUNCH(8, false, 16); else GMR_LANE_LAUNCH(8, false, 8); }
  } else {
    if (packed) { if (wide) GMR_LANE_LAUNCH(4, true, 16); else GMR_LANE_LAUNCH(4, true, 8); }
    else { if (wide) GMR_LANE_LAUNCH(4, false, 16); else GMR_LANE_LAUNCH(4, false, 8); }
  }
#undef GMR_LANE_LAUNCH
  GMR_LAUNCHED();
  if (flags & GMR_SPMM_HUB_FIXUP) {  // the plan split hub rows: add their segment partials in order
    if (!partial) {
      gmr::set_error("gmr_spmm", "plan has split hub rows (GMR_SPMM_HUB_FIXUP): partial buffer needed");
      return GMR_ERR_ARG;
    }
    hipLaunchKernelGGL(lane_fix_kernel, dim3(32), dim3(256), 0, st0, plan, n_rows, nnz, 64 * n_blocks, partial, alpha,
                       beta, d);
    GMR_LAUNCHED();
  }
  return GMR_OK;
}

extern "C" int gmr_spmm_multi_f32(const int32_t* col, const float* val, int64_t n_rows, int64_t nnz,
                                  const int32_t* plan, int32_t seg_nnz, int32_t n_blocks, const float* const* x_lo,
                                  const int64_t* ld_lo, const float* const* x_hi, const int64_t* ld_hi, int64_t split,
                                  float alpha, float beta, float* const* y_blocks, const int64_t* ld_y,
                                  float* partial, int32_t flags, void* stream) {
  GMR_ARG(plan && x_lo && ld_lo && y_blocks && ld_y && (nnz == 0 || (col && val)), "null pointer");
  GMR_ARG(lane_l(seg_nnz) || is_chunk(seg_nnz), "per-block outputs need a lane or chunk plan");
  GMR_ARG(n_blocks == 1 || n_blocks == 2 || n_blocks == 4, "n_blocks must be 1, 2 or 4");
  GMR_ARG(n_rows > 0 && nnz >= 0 && ((uintptr_t)plan & 15) == 0, "bad shape");
  Src s;
  Dst d;
  s.split = split;
  s.panel_rows = 0;
  for (int b = 0; b < 4; ++b) {
    const int bb = b < n_blocks ? b : 0;
    s.lo[b] = x_lo[bb];
    s.ld_lo[b] = ld_lo[bb];
    s.hi[b] = (split < n_rows && x_hi) ? x_hi[bb] : x_lo[bb];
    s.ld_hi[b] = (split < n_rows && ld_hi) ? ld_hi[bb] : ld_lo[bb];
    d.y[b] = y_blocks[bb];
    d.ld[b] = ld_y[bb];
    GMR_ARG(s.lo[b] && s.hi[b] && d.y[b], "null block");
    GMR_ARG((((uintptr_t)s.lo[b] | (uintptr_t)s.hi[b] | (uintptr_t)d.y[b]) & 15) == 0, "blocks must be 16-byte aligned");
    GMR_ARG(s.ld_lo[b] % 4 == 0 && s.ld_hi[b] % 4 == 0 && d.ld[b] % 4 == 0 && d.ld[b] >= 64, "bad block stride");
  }
  return lane_launch(col, val, n_rows, nnz, plan, seg_nnz, n_blocks, s, alpha, beta, d, partial, flags,
                     (hipStream_t)stream);
}

extern "C" int gmr_spmm_jobs_f32(int32_t n_jobs, const gmr_spmm_job* jobs, void* stream) {
  GMR_ARG(jobs && n_jobs >= 1 && n_jobs <= kMaxJobs, "1 to 4 jobs");
  LaneJobs J;
  int lpr = 0, off = 0;
  bool any_fix = false;
  for (int q = 0; q < n_jobs; ++q) {
    const gmr_spmm_job& g = jobs[q];
    GMR_ARG(g.plan && (g.nnz == 0 || (g.col && g.val)), "job: null pointer");
    GMR_ARG(lane_l(g.seg_nnz), "job: jobs take lane plans (GMR_SPMM_LANE_PLAN [| GMR_SPMM_PACKED] | L)");
    GMR_ARG(g.n_blocks == 1 || g.n_blocks == 2 || g.n_blocks == 4, "job: n_blocks must be 1, 2 or 4");
    GMR_ARG(g.n_rows > 0 && g.n_rows < (1ll << 31) && g.nnz >= 0 && ((uintptr_t)g.plan & 15) == 0, "job: bad shape");
    const int l = lane_lpr(g.n_blocks);
    GMR_ARG(lpr == 0 || l == lpr, "jobs of one launch need one lane width (n_blocks 1 and 2 together, 4 alone)");
    lpr = l;
    LaneJob& j = J.j[q];
    j.col = g.col;
    j.val = g.val;
    j.plan = g.plan;
    j.part = g.partial;
    j.nnz = g.nnz;
    j.alpha = g.alpha;
    j.beta = g.beta;
    j.n_rows = (int)g.n_rows;
    j.packed = lane_packed(g.seg_nnz) ? 1 : 0;
    j.fix = (g.flags & GMR_SPMM_HUB_FIXUP) ? 1 : 0;
    j.ncols = 64 * g.n_blocks;
    j.nt = lane_nt();
    GMR_ARG(!j.fix || g.partial, "job: plan has split hub rows (GMR_SPMM_HUB_FIXUP): partial buffer needed");
    any_fix = any_fix || j.fix;
    j.src.split = g.split;
    j.src.panel_rows = 0;
    for (int b = 0; b < 4; ++b) {
      const int bb = b < g.n_blocks ? b : 0;
      j.src.lo[b] = g.x_lo[bb];
      j.src.ld_lo[b] = g.ld_lo[bb];
      const bool two = g.split < g.n_rows && g.x_hi[bb];
      j.src.hi[b] = two ? g.x_hi[bb] : g.x_lo[bb];
      j.src.ld_hi[b] = two ? g.ld_hi[bb] : g.ld_lo[bb];
      j.dst.y[b] = g.y[bb];
      j.dst.ld[b] = g.ld_y[bb];
      GMR_ARG(j.src.lo[b] && j.src.hi[b] && j.dst.y[b], "job: null block");
      GMR_ARG((((uintptr_t)j.src.lo[b] | (uintptr_t)j.src.hi[b] | (uintptr_t)j.dst.y[b]) & 15) == 0,
              "job: blocks must be 16-byte aligned");
      GMR_ARG(j.src.ld_lo[b] % 4 == 0 && j.src.ld_hi[b] % 4 == 0 && j.dst.ld[b] % 4 == 0 && j.dst.ld[b] >= 64,
              "job: bad block stride");
    }
    lane_grid(g.n_rows, g.n_blocks, lpr, j.packed, j.S, j.wpx);
    J.off[q] = off;
    off += 8 * j.wpx;
  }
  for (int q = n_jobs; q <= kMaxJobs; ++q) J.off[q] = off;
  J.n = n_jobs;
  hipStream_t st = (hipStream_t)stream;
  const bool wide = lane_eb() == 16;
  if (lpr == 8) {
    if (wide) hipLaunchKernelGGL((spmm_lane_jobs_kernel<8, 16>), dim3(off), dim3(kLaneThreads), 0, st, J);
    else hipLaunchKernelGGL((spmm_lane_jobs_kernel<8, 8>), dim3(off), dim3(kLaneThreads), 0, st, J);
  } else {
    if (wide) hipLaunchKernelGGL((spmm_lane_jobs_kernel<4, 16>), dim3(off), dim3(kLaneThreads), 0, st, J);
    else hipLaunchKernelGGL((spmm_lane_jobs_kernel<4, 8>), dim3(off), dim3(kLaneThreads), 0, st, J);
  }
  GMR_LAUNCHED();
  if (any_fix) {
    hipLaunchKernelGGL(lane_fix_jobs_kernel, dim3(32), dim3(256), 0, st, J);
    GMR_LAUNCHED();
  }
  return GMR_OK;
}

extern "C" int gmr_spmm_csr_f32(const int32_t* rowptr, const int32_t* col, const float* val, int64_t n_rows,
                                int64_t nnz, const int32_t* plan, int32_t seg_nnz, float* partial, int32_t n_blocks,
                                const float* const* x_lo, const int64_t* ld_lo, const float* const* x_hi,
                                const int64_t* ld_hi, int64_t split, float alpha, float beta, float* y, int64_t ldy,
                                int32_t flags, void* stream) {
  GMR_ARG(rowptr && (nnz == 0 || (col && val)) && plan && y && x_lo && ld_lo, "null pointer");
  GMR_ARG(n_blocks == 1 || n_blocks == 2 || n_blocks == 4, "n_blocks must be 1, 2 or 4");
  GMR_ARG(n_rows > 0 && nnz >= 0 && ldy >= 64 * n_blocks && ldy % 4 == 0, "bad shape");
  GMR_ARG(((uintptr_t)y & 15) == 0, "y must be 16-byte aligned");
  Src s;
  s.split = split;
  s.panel_rows = 0;
  for (int b = 0; b < 4; ++b) {
    int bb = b < n_blocks ? b : 0;
    s.lo[b] = x_lo[bb];
    s.ld_lo[b] = ld_lo[bb];
    s.hi[b] = (split < n_rows && x_hi) ? x_hi[bb] : x_lo[bb];
    s.ld_hi[b] = (split < n_rows && ld_hi) ? ld_hi[bb] : ld_lo[bb];
    GMR_ARG(s.lo[b] && s.hi[b], "null source block");
    GMR_ARG(((uintptr_t)s.lo[b] & 15) == 0 && ((uintptr_t)s.hi[b] & 15) == 0, "sources must be 16-byte aligned");
    GMR_ARG(s.ld_lo[b] % 4 == 0 && s.ld_hi[b] % 4 == 0, "source ld must be a multiple of 4");
  }
  hipStream_t st0 = (hipStream_t)stream;
  if (is_chunk(seg_nnz)) {
    GMR_ARG(((uintptr_t)plan & 15) == 0, "plan must be 16-byte aligned");
    return lane_launch(col, val, n_rows, nnz, plan, seg_nnz, n_blocks, s, alpha, beta, dst_rowmajor(y, ldy, n_blocks),
                       partial, flags, st0);
  }
  if (seg_nnz & GMR_SPMM_LANE_PLAN) {
    GMR_ARG(lane_l(seg_nnz), "bad lane plan seg_nnz");
    GMR_ARG(((uintptr_t)plan & 15) == 0, "plan must be 16-byte aligned");
    return lane_launch(col, val, n_rows, nnz, plan, seg_nnz, n_blocks, s, alpha, beta, dst_rowmajor(y, ldy, n_blocks),
                       partial, flags, st0);
  }
  if (seg_nnz >= 512) {
    const int64_t mb = blk_max_blocks(n_rows, nnz, seg_nnz);
    const int rp = 8 / (2 * n_blocks);
    const dim3 grid((unsigned)(8 * ((mb + rp - 1) / rp)));
    const size_t lds = sizeof(int) * (size_t)(seg_nnz + 1);
    switch (n_blocks) {
      case 1:
        hipLaunchKernelGGL(spmm_blk_kernel<1>, grid, dim3(kBlkThreads), lds, st0, rowptr, col, val, plan, seg_nnz,
                           (int)mb, s, alpha, beta, y, ldy);
        break;
      case 2:
        hipLaunchKernelGGL(spmm_blk_kernel<2>, grid, dim3(kBlkThreads), lds, st0, rowptr, col, val, plan, seg_nnz,
                           (int)mb, s, alpha, beta, y, ldy);
        break;
      default:
        hipLaunchKernelGGL(spmm_blk_kernel<4>, grid, dim3(kBlkThreads), lds, st0, rowptr, col, val, plan, seg_nnz,
                           (int)mb, s, alpha, beta, y, ldy);
        break;
    }
    GMR_LAUNCHED();
    return GMR_OK;
  }
  PlanView pv = plan_view(const_cast<int32_t*>(plan), n_rows, nnz, seg_nnz);
  const int64_t max_seg = plan_max_seg(n_rows, nnz, seg_nnz);
  const int64_t max_fix = plan_max_fix(n_rows, nnz, seg_nnz);
  hipStream_t st = (hipStream_t)stream;
  const int grid = gmr::grid_for(max_seg, 4);
  const int fix_grid = gmr::grid_for(max_fix * 16 * n_blocks, 256);
  const bool fix = !(flags & GMR_SPMM_NO_SPLIT_ROWS);
#define GMR_SPMM_LAUNCH(NBV)                                                                                       \
  hipLaunchKernelGGL(spmm_seg_kernel<NBV>, dim3(grid), dim3(256), 0, st, col, val, pv, s, alpha, beta, y, ldy,     \
                     partial);                                                                                   \
  GMR_LAUNCHED();                                                                                                \
  if (fix)                                                                                                       \
    hipLaunchKernelGGL(spmm_fix_kernel<NBV>, dim3(fix_grid), dim3(256), 0, st, pv, alpha, beta, y, ldy, partial);
  switch (n_blocks) {
    case 1: GMR_SPMM_LAUNCH(1); break;
    case 2: GMR_SPMM_LAUNCH(2); break;
    default: GMR_SPMM_LAUNCH(4); break;
  }
#undef GMR_SPMM_LAUNCH
  GMR_LAUNCHED();
  return GMR_OK;
}
