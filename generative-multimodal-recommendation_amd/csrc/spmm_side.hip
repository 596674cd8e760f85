// K1 — side-split CSR SpMM for the bipartite graph-conv adjacencies (gfx950).
//
// Replaces torch.spmm / torch.sparse.mm on DiffMM's norm_adj (reference models/diffmm.py:88-107,
// 136-191, 285) and the rebuilt UI graphs (common/trainer.py:464-485).  Y = alpha * A X + beta * Y,
// A an n x n CSR whose rows split at `split` into a user side [0, split) and an item side
// [split, n): a user row of norm_adj = [[0, R], [R^T, 0]] reads only item rows of X and an item row
// only user rows (a rebuilt UI graph adds one self loop per row).
//
// Measured on MI355X (scripts/micro/side_spmm.hip, profiles/r03_spmm_side_micro.txt): the graph-conv
// SpMM is bound by the L2's request rate (~14 line requests per clock per XCD) and by two
// latency tails, not by HBM bytes.  So:
//   * XCD groups: the launch's XCDs are split into (side, 32-column slice) groups (d = 128: 4 slices
//     x 2 sides = one group per XCD; d = 64: 2 XCDs per group; d = 256: two phases per XCD).  An
//     XCD's L2 then holds only the OTHER side's 128-byte slice of X (items 7,050 x 128 B = 0.9 MB,
//     users 19,445 x 128 B = 2.5 MB at baby) and every gather is ONE whole line;
//   * entry-stream tasks: each side's CSR entries are cut, at row boundaries, into tasks of <= T
//     consecutive entries (several whole rows); a lane group of 8 lanes (32 columns = 8 x float4)
//     streams a task EB entries at a time with the next EB (col, val) pairs in flight, crossing row
//     ends inside the stream (a packed entry carries a row-end bit), so no per-row descriptor round
//     trip and no idle gather slots on short rows;
//   * hub rows (degree > T: the Zipf-popular items) are cut into pieces of <= T entries, each an
//     ordinary task whose sum goes to a partial row (write-through sc1 stores); the lane group whose
//     agent-scope counter add comes last sums the pieces IN PIECE ORDER (sc1 loads) and writes the row,
//     then re-arms the counter: one launch, deterministic sums (the MI355X_MICROARCH.md hand-off form
//     "agent-scope atomic add ... the workgroup whose add came last ... sc1 stores and loads");
//   * a short-row entry sum runs in CSR order from zero (acc = fma(v, x, acc)), the order of the lane
//     plan's short rows; hub rows add their pieces in order.
// Plan (int32 words, built on the host by gmr_spmm_side_plan_build, entries packed on the device by
// gmr_spmm_side_pack): header[16], tasks int4 {beg, end, first row, slot | -1} (side 0 then side 1),
// empty rows, hubs int4 {row, first slot, pieces, 0}, slot -> hub, packed int2 {col | last << 31, val}.
// Scratch (caller-owned, zeroed once): kSideCounters ints of per-(hub, slice) counters, then one
// 256-float partial row per slot.
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "gmr_common.h"

namespace {

constexpr int kSideHdr = 16;
constexpr int kSideMagic = 0x53494445;  // 'SIDE'
constexpr int kSideThreads = 256;
constexpr int64_t kSideCounterWords = 8;  // counters per hub (one per 32-column slice, d <= 256)

enum { H_MAGIC, H_NROWS, H_SPLIT, H_T, H_TASK, H_NT0, H_NT1, H_EMPTY, H_NE0, H_NE1, H_HUB, H_NHUB, H_SLOT, H_NSLOT,
       H_PACKED, H_NNZ };

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct SideSrc {
  const float* lo[4];
  const float* hi[4];
  int64_t ld_lo[4];
  int64_t ld_hi[4];
  int64_t split;
};
struct SideDst {
  float* y[4];
  int64_t ld[4];
};

__device__ __forceinline__ float4 f4_zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// NS = 32-column slices of the product (d = 32 NS), EB = entries in flight per lane group
template <int EB, int NS>
__global__ void __launch_bounds__(kSideThreads) spmm_side_kernel(const int* __restrict__ plan, SideSrc src,
                                                                  float alpha, float beta, SideDst dst,
                                                                  float* __restrict__ scratch, int wpx, int nt) {
  constexpr int G = 2 * NS;                    // (side, slice) groups
  constexpr int PHASES = G > 8 ? G / 8 : 1;    // groups per XCD, one after the other
  constexpr int P = G >= 8 ? 1 : 8 / G;        // XCDs per group
  constexpr int EPL = EB / 8;                  // packed entries per lane per round
  const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane >> 3, sub = lane & 7, gbase = grp * 8;
  const int* hdr = plan;
  const int4* __restrict__ tasks = reinterpret_cast<const int4*>(plan + hdr[H_TASK]);
  const int* __restrict__ empty = plan + hdr[H_EMPTY];
  const int4* __restrict__ hubs = reinterpret_cast<const int4*>(plan + hdr[H_HUB]);
  const int* __restrict__ slotmap = plan + hdr[H_SLOT];
  const int2* __restrict__ packed = reinterpret_cast<const int2*>(plan + hdr[H_PACKED]);
  int* counters = reinterpret_cast<int*>(scratch);
  float* part = scratch + ((int64_t)hdr[H_NHUB] * kSideCounterWords + 3) / 4 * 4;
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(part, 0, 0x7fffffff, 0x00020000);
  const int64_t split = src.split;
#pragma unroll 1
  for (int ph = 0; ph < PHASES; ++ph) {
    const int g = G >= 8 ? xcd + 8 * ph : xcd % G;
    const int part_i = G >= 8 ? 0 : xcd / G;
    const int side = g / NS, slice = g % NS;
    const int c0 = slice * 32 + sub * 4;       // this lane's 4 columns
    const int blk = c0 >> 6, cin = c0 & 63;
    const float* __restrict__ lo = src.lo[blk] + cin;
    const float* __restrict__ hi = src.hi[blk] + cin;
    const int64_t ldl = src.ld_lo[blk], ldh = src.ld_hi[blk];
    float* __restrict__ yc = dst.y[blk] + cin;
    const int64_t ldy = dst.ld[blk];
    const int n_lg = P * wpx * (kSideThreads / 8);
    const int lg = (part_i * wpx + k) * (kSideThreads / 8) + wid * 8 + grp;
    auto store = [&](int row, float4 acc) {
      float* yp = yc + (int64_t)row * ldy;
      float4 o = gmr::f4_scale(alpha, acc);
      if (beta != 0.f) o = gmr::f4_fma(beta, *reinterpret_cast<const float4*>(yp), o);
      if (nt) {
        f32x4 ov = {o.x, o.y, o.z, o.w};
        __builtin_nontemporal_store(ov, reinterpret_cast<f32x4*>(yp));
      } else {
        *reinterpret_cast<float4*>(yp) = o;
      }
    };
    // empty rows of this side: Y = beta Y (alpha A X is zero there)
    const int e0 = side == 0 ? 0 : hdr[H_NE0], ne = side == 0 ? hdr[H_NE0] : hdr[H_NE1];
    for (int i = lg; i < ne; i += n_lg) store(empty[e0 + i], f4_zero());
    const int t0 = side == 0 ? 0 : hdr[H_NT0], ntk = side == 0 ? hdr[H_NT0] : hdr[H_NT1];
#pragma unroll 1
    for (int ti = lg; ti < ntk; ti += n_lg) {
      const int4 tk = tasks[t0 + ti];
      const int end = tk.y;
      int row = tk.z;
      const bool piece = tk.w >= 0;
      float4 acc = f4_zero();
      int2 rec[EPL];
#pragma unroll
      for (int q = 0; q < EPL; ++q) {
        const int i = tk.x + q * 8 + sub;
        rec[q] = i < end ? packed[i] : make_int2(0, 0);
      }
#pragma unroll 1
      for (int e = tk.x; e < end; e += EB) {
        float4 xs[EB];
        float vs[EB];
        int cs[EB];
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          cs[u] = __shfl(rec[u / 8].x, gbase + u % 8);
          vs[u] = __int_as_float(__shfl(rec[u / 8].y, gbase + u % 8));
          const int c = cs[u] & 0x7fffffff;
          xs[u] = f4_zero();
          if (e + u < end)
            xs[u] = *reinterpret_cast<const float4*>(c < split ? lo + (int64_t)c * ldl : hi + (int64_t)(c - split) * ldh);
        }
        const int en = e + EB;  // the next round's entries travel while these gathers land
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
          const int i = en + q * 8 + sub;
          rec[q] = i < end ? packed[i] : make_int2(0, 0);
        }
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          if (e + u < end) {
            acc = gmr::f4_fma(vs[u], xs[u], acc);
            if (cs[u] < 0 && !piece) {  // row end inside a whole-row task
              store(row, acc);
              ++row;
              acc = f4_zero();
            }
          }
        }
      }
      if (piece) {
        // hub piece: partial row tk.w, write-through; the last arriving piece of (hub, slice) adds
        // all pieces in order and writes the row
        const int slot = tk.w;
        f32x4 pv = {acc.x, acc.y, acc.z, acc.w};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pv), prs, (slot * 256 + c0) * 4, 0, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int h = slotmap[slot];
        const int4 hb = hubs[h];
        int* cnt = counters + (int64_t)h * kSideCounterWords + slice;
        int old = 0;
        if (sub == 0) old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = __shfl(old, gbase);
        if (old == hb.z - 1) {
          float4 s = f4_zero();
#pragma unroll 4
          for (int j = 0; j < hb.z; ++j) {
            const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(prs, ((hb.y + j) * 256 + c0) * 4, 0, 16);
            const f32x4 f = __builtin_bit_cast(f32x4, r);
            s = gmr::f4_add(s, make_float4(f.x, f.y, f.z, f.w));
          }
          store(hb.x, s);
          if (sub == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
}

// packed entries: {col | (last entry of its row) << 31, val}
__global__ void __launch_bounds__(256) side_pack_kernel(const int* __restrict__ rowptr, const int* __restrict__ col,
                                                        const float* __restrict__ val, int64_t n_rows,
                                                        int2* __restrict__ packed) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_rows; r += (int64_t)gridDim.x * blockDim.x) {
    const int beg = rowptr[r], end = rowptr[r + 1];
    for (int e = beg; e < end; ++e)
      packed[e] = make_int2(col[e] | (e == end - 1 ? (int)0x80000000u : 0), __float_as_int(val[e]));
  }
}

struct SidePlanHost {
  std::vector<int4> tasks[2], hubs;
  std::vector<int> empty[2], slotmap;
};

void side_plan_host(const int32_t* rp, int64_t n_rows, int64_t split, int T, SidePlanHost& p) {
  int slot = 0;
  for (int s = 0; s < 2; ++s) {
    const int64_t r0 = s == 0 ? 0 : split, r1 = s == 0 ? split : n_rows;
    int beg = -1, row0 = -1, cnt = 0, end = 0;
    auto flush = [&]() {
      if (beg >= 0) p.tasks[s].push_back(make_int4(beg, end, row0, -1));
      beg = -1;
      cnt = 0;
    };
    for (int64_t r = r0; r < r1; ++r) {
      const int b = rp[r], e = rp[r + 1], deg = e - b;
      if (deg == 0) {
        flush();
        p.empty[s].push_back((int)r);
      } else if (deg > T) {
        flush();
        const int pieces = (deg + T - 1) / T, pl = (deg + pieces - 1) / pieces;
        const int h = (int)p.hubs.size();
        p.hubs.push_back(make_int4((int)r, slot, pieces, 0));
        for (int j = 0; j < pieces; ++j) {
          p.tasks[s].push_back(make_int4(b + j * pl, std::min(e, b + (j + 1) * pl), (int)r, slot + j));
          p.slotmap.push_back(h);
        }
        slot += pieces;
      } else {
        if (cnt + deg > T) flush();
        if (beg < 0) {
          beg = b;
          row0 = (int)r;
        }
        cnt += deg;
        end = e;
      }
    }
    flush();
  }
}

int64_t r4(int64_t v) { return (v + 3) / 4 * 4; }

struct SideLayout {
  int64_t task, empty, hub, slot, packed, words;
};
SideLayout side_layout(const SidePlanHost& p, int64_t nnz) {
  SideLayout l;
  l.task = kSideHdr;
  l.empty = l.task + 4 * (int64_t)(p.tasks[0].size() + p.tasks[1].size());
  l.hub = r4(l.empty + (int64_t)(p.empty[0].size() + p.empty[1].size()));
  l.slot = l.hub + 4 * (int64_t)p.hubs.size();
  l.packed = r4(l.slot + (int64_t)p.slotmap.size());
  l.words = l.packed + 2 * nnz;
  return l;
}

int side_wpx() {  // workgroups per XCD (GMR_SPMM_SIDE_WPX overrides, for tuning)
  static const int v = [] {
    const char* s = getenv("GMR_SPMM_SIDE_WPX");
    const int x = s ? atoi(s) : 0;
    return x > 0 && x <= 1024 ? x : 64;
  }();
  return v;
}

int side_eb() {  // entries in flight per lane group (GMR_SPMM_SIDE_EB = 8 or 16)
  static const int v = [] {
    const char* s = getenv("GMR_SPMM_SIDE_EB");
    return s && atoi(s) == 8 ? 8 : 16;
  }();
  return v;
}

int side_nt() {  // non-temporal Y stores (GMR_SPMM_NT semantics: 0 = plain)
  static const int v = [] {
    const char* s = getenv("GMR_SPMM_NT");
    return s ? (atoi(s) & 1) : 1;
  }();
  return v;
}

template <int NS>
void side_launch(int eb, const int* plan, const SideSrc& src, float alpha, float beta, const SideDst& dst,
                 float* scratch, int wpx, int nt, hipStream_t st) {
  if (eb == 8)
    hipLaunchKernelGGL((spmm_side_kernel<8, NS>), dim3(8 * wpx), dim3(kSideThreads), 0, st, plan, src, alpha, beta, dst,
                       scratch, wpx, nt);
  else
    hipLaunchKernelGGL((spmm_side_kernel<16, NS>), dim3(8 * wpx), dim3(kSideThreads), 0, st, plan, src, alpha, beta,
                       dst, scratch, wpx, nt);
}

}  // namespace

extern "C" int64_t gmr_spmm_side_plan_words(const int32_t* rowptr_host, int64_t n_rows, int64_t split, int32_t T) {
  if (!rowptr_host || n_rows <= 0 || split < 0 || split > n_rows || T < 8 || T > 4096) return -1;
  SidePlanHost p;
  side_plan_host(rowptr_host, n_rows, split, T, p);
  return side_layout(p, rowptr_host[n_rows]).words;
}

extern "C" int gmr_spmm_side_plan_build(const int32_t* rowptr_host, int64_t n_rows, int64_t split, int32_t T,
                                        int32_t* plan_host, int64_t words) {
  GMR_ARG(rowptr_host && plan_host && n_rows > 0 && split >= 0 && split <= n_rows, "bad args");
  GMR_ARG(T >= 8 && T <= 4096, "T must be in [8, 4096]");
  GMR_ARG(n_rows < (1 << 30) && rowptr_host[n_rows] < (1ll << 31) - 1, "too large for int32 plans");
  SidePlanHost p;
  side_plan_host(rowptr_host, n_rows, split, T, p);
  const int64_t nnz = rowptr_host[n_rows];
  const SideLayout l = side_layout(p, nnz);
  GMR_ARG(words >= l.words, "plan buffer smaller than gmr_spmm_side_plan_words(...)");
  int32_t* h = plan_host;
  h[H_MAGIC] = kSideMagic;
  h[H_NROWS] = (int)n_rows;
  h[H_SPLIT] = (int)split;
  h[H_T] = T;
  h[H_TASK] = (int)l.task;
  h[H_NT0] = (int)p.tasks[0].size();
  h[H_NT1] = (int)p.tasks[1].size();
  h[H_EMPTY] = (int)l.empty;
  h[H_NE0] = (int)p.empty[0].size();
  h[H_NE1] = (int)p.empty[1].size();
  h[H_HUB] = (int)l.hub;
  h[H_NHUB] = (int)p.hubs.size();
  h[H_SLOT] = (int)l.slot;
  h[H_NSLOT] = (int)p.slotmap.size();
  h[H_PACKED] = (int)l.packed;
  h[H_NNZ] = (int)nnz;
  int4* t = reinterpret_cast<int4*>(h + l.task);
  for (int s = 0; s < 2; ++s)
    for (const int4& x : p.tasks[s]) *t++ = x;
  int* e = h + l.empty;
  for (int s = 0; s < 2; ++s)
    for (int r : p.empty[s]) *e++ = r;
  for (int64_t i = l.empty + (int64_t)(p.empty[0].size() + p.empty[1].size()); i < l.hub; ++i) h[i] = 0;
  int4* hb = reinterpret_cast<int4*>(h + l.hub);
  for (const int4& x : p.hubs) *hb++ = x;
  int* sm = h + l.slot;
  for (int x : p.slotmap) *sm++ = x;
  for (int64_t i = l.slot + (int64_t)p.slotmap.size(); i < l.packed; ++i) h[i] = 0;
  return GMR_OK;
}

extern "C" int64_t gmr_spmm_side_scratch_floats(const int32_t* plan_host) {
  if (!plan_host || plan_host[H_MAGIC] != kSideMagic) return -1;
  return r4((int64_t)plan_host[H_NHUB] * kSideCounterWords) + 256 * (int64_t)std::max(plan_host[H_NSLOT], 1);
}

extern "C" int gmr_spmm_side_pack(const int32_t* rowptr, const int32_t* col, const float* val, int64_t n_rows,
                                  int64_t nnz, int64_t packed_off, int32_t* plan, void* stream) {
  GMR_ARG(rowptr && col && val && plan && n_rows > 0 && packed_off > 0 && packed_off % 2 == 0, "bad args");
  if (nnz == 0) return GMR_OK;
  hipLaunchKernelGGL(side_pack_kernel, dim3(gmr::grid_for(n_rows, 256, 4096)), dim3(256), 0, (hipStream_t)stream,
                     rowptr, col, val, n_rows, reinterpret_cast<int2*>(plan + packed_off));
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_spmm_side_f32(const int32_t* plan, int32_t n_blocks, const float* const* x_lo, const int64_t* ld_lo,
                                 const float* const* x_hi, const int64_t* ld_hi, int64_t split, float alpha, float beta,
                                 float* const* y, const int64_t* ld_y, float* scratch, void* stream) {
  GMR_ARG(plan && scratch && x_lo && ld_lo && x_hi && ld_hi && y && ld_y, "null argument");
  GMR_ARG(n_blocks == 1 || n_blocks == 2 || n_blocks == 4, "1, 2 or 4 blocks of 64 columns");
  SideSrc s;
  SideDst d;
  for (int b = 0; b < 4; ++b) {
    const bool on = b < n_blocks;
    s.lo[b] = on ? x_lo[b] : nullptr;
    s.hi[b] = on ? x_hi[b] : nullptr;
    s.ld_lo[b] = on ? ld_lo[b] : 0;
    s.ld_hi[b] = on ? ld_hi[b] : 0;
    d.y[b] = on ? y[b] : nullptr;
    d.ld[b] = on ? ld_y[b] : 0;
    if (on) {
      GMR_ARG(s.lo[b] && s.hi[b] && d.y[b], "null block pointer");
      GMR_ARG(((uintptr_t)s.lo[b] | (uintptr_t)s.hi[b] | (uintptr_t)d.y[b]) % 16 == 0, "blocks must be 16-byte aligned");
      GMR_ARG(s.ld_lo[b] % 4 == 0 && s.ld_hi[b] % 4 == 0 && d.ld[b] % 4 == 0 && d.ld[b] >= 64,
              "leading dimensions must be multiples of 4");
    }
  }
  s.split = split;
  const hipStream_t st = (hipStream_t)stream;
  const int eb = side_eb(), wpx = side_wpx(), nt = side_nt();
  if (n_blocks == 1)
    side_launch<2>(eb, plan, s, alpha, beta, d, scratch, wpx, nt, st);
  else if (n_blocks == 2)
    side_launch<4>(eb, plan, s, alpha, beta, d, scratch, wpx, nt, st);
  else
    side_launch<8>(eb, plan, s, alpha, beta, d, scratch, wpx, nt, st);
  GMR_LAUNCHED();
  return GMR_OK;
}
