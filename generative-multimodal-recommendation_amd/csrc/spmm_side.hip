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
//   * entry-stream tasks: each side's rows of degree <= T are cut, at row boundaries, into tasks of
//     <= T consecutive CSR entries (several whole rows); a lane group of 8 lanes (32 columns = 8 x
//     float4) streams a task EB entries at a time, the next EB (col, val) pairs (and after the last
//     round the NEXT task's first ones) in flight while the gathers land, crossing row ends inside
//     the stream (a packed entry carries a row-end bit): no per-row descriptor round trip and no idle
//     gather slots on short rows;
//   * hub rows (degree > T: the Zipf-popular items) are wave tasks, longest first: blocks of <= 8 TW
//     entries whose 8 lane groups split the block evenly and meet in a xor butterfly.  A row of
//     several blocks publishes each block sum write-through (sc1); the WAVE whose agent-scope counter
//     add comes last loads all block sums (sc1, 8 lane groups in parallel), adds them in a fixed order
//     and writes the row, then re-arms the counter (the MI355X_MICROARCH.md hand-off form "agent-scope
//     atomic add ... the workgroup whose add came last ... sc1 stores and loads").  One launch; a
//     one-lane-group serial combine of many pieces was the tail (profiles/r03b_sweep.txt);
//   * a short row's sum runs in CSR order from zero (acc = fma(v, x, acc)), the order of the lane
//     plan's short rows; a hub row's sum order is fixed by its plan: deterministic.
// Plan (int32 words, built on the host by gmr_spmm_side_plan_build, entries packed on the device by
// gmr_spmm_side_pack): header[32], lane tasks int4 {beg, end, first row, -1} (side 0 then side 1),
// wave tasks int4 {beg, end, row, slot | -1}, empty rows, hubs int4 {row, first slot, blocks, 0},
// slot -> hub, packed int2 {col | last << 31, val}.
// Scratch (caller-owned, zeroed once): per-(hub, slice) counters, then one 256-float partial row
// per slot.
#include <stdlib.h>

#include <algorithm>
#include <type_traits>
#include <vector>

#include "gmr_common.h"

namespace {

constexpr int kSideHdr = 32;
constexpr int kSideMagic = 0x53494446;  // 'SIDF'
constexpr int kSideThreads = 256;
constexpr int64_t kSideCounterWords = 8;  // counters per hub (one per 32-column slice, d <= 256)

enum { H_MAGIC, H_NROWS, H_SPLIT, H_T, H_TASK, H_NT0, H_NT1, H_EMPTY, H_NE0, H_NE1, H_HUB, H_NHUB, H_SLOT, H_NSLOT,
       H_PACKED, H_NNZ, H_WAVE, H_NW0, H_NW1, H_TW,
       // degree-class plan (Tw flag GMR_SIDE_CLASSES): short rows grouped by degree
       H_DC, H_CLS, H_PERM, H_DSTO, H_NSR, H_PACKB, H_NSE };
// rows of the degree-class plan: degree 1 .. 16 (longer rows are hub rows: classes up to 48 with several
// gather rounds per lane-group row measured slower on the item side, profiles/r04h_spmm_classes_probe.txt)
constexpr int kSideDcMax = 16;
constexpr int kSideDcRound = 16; // entries per lane-group gather round; rows of degree <= 16 share one round
__host__ __device__ constexpr int dc_rows_per_task(int d) { return d <= kSideDcRound ? kSideDcRound / d : 1; }

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
  const float* z[4];  // the beta term's source (Y = alpha A X + beta Z; z = y for the in-place form)
  int64_t ldz[4];
};

__device__ __forceinline__ float4 f4_zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ float4 shx(float4 v, int m) { return gmr::shfl_xor_f4(v, m); }
// sum over the 8 lane groups of a wave (xor butterfly: every group ends with the same bits)
__device__ __forceinline__ float4 wave_groups_sum(float4 a) {
  a = gmr::f4_add(a, shx(a, 8));
  a = gmr::f4_add(a, shx(a, 16));
  return gmr::f4_add(a, shx(a, 32));
}

// lane J of each 8-lane group to the whole group, in registers: DPP row_newbcast (gfx950) broadcasts lane
// n of each 16-lane row, so two of them (lanes J and 8 + J) and a select by half-row give each group its
// own lane J (a __shfl is an LDS round trip: the gathers of a round waited on 16 of them in a chain)
template <int J>
__device__ __forceinline__ int grp_bcast_t(int x) {
  const int lo = __builtin_amdgcn_update_dpp(0, x, 0x150 + J, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, x, 0x158 + J, 0xf, 0xf, false);
  return (threadIdx.x & 8) ? hi : lo;
}
__device__ __forceinline__ int grp_bcast(int x, int j) {  // j is a constant after unrolling
  switch (j) {
    case 0: return grp_bcast_t<0>(x);
    case 1: return grp_bcast_t<1>(x);
    case 2: return grp_bcast_t<2>(x);
    case 3: return grp_bcast_t<3>(x);
    case 4: return grp_bcast_t<4>(x);
    case 5: return grp_bcast_t<5>(x);
    case 6: return grp_bcast_t<6>(x);
    default: return grp_bcast_t<7>(x);
  }
}

// NS = 32-column slices of the product (d = 32 NS), EB = entries in flight per lane group.  The body of one
// product; spmm_side_kernel runs one, spmm_side_jobs_kernel up to four independent ones (blockIdx.y).
// ONE: only the rows of side `only` are computed (the other side's rows are left as they are), and all 8 XCDs
// work on it: NS slice groups of 8 / NS XCDs (the DiffMM backward's second GCN hop, whose user rows equal the
// first hop's, models/diffmm.py:141-153)
template <int EB, int NS, bool ONE = false>
__device__ __forceinline__ void side_body(const int* __restrict__ plan, const SideSrc& src, float alpha, float beta,
                                          const SideDst& dst, float* __restrict__ scratch, int wpx, int nt,
                                          int only = 0) {
  constexpr int G = ONE ? NS : 2 * NS;         // (side, slice) groups
  constexpr int PHASES = G > 8 ? G / 8 : 1;    // groups per XCD, one after the other
  constexpr int P = G >= 8 ? 1 : 8 / G;        // XCDs per group
  constexpr int EPL = EB / 8;                  // packed entries per lane per round
  constexpr int NWV = kSideThreads / 64;       // waves per workgroup
  const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane >> 3, sub = lane & 7, gbase = grp * 8;
  const int* hdr = plan;
  const int4* __restrict__ tasks = reinterpret_cast<const int4*>(plan + hdr[H_TASK]);
  const int4* __restrict__ wtasks = reinterpret_cast<const int4*>(plan + hdr[H_WAVE]);
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
    const int side = ONE ? only : g / NS, slice = g % NS;
    const int c0 = slice * 32 + sub * 4;       // this lane's 4 columns
    const int blk = c0 >> 6, cin = c0 & 63;
    const float* __restrict__ lo = src.lo[blk] + cin;
    const float* __restrict__ hi = src.hi[blk] + cin;
    const int64_t ldl = src.ld_lo[blk], ldh = src.ld_hi[blk];
    float* __restrict__ yc = dst.y[blk] + cin;
    const int64_t ldy = dst.ld[blk];
    const float* __restrict__ zc = dst.z[blk] + cin;
    const int64_t ldz = dst.ldz[blk];
    auto store = [&](int row, float4 acc) {
      float* yp = yc + (int64_t)row * ldy;
      float4 o = gmr::f4_scale(alpha, acc);
      if (beta != 0.f) o = gmr::f4_fma(beta, *reinterpret_cast<const float4*>(zc + (int64_t)row * ldz), o);
      if (nt) {
        f32x4 ov = {o.x, o.y, o.z, o.w};
        __builtin_nontemporal_store(ov, reinterpret_cast<f32x4*>(yp));
      } else {
        *reinterpret_cast<float4*>(yp) = o;
      }
    };
    auto gather = [&](int c) -> float4 {
      return *reinterpret_cast<const float4*>(c < split ? lo + (int64_t)c * ldl : hi + (int64_t)(c - split) * ldh);
    };
    // ---- hub rows (degree > T): wave tasks, longest first.  The 8 lane groups split the block's
    // entries evenly and meet in a butterfly; a row of several blocks publishes each block sum
    // write-through and the wave whose counter add comes last adds the blocks in order.
    {
      const int n_wv = P * wpx * NWV, wv = (part_i * wpx + k) * NWV + wid;
      const int w0 = side == 0 ? 0 : hdr[H_NW0], nwk = side == 0 ? hdr[H_NW0] : hdr[H_NW1];
      // the next task's descriptor is loaded at the top of a task and its first entries during the
      // task's last gather round: one memory round trip per task instead of three
      int wi = wv;
      int4 tk = wi < nwk ? wtasks[w0 + wi] : make_int4(0, 0, 0, -1);
      int b, end;
      {
        const int pl = (tk.y - tk.x + 7) >> 3;
        b = tk.x + grp * pl;
        end = min(tk.y, b + pl);
      }
      int2 rec[EPL];
#pragma unroll
      for (int q = 0; q < EPL; ++q) {
        const int i = b + q * 8 + sub;
        rec[q] = i < end ? packed[i] : make_int2(0, 0);
      }
#pragma unroll 1
      for (; wi < nwk; wi += n_wv) {
        const int wn = wi + n_wv;
        const int4 tkn = wn < nwk ? wtasks[w0 + wn] : make_int4(0, 0, 0, -1);
        float4 acc = f4_zero();
        const int bt = b, et = end;
#pragma unroll 1
        for (int e = bt; e < et; e += EB) {
          float4 xs[EB];
          int2 cur[EPL];  // this round's entries: their values are shuffled out again at the FMAs
#pragma unroll
          for (int u = 0; u < EB; ++u) {
            const int c = grp_bcast(rec[u / 8].x, u % 8) & 0x7fffffff;
            xs[u] = f4_zero();
            if (e + u < et) xs[u] = gather(c);
          }
          int nb = e + EB, nend = et;
          if (e + EB >= et) {  // last round of this task: the next task's first entries
            const int pl = (tkn.y - tkn.x + 7) >> 3;
            nb = tkn.x + grp * pl;
            nend = min(tkn.y, nb + pl);
            b = nb;
            end = nend;
          }
#pragma unroll
          for (int q = 0; q < EPL; ++q) {
            cur[q] = rec[q];
            const int i = nb + q * 8 + sub;
            rec[q] = i < nend ? packed[i] : make_int2(0, 0);
          }
#pragma unroll
          for (int u = 0; u < EB; ++u)
            if (e + u < et) acc = gmr::f4_fma(__int_as_float(grp_bcast(cur[u / 8].y, u % 8)), xs[u], acc);
        }
        if (bt >= et) {  // this group had no entries (a short block): still move on to the next task
          const int pl = (tkn.y - tkn.x + 7) >> 3;
          b = tkn.x + grp * pl;
          end = min(tkn.y, b + pl);
#pragma unroll
          for (int q = 0; q < EPL; ++q) {
            const int i = b + q * 8 + sub;
            rec[q] = i < end ? packed[i] : make_int2(0, 0);
          }
        }
        acc = wave_groups_sum(acc);
        const int4 tkc = tk;
        tk = tkn;
        if (tkc.w < 0) {
          if (grp == 0) store(tkc.z, acc);
          continue;
        }
        if (grp == 0) {
          f32x4 pv = {acc.x, acc.y, acc.z, acc.w};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, pv), prs, (tkc.w * 256 + c0) * 4, 0, 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int h = slotmap[tkc.w];
        const int4 hb = hubs[h];
        int* cnt = counters + (int64_t)h * kSideCounterWords + slice;
        // Ordering without agent-scope fences (an agent-scope release on gfx950 writes back the XCD's dirty
        // L2 lines: per hub partial it took the epoch's SpMM class 12.6 -> 21.2 ms, profiles/r04ev2_bench.err, profiles/r04ev2_bench_fenced_spmm.json):
        // the partial is stored and re-read with device-scope (sc1) buffer ops, which bypass the per-XCD L2s;
        // the store has completed (vmcnt(0), whose "memory" clobber also keeps the compiler from moving the
        // counter add above it) before the add is issued; the last block's loads are control-dependent on
        // the add's returned value, so they issue after every other block's add, i.e. after its store.
        int old = 0;
        if (lane == 0) old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = __shfl(old, 0);
        if (old == hb.z - 1) {  // last block of the row: every block sum is published
          float4 s = f4_zero();
          for (int j = grp; j < hb.z; j += 8) {
            const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(prs, ((hb.y + j) * 256 + c0) * 4, 0, 16);
            const f32x4 f = __builtin_bit_cast(f32x4, r);
            s = gmr::f4_add(s, make_float4(f.x, f.y, f.z, f.w));
          }
          s = wave_groups_sum(s);
          if (grp == 0) store(hb.x, s);
          if (lane == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    if (hdr[H_DC]) {
      // ---- short rows by degree class (plan GMR_SIDE_CLASSES): a wave job is 8 lane-group tasks of one
      // degree d: each task is k = 16 / d whole rows (k d <= 16 entries, one gather round); rows of the class
      // in row order.  d is uniform across
      // the wave, so the row ends fall on the same entry slots in every group: k full-width stores per job
      // instead of one masked store per slot, and slots past k d are skipped outright.  The next round's
      // (or job's) entries and row ids are in flight while the current gathers land.
      const int4* __restrict__ cls = reinterpret_cast<const int4*>(plan + hdr[H_CLS]) + side * (kSideDcMax + 1);
      const int* __restrict__ perm = plan + hdr[H_PERM];
      const int2* __restrict__ pB = reinterpret_cast<const int2*>(plan + hdr[H_PACKB]);
      const int n_wv = P * wpx * NWV;
      const int wv = n_wv - 1 - ((part_i * wpx + k) * NWV + __builtin_amdgcn_readfirstlane(wid));
      {  // Y = beta Y on empty rows (lane groups, as the task plan)
        const int n_lg = P * wpx * (kSideThreads / 8);
        const int lg = n_lg - 1 - ((part_i * wpx + k) * (kSideThreads / 8) + wid * 8 + grp);
        const int e0 = side == 0 ? 0 : hdr[H_NE0], ne = side == 0 ? hdr[H_NE0] : hdr[H_NE1];
        for (int i = lg; i < ne; i += n_lg) store(empty[e0 + i], f4_zero());
      }
      // the side's class records, one per lane (lanes 0 .. 16): a job's class is found by one ballot over
      // them (a serial scan of scalar loads cost a memory round trip per class)
      const int4 cl_l = lane <= kSideDcMax ? cls[lane] : make_int4(INT32_MAX, 0, 0, 0);
      const int nj = __builtin_amdgcn_readlane(cl_l.x, kSideDcMax);  // total jobs (the terminator's first job)
      struct Job {
        int d, k, nrow, ne, eb;
        int2 e0, e1;
        int pr0, pr1;
      };
      auto load_job = [&](int job) {
        Job J;
        J.d = 0, J.k = 0, J.nrow = 0, J.ne = 0, J.eb = 0;
        J.e0 = J.e1 = make_int2(0, 0);
        J.pr0 = J.pr1 = 0;
        // no early exit past the last job (its loads would sit under a branch): every load is issued, from
        // clamped indices, and a job >= nj gets no rows
        // class = the number of classes 1 .. 15 whose first job is <= job (class 0 starts at job 0)
        const unsigned long long bl = __ballot(lane >= 1 && lane < kSideDcMax && cl_l.x <= job);
        const int ci = __popcll(bl);
        const int4 c = make_int4(__builtin_amdgcn_readlane(cl_l.x, ci), __builtin_amdgcn_readlane(cl_l.y, ci),
                                 __builtin_amdgcn_readlane(cl_l.z, ci),
                                 __builtin_amdgcn_readlane(cl_l.w, ci));  // {first job, perm row, packedB entry, rows}
        J.d = ci + 1;
        J.k = dc_rows_per_task(J.d);
        const int r0 = (job - c.x) * 8 * J.k + grp * J.k;  // this group's first row of the class
        J.nrow = job < nj ? max(0, min(J.k, c.w - r0)) : 0;
        J.ne = J.nrow * J.d;
        J.eb = c.z + r0 * J.d;
        // unconditional loads (clamped index, value selected after): a load under a branch makes the
        // compiler's vmcnt accounting give up and wait for every outstanding store with vmcnt(0)
        const int nse = hdr[H_NSE] - 1, nsr = hdr[H_NSR] - 1;
        const int2 a0 = pB[max(0, min(J.eb + sub, nse))], a1 = pB[max(0, min(J.eb + 8 + sub, nse))];
        const int q0 = perm[max(0, min(c.y + r0 + sub, nsr))], q1 = perm[max(0, min(c.y + r0 + 8 + sub, nsr))];
        J.e0 = sub < J.ne ? a0 : make_int2(0, 0);
        J.e1 = 8 + sub < J.ne ? a1 : make_int2(0, 0);
        J.pr0 = q0;
        J.pr1 = q1;
        return J;
      };
      // the job loop twice, for beta == 0 and beta != 0 (a load of Y under a run-time branch would cost
      // the counted vmcnt waits of the whole loop)
      auto run_jobs = [&](auto beta_tag) {
        constexpr bool BETA = decltype(beta_tag)::value;
        auto store_row = [&](int row, float4 acc) {
          float* yp = yc + (int64_t)row * ldy;
          float4 o = gmr::f4_scale(alpha, acc);
          if constexpr (BETA) o = gmr::f4_fma(beta, *reinterpret_cast<const float4*>(zc + (int64_t)row * ldz), o);
          if (nt) {
            f32x4 ov = {o.x, o.y, o.z, o.w};
            __builtin_nontemporal_store(ov, reinterpret_cast<f32x4*>(yp));
          } else {
            *reinterpret_cast<float4*>(yp) = o;
          }
        };
      Job J = load_job(wv);
#pragma unroll 1
      for (int job = wv; job < nj; job += n_wv) {
        const Job C = J;
        // the next job's entries and rows are loaded BEFORE this job's gathers: they travel while the
        // gathers land, and the wait for them at the next job counts the 16 younger gathers — it never
        // waits for this job's row stores, which come after them in the in-order vmcnt stream
        J = load_job(job + n_wv);
        // all 16 gathers issued unconditionally (an idle slot re-reads row 0 of X, an L2 hit, and is
        // zeroed), so the FMA of slot u waits with a counted vmcnt
        float4 xs[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int c = grp_bcast(u < 8 ? C.e0.x : C.e1.x, u % 8);
          xs[u] = gather(u < C.ne ? c : 0);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (u >= C.ne) xs[u] = f4_zero();
        float4 acc = f4_zero();
        int j = 0, nxt = C.d - 1;  // uniform: row counter, slot of the next row end
        const int kd = C.k * C.d;  // uniform: entry slots of this job's tasks
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          if (u < kd) {
            acc = gmr::f4_fma(__int_as_float(grp_bcast(u < 8 ? C.e0.y : C.e1.y, u % 8)), xs[u], acc);
            if (u == nxt) {
              const int row = __shfl(j < 8 ? C.pr0 : C.pr1, gbase + (j & 7));
              if (j < C.nrow) store_row(row, acc);
              acc = f4_zero();
              ++j;
              nxt += C.d;
            }
          }
        }
      }
      };
      if (beta != 0.f) run_jobs(std::true_type{});
      else run_jobs(std::false_type{});
      continue;
    }
    // ---- short rows: lane-group tasks of <= T entries (whole rows), the next task's descriptor and
    // first entries in flight while the current one gathers
    // lane groups numbered from the last wave down: the waves that took hub blocks (numbered from the
    // first wave up) get short-row tasks last
    const int n_lg = P * wpx * (kSideThreads / 8);
    const int lg = n_lg - 1 - ((part_i * wpx + k) * (kSideThreads / 8) + wid * 8 + grp);
    const int e0 = side == 0 ? 0 : hdr[H_NE0], ne = side == 0 ? hdr[H_NE0] : hdr[H_NE1];
    for (int i = lg; i < ne; i += n_lg) store(empty[e0 + i], f4_zero());  // Y = beta Y on empty rows
    const int t0 = side == 0 ? 0 : hdr[H_NT0], ntk = side == 0 ? hdr[H_NT0] : hdr[H_NT1];
    int ti = lg;
    int4 tk = ti < ntk ? tasks[t0 + ti] : make_int4(0, 0, 0, 0);
    int2 rec[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) {
      const int i = tk.x + q * 8 + sub;
      rec[q] = i < tk.y ? packed[i] : make_int2(0, 0);
    }
#pragma unroll 1
    while (ti < ntk) {
      const int tn = ti + n_lg;
      const int4 tkn = tn < ntk ? tasks[t0 + tn] : make_int4(0, 0, 0, 0);
      const int end = tk.y;
      int row = tk.z;
      float4 acc = f4_zero();
#pragma unroll 1
      for (int e = tk.x; e < end; e += EB) {
        float4 xs[EB];
        int2 cur[EPL];  // this round's entries: col (row-end bit) and val are shuffled out again at the FMAs
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          xs[u] = f4_zero();
          if (e + u < end) xs[u] = gather(grp_bcast(rec[u / 8].x, u % 8) & 0x7fffffff);
        }
        // the next round's entries (the next task's first ones after the last round) travel while
        // these gathers land
        const bool last = e + EB >= end;
        const int nb = last ? tkn.x : e + EB, nend = last ? tkn.y : end;
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
          cur[q] = rec[q];
          const int i = nb + q * 8 + sub;
          rec[q] = i < nend ? packed[i] : make_int2(0, 0);
        }
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          if (e + u < end) {
            acc = gmr::f4_fma(__int_as_float(grp_bcast(cur[u / 8].y, u % 8)), xs[u], acc);
            if (grp_bcast(cur[u / 8].x, u % 8) < 0) {  // row end
              store(row, acc);
              ++row;
              acc = f4_zero();
            }
          }
        }
      }
      tk = tkn;
      ti = tn;
    }
  }
}

template <int EB, int NS, bool ONE = false>
__global__ void __launch_bounds__(kSideThreads) spmm_side_kernel(const int* __restrict__ plan, SideSrc src,
                                                                  float alpha, float beta, SideDst dst,
                                                                  float* __restrict__ scratch, int wpx, int nt,
                                                                  int only) {
  side_body<EB, NS, ONE>(plan, src, alpha, beta, dst, scratch, wpx, nt, only);
}

// Multi-job launch (round 5, gmr_spmm_side_jobs_f32): independent side-split products of the same width in one
// grid, job = blockIdx.y.  gridDim.x = 8 wpx is a multiple of 8, so a workgroup's XCD (its linear id mod 8) is
// blockIdx.x mod 8 in every job: each job keeps the (side, slice) -> XCD map of its own launch.  Each job has
// its own plan and hub scratch, so the sums are those of separate launches bit for bit.
struct SideJob {
  const int* plan;
  float* scratch;
  SideSrc src;
  SideDst dst;
};
struct SideJobs {
  SideJob j[4];
};
template <int EB, int NS>
__global__ void __launch_bounds__(kSideThreads) spmm_side_jobs_kernel(SideJobs jobs, float alpha, float beta, int wpx,
                                                                       int nt) {
  const int y = blockIdx.y;
  const SideJob& J = jobs.j[y];
  side_body<EB, NS>(J.plan, J.src, alpha, beta, J.dst, J.scratch, wpx, nt);
}


// packed entries: {col | (last entry of its row) << 31, val}: one thread per entry (coalesced), then one
// per row sets its last entry's bit (a per-row loop serialised the hub rows of a rebuilt graph: 790 us)
__global__ void __launch_bounds__(256) side_pack_kernel(const int* __restrict__ col, const float* __restrict__ val,
                                                        int64_t nnz, int2* __restrict__ packed) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * blockDim.x)
    packed[e] = make_int2(col[e], __float_as_int(val[e]));
}
__global__ void __launch_bounds__(256) side_last_kernel(const int* __restrict__ rowptr, int64_t n_rows,
                                                        int2* __restrict__ packed) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_rows; r += (int64_t)gridDim.x * blockDim.x) {
    const int beg = rowptr[r], end = rowptr[r + 1];
    if (end > beg) packed[end - 1].x |= (int)0x80000000u;
  }
}

struct SidePlanHost {
  std::vector<int4> tasks[2], waves[2], hubs;
  std::vector<int> empty[2], slotmap;
  bool dc = false;                 // degree-class plan: short rows in classes, not tasks
  std::vector<int4> cls;           // per side kSideDcMax + 1 {first job, first perm row, first packedB entry, rows}
  std::vector<int> perm, dsto;     // short rows (side, degree, row order) and their packedB offsets
  int64_t short_entries = 0;
};

// rows of degree <= T: lane-group tasks of <= T entries (whole rows, cut at empty rows); longer rows:
// wave tasks of <= 8 TW entries (blocks), a row of several blocks gets a hub record and slots
void side_plan_host(const int32_t* rp, int64_t n_rows, int64_t split, int T, int TW, SidePlanHost& p, bool dc = false) {
  int slot = 0;
  p.dc = dc;
  if (dc) T = kSideDcMax;
  for (int s = 0; s < 2; ++s) {
    if (dc) {  // classes: rows of degree d (1..16) in row order; a job = 8 tasks of k = 16 / d rows
      const int64_t r0 = s == 0 ? 0 : split, r1 = s == 0 ? split : n_rows;
      std::vector<int> by[kSideDcMax + 1];
      for (int64_t r = r0; r < r1; ++r) {
        const int d = rp[r + 1] - rp[r];
        if (d >= 1 && d <= kSideDcMax) by[d].push_back((int)r);
      }
      int job = 0;
      for (int d = 1; d <= kSideDcMax; ++d) {
        const int k = dc_rows_per_task(d), n = (int)by[d].size();
        p.cls.push_back(make_int4(job, (int)p.perm.size(), (int)p.short_entries, n));
        for (int r : by[d]) {
          p.perm.push_back(r);
          p.dsto.push_back((int)p.short_entries);
          p.short_entries += d;
        }
        job += (n + 8 * k - 1) / (8 * k);
      }
      p.cls.push_back(make_int4(job, (int)p.perm.size(), (int)p.short_entries, 0));  // terminator
    }
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
        const int blocks = (deg + 8 * TW - 1) / (8 * TW), bl = (deg + blocks - 1) / blocks;
        if (blocks == 1) {
          p.waves[s].push_back(make_int4(b, e, (int)r, -1));
          continue;
        }
        const int h = (int)p.hubs.size();
        p.hubs.push_back(make_int4((int)r, slot, blocks, 0));
        for (int j = 0; j < blocks; ++j) {
          p.waves[s].push_back(make_int4(b + j * bl, std::min(e, b + (j + 1) * bl), (int)r, slot + j));
          p.slotmap.push_back(h);
        }
        slot += blocks;
      } else if (dc) {
        flush();  // degree-class plan: the short row is in its class (above)
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
    std::stable_sort(p.waves[s].begin(), p.waves[s].end(),
                     [](const int4& a, const int4& c) { return a.y - a.x > c.y - c.x; });  // longest first
  }
}

int64_t r4(int64_t v) { return (v + 3) / 4 * 4; }

struct SideLayout {
  int64_t task, wave, empty, hub, slot, packed, cls, perm, dsto, packb, words;
};
SideLayout side_layout(const SidePlanHost& p, int64_t nnz) {
  SideLayout l;
  l.task = kSideHdr;
  l.wave = l.task + 4 * (int64_t)(p.tasks[0].size() + p.tasks[1].size());
  l.empty = l.wave + 4 * (int64_t)(p.waves[0].size() + p.waves[1].size());
  l.hub = r4(l.empty + (int64_t)(p.empty[0].size() + p.empty[1].size()));
  l.slot = l.hub + 4 * (int64_t)p.hubs.size();
  l.packed = r4(l.slot + (int64_t)p.slotmap.size());
  l.cls = r4(l.packed + 2 * nnz);  // int4 records: 16-byte aligned
  l.perm = l.cls + 4 * (int64_t)p.cls.size();
  l.dsto = l.perm + (int64_t)p.perm.size();
  l.packb = r4(l.dsto + (int64_t)p.dsto.size());
  // 4 zero words past the packed entries: the degree-class job loader issues its perm / packedB loads
  // from clamped indices even when the plan has no class rows (H_NSR == 0), and then they land here
  l.words = l.packb + 2 * p.short_entries + 4;
  return l;
}

// launch shape: workgroups per XCD and entries in flight per lane group (GMR_SPMM_SIDE_WPX /
// GMR_SPMM_SIDE_EB at first use; gmr_spmm_side_tune sets them at run time, for sweeps)
int g_side_wpx = -1, g_side_eb = -1;
bool g_side_tuned = false;  // gmr_spmm_side_tune overrides the caller's per-graph wpx
int side_wpx() {
  if (g_side_wpx < 0) {
    const char* s = getenv("GMR_SPMM_SIDE_WPX");
    const int x = s ? atoi(s) : 0;
    g_side_wpx = x > 0 && x <= 1024 ? x : 64;
  }
  return g_side_wpx;
}
int side_eb() {
  if (g_side_eb < 0) {
    const char* s = getenv("GMR_SPMM_SIDE_EB");
    g_side_eb = s && atoi(s) == 8 ? 8 : 16;
  }
  return g_side_eb;
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
                 float* scratch, int wpx, int nt, hipStream_t st, int only = -1) {
  if (only >= 0) {  // one side, on all eight XCDs
    if (eb == 8)
      hipLaunchKernelGGL((spmm_side_kernel<8, NS, true>), dim3(8 * wpx), dim3(kSideThreads), 0, st, plan, src, alpha,
                         beta, dst, scratch, wpx, nt, only);
    else
      hipLaunchKernelGGL((spmm_side_kernel<16, NS, true>), dim3(8 * wpx), dim3(kSideThreads), 0, st, plan, src, alpha,
                         beta, dst, scratch, wpx, nt, only);
    return;
  }
  if (eb == 8)
    hipLaunchKernelGGL((spmm_side_kernel<8, NS>), dim3(8 * wpx), dim3(kSideThreads), 0, st, plan, src, alpha, beta, dst,
                       scratch, wpx, nt, 0);
  else
    hipLaunchKernelGGL((spmm_side_kernel<16, NS>), dim3(8 * wpx), dim3(kSideThreads), 0, st, plan, src, alpha, beta,
                       dst, scratch, wpx, nt, 0);
}

template <int NS>
void side_jobs_launch(int eb, int njobs, const SideJobs& jobs, float alpha, float beta, int wpx, int nt,
                      hipStream_t st) {
  const dim3 grid((unsigned)(8 * wpx), (unsigned)njobs);
  if (eb == 8)
    hipLaunchKernelGGL((spmm_side_jobs_kernel<8, NS>), grid, dim3(kSideThreads), 0, st, jobs, alpha, beta, wpx, nt);
  else
    hipLaunchKernelGGL((spmm_side_jobs_kernel<16, NS>), grid, dim3(kSideThreads), 0, st, jobs, alpha, beta, wpx, nt);
}

// one job's block pointers / strides from the C-ABI arrays (entries [4 q, 4 q + n_blocks) of job q)
int side_fill(int n_blocks, const float* const* x_lo, const int64_t* ld_lo, const float* const* x_hi,
              const int64_t* ld_hi, int64_t split, float* const* y, const int64_t* ld_y, SideSrc& s, SideDst& d) {
  for (int b = 0; b < 4; ++b) {
    const bool on = b < n_blocks;
    s.lo[b] = on ? x_lo[b] : nullptr;
    s.hi[b] = on ? x_hi[b] : nullptr;
    s.ld_lo[b] = on ? ld_lo[b] : 0;
    s.ld_hi[b] = on ? ld_hi[b] : 0;
    d.y[b] = on ? y[b] : nullptr;
    d.ld[b] = on ? ld_y[b] : 0;
    d.z[b] = d.y[b];
    d.ldz[b] = d.ld[b];
    if (on) {
      GMR_ARG(s.lo[b] && s.hi[b] && d.y[b], "null block pointer");
      GMR_ARG(((uintptr_t)s.lo[b] | (uintptr_t)s.hi[b] | (uintptr_t)d.y[b]) % 16 == 0, "blocks must be 16-byte aligned");
      GMR_ARG(s.ld_lo[b] % 4 == 0 && s.ld_hi[b] % 4 == 0 && d.ld[b] % 4 == 0 && d.ld[b] >= 64,
              "leading dimensions must be multiples of 4");
    }
  }
  s.split = split;
  return GMR_OK;
}

}  // namespace

extern "C" int gmr_spmm_side_jobs_f32(int32_t njobs, const int32_t* const* plans, float* const* scratch,
                                      int32_t n_blocks, const float* const* x_lo, const int64_t* ld_lo,
                                      const float* const* x_hi, const int64_t* ld_hi, const int64_t* split,
                                      float alpha, float beta, float* const* y, const int64_t* ld_y, int32_t wpx,
                                      void* stream) {
  GMR_ARG(njobs >= 1 && njobs <= 4, "1 to 4 jobs");
  GMR_ARG(plans && scratch && x_lo && ld_lo && x_hi && ld_hi && split && y && ld_y, "null argument");
  GMR_ARG(wpx >= 0 && wpx <= 1024, "wpx in [0, 1024] (0 = default)");
  GMR_ARG(n_blocks == 1 || n_blocks == 2 || n_blocks == 4, "1, 2 or 4 blocks of 64 columns");
  SideJobs jobs{};
  for (int q = 0; q < njobs; ++q) {
    GMR_ARG(plans[q] && scratch[q], "null plan / scratch");
    jobs.j[q].plan = plans[q];
    jobs.j[q].scratch = scratch[q];
    if (side_fill(n_blocks, x_lo + 4 * q, ld_lo + 4 * q, x_hi + 4 * q, ld_hi + 4 * q, split[q], y + 4 * q, ld_y + 4 * q,
                  jobs.j[q].src, jobs.j[q].dst) != GMR_OK)
      return GMR_ERR_ARG;
  }
  const hipStream_t st = (hipStream_t)stream;
  const int eb = side_eb(), nt = side_nt();
  if (wpx == 0 || getenv("GMR_SPMM_SIDE_WPX") || g_side_tuned) wpx = side_wpx();
  if (n_blocks == 1)
    side_jobs_launch<2>(eb, njobs, jobs, alpha, beta, wpx, nt, st);
  else if (n_blocks == 2)
    side_jobs_launch<4>(eb, njobs, jobs, alpha, beta, wpx, nt, st);
  else
    side_jobs_launch<8>(eb, njobs, jobs, alpha, beta, wpx, nt, st);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_spmm_side_tune(int32_t wpx, int32_t eb) {
  GMR_ARG(wpx > 0 && wpx <= 1024 && (eb == 8 || eb == 16), "wpx in [1, 1024], eb 8 or 16");
  g_side_wpx = wpx;
  g_side_eb = eb;
  g_side_tuned = true;
  return GMR_OK;
}

// T argument: bits 0-15 = T (entries of a short-row task, rows of degree > T are hub rows), bits
// 16-23 = TW (entries per lane group of a hub block: blocks of 8 TW; 0 = 32)
inline int side_T(int32_t Tw) { return Tw & 0xFFFF; }
inline int side_TW(int32_t Tw) { return (Tw >> 16) & 0xFF ? (Tw >> 16) & 0xFF : 32; }
inline bool side_DC(int32_t Tw) { return (Tw & GMR_SIDE_CLASSES) != 0; }

extern "C" int64_t gmr_spmm_side_plan_words(const int32_t* rowptr_host, int64_t n_rows, int64_t split, int32_t Tw) {
  const int T = side_T(Tw), TW = side_TW(Tw);
  if (!rowptr_host || n_rows <= 0 || split < 0 || split > n_rows || T < 8 || T > 4096 || TW < 4) return -1;
  SidePlanHost p;
  side_plan_host(rowptr_host, n_rows, split, T, TW, p, side_DC(Tw));
  return side_layout(p, rowptr_host[n_rows]).words;
}

extern "C" int gmr_spmm_side_plan_build(const int32_t* rowptr_host, int64_t n_rows, int64_t split, int32_t Tw,
                                        int32_t* plan_host, int64_t words) {
  const int T = side_T(Tw), TW = side_TW(Tw);
  GMR_ARG(rowptr_host && plan_host && n_rows > 0 && split >= 0 && split <= n_rows, "bad args");
  GMR_ARG(T >= 8 && T <= 4096 && TW >= 4, "T must be in [8, 4096], TW >= 4");
  GMR_ARG(n_rows < (1 << 30) && rowptr_host[n_rows] < (1ll << 31) - 1, "too large for int32 plans");
  SidePlanHost p;
  side_plan_host(rowptr_host, n_rows, split, T, TW, p, side_DC(Tw));
  const int64_t nnz = rowptr_host[n_rows];
  const SideLayout l = side_layout(p, nnz);
  GMR_ARG(words >= l.words, "plan buffer smaller than gmr_spmm_side_plan_words(...)");
  // hub partial rows are addressed by 32-bit buffer offsets (slot * 256 + column) * 4 bytes
  GMR_ARG((int64_t)p.slotmap.size() * 1024 < INT32_MAX, "too many hub slots for 32-bit partial offsets");
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
  h[H_WAVE] = (int)l.wave;
  h[H_NW0] = (int)p.waves[0].size();
  h[H_NW1] = (int)p.waves[1].size();
  h[H_TW] = TW;
  for (int i = H_TW + 1; i < kSideHdr; ++i) h[i] = 0;
  GMR_ARG(l.words < INT32_MAX, "plan too large for int32 offsets");
  h[H_DC] = p.dc ? 1 : 0;
  h[H_CLS] = (int)l.cls;
  h[H_PERM] = (int)l.perm;
  h[H_DSTO] = (int)l.dsto;
  h[H_NSR] = (int)p.perm.size();
  h[H_PACKB] = (int)l.packb;
  h[H_NSE] = (int)p.short_entries;
  int4* cl = reinterpret_cast<int4*>(h + l.cls);
  for (const int4& x : p.cls) *cl++ = x;
  for (size_t i = 0; i < p.perm.size(); ++i) h[l.perm + i] = p.perm[i];
  for (size_t i = 0; i < p.dsto.size(); ++i) h[l.dsto + i] = p.dsto[i];
  for (int64_t i = l.packed + 2 * nnz; i < l.cls; ++i) h[i] = 0;
  for (int64_t i = l.dsto + (int64_t)p.dsto.size(); i < l.packb; ++i) h[i] = 0;
  for (int64_t i = l.packb + 2 * p.short_entries; i < l.words; ++i) h[i] = 0;
  int4* t = reinterpret_cast<int4*>(h + l.task);
  for (int s = 0; s < 2; ++s)
    for (const int4& x : p.tasks[s]) *t++ = x;
  for (int s = 0; s < 2; ++s)
    for (const int4& x : p.waves[s]) *t++ = x;
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
  int2* packed = reinterpret_cast<int2*>(plan + packed_off);
  hipLaunchKernelGGL(side_pack_kernel, dim3(gmr::grid_for(nnz, 256, 8192)), dim3(256), 0, (hipStream_t)stream, col, val,
                     nnz, packed);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(side_last_kernel, dim3(gmr::grid_for(n_rows, 256, 4096)), dim3(256), 0, (hipStream_t)stream, rowptr,
                     n_rows, packed);
  GMR_LAUNCHED();
  return GMR_OK;
}

// packedB: the short rows' (col, val) in class order, one thread per short row (<= 16 entries each)
__global__ void __launch_bounds__(256) side_pack_classes_kernel(const int* __restrict__ rowptr, const int* __restrict__ col,
                                                                const float* __restrict__ val, int n_short,
                                                                const int* __restrict__ perm, const int* __restrict__ dsto,
                                                                int2* __restrict__ pb) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n_short; q += gridDim.x * blockDim.x) {
    const int r = perm[q], b = rowptr[r], e = rowptr[r + 1], o = dsto[q];
    for (int i = b; i < e; ++i) pb[o + i - b] = make_int2(col[i], __float_as_int(val[i]));
  }
}

extern "C" int gmr_spmm_side_pack_classes(const int32_t* rowptr, const int32_t* col, const float* val,
                                          const int32_t* plan_host, int32_t* plan, void* stream) {
  GMR_ARG(rowptr && col && val && plan_host && plan && plan_host[H_MAGIC] == kSideMagic, "bad args");
  if (!plan_host[H_DC] || plan_host[H_NSR] == 0) return GMR_OK;
  hipLaunchKernelGGL(side_pack_classes_kernel, dim3(gmr::grid_for(plan_host[H_NSR], 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, rowptr, col, val, plan_host[H_NSR], plan + plan_host[H_PERM],
                     plan + plan_host[H_DSTO], reinterpret_cast<int2*>(plan + plan_host[H_PACKB]));
  GMR_LAUNCHED();
  return GMR_OK;
}

namespace {
int side_call(const int32_t* plan, int32_t n_blocks, const float* const* x_lo, const int64_t* ld_lo,
              const float* const* x_hi, const int64_t* ld_hi, int64_t split, float alpha, float beta,
              const float* const* z, const int64_t* ld_z, float* const* y, const int64_t* ld_y, int32_t only,
              float* scratch, int32_t wpx, void* stream) {
  GMR_ARG(plan && scratch && x_lo && ld_lo && x_hi && ld_hi && y && ld_y, "null argument");
  GMR_ARG(wpx >= 0 && wpx <= 1024, "wpx in [0, 1024] (0 = default)");
  GMR_ARG(n_blocks == 1 || n_blocks == 2 || n_blocks == 4, "1, 2 or 4 blocks of 64 columns");
  GMR_ARG(only >= -1 && only <= 1, "only_side must be -1 (both), 0 (rows < split) or 1 (rows >= split)");
  SideSrc s;
  SideDst d;
  if (side_fill(n_blocks, x_lo, ld_lo, x_hi, ld_hi, split, y, ld_y, s, d) != GMR_OK) return GMR_ERR_ARG;
  if (z) {
    GMR_ARG(ld_z, "null ld_z");
    for (int b = 0; b < n_blocks; ++b) {
      GMR_ARG(z[b] && ((uintptr_t)z[b]) % 16 == 0 && ld_z[b] % 4 == 0 && ld_z[b] >= 64,
              "z blocks: 16-byte aligned, leading dimension a multiple of 4 and >= 64");
      d.z[b] = z[b];
      d.ldz[b] = ld_z[b];
    }
  }
  const hipStream_t st = (hipStream_t)stream;
  const int eb = side_eb(), nt = side_nt();
  if (wpx == 0 || getenv("GMR_SPMM_SIDE_WPX") || g_side_tuned) wpx = side_wpx();
  if (n_blocks == 1)
    side_launch<2>(eb, plan, s, alpha, beta, d, scratch, wpx, nt, st, only);
  else if (n_blocks == 2)
    side_launch<4>(eb, plan, s, alpha, beta, d, scratch, wpx, nt, st, only);
  else
    side_launch<8>(eb, plan, s, alpha, beta, d, scratch, wpx, nt, st, only);
  GMR_LAUNCHED();
  return GMR_OK;
}
}  // namespace

extern "C" int gmr_spmm_side_f32(const int32_t* plan, int32_t n_blocks, const float* const* x_lo, const int64_t* ld_lo,
                                 const float* const* x_hi, const int64_t* ld_hi, int64_t split, float alpha, float beta,
                                 float* const* y, const int64_t* ld_y, float* scratch, int32_t wpx, void* stream) {
  return side_call(plan, n_blocks, x_lo, ld_lo, x_hi, ld_hi, split, alpha, beta, nullptr, nullptr, y, ld_y, -1,
                   scratch, wpx, stream);
}

extern "C" int gmr_spmm_side2_f32(const int32_t* plan, int32_t n_blocks, const float* const* x_lo, const int64_t* ld_lo,
                                  const float* const* x_hi, const int64_t* ld_hi, int64_t split, float alpha, float beta,
                                  const float* const* z, const int64_t* ld_z, float* const* y, const int64_t* ld_y,
                                  int32_t only_side, float* scratch, int32_t wpx, void* stream) {
  return side_call(plan, n_blocks, x_lo, ld_lo, x_hi, ld_hi, split, alpha, beta, z, ld_z, y, ld_y, only_side, scratch,
                   wpx, stream);
}
