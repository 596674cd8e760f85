// K3/K4 — fp32 GEMM on the bf16 matrix cores by exact operand splitting (GMR_GEMM_X6).
// Same operand, epilogue, split-K and tile-order conventions as gemm.hip (gemm_impl.h).
#include <stdlib.h>

#include <type_traits>

#include "gemm_impl.h"

namespace {
using namespace gmr_gemm;

// ---------------------------------------------------------------------------------------------
// Split-bf16 variant (GMR_GEMM_X6): fp32 operands on the bf16 matrix cores.  Each fp32 x is split
// on its way into LDS into three bf16 terms x = hi + mid + lo, EXACTLY (round-to-nearest splits:
// 3 x 8 significand bits hold fp32's 24), and a product a*b is accumulated as the six bf16 MFMA
// products hi*hi + hi*mid + mid*hi + hi*lo + lo*hi + mid*mid (v_mfma_f32_32x32x16_bf16: bf16
// products are exact in fp32, fp32 accumulation).  The three dropped terms (mid*lo, lo*mid,
// lo*lo) are below 2^-23 |a b|, i.e. at the rounding of an fp32 product, so the sums carry fp32
// accuracy (tests/test_kernels_gpu.py checks the error against fp64 next to the fp32-MFMA kernel's).
// Six 32x32x16 bf16 MFMAs (6 x 32 cycles) replace eight 32x32x2 f32 ones (8 x 64 cycles) per
// 32x32x16 block: 2.7x the fp32 MFMA rate at the instruction level.
// LDS: per stage and operand three planes [rows][32 k] of bf16 (64-byte rows); the 16-byte k
// chunk c of row r sits at chunk c ^ ((r >> 2) & 3), so the 16 lanes of a fragment read hit 16
// distinct bank groups.  Register staging (the split needs the values in VGPRs anyway); NBUF = 2
// double-buffers LDS (one barrier per k tile), NBUF = 1 for the 256^2 tile (2 barriers).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int x6_swz(int r) { return (r >> 2) & 3; }

// Edge values: rounding a finite |x| above bf16's largest value (0x1.fep127) to bf16 gives
// inf and then NaN terms, so x is clamped into bf16's range first (one v_med3_f32): hi = +-0x1.fep127
// exactly and x - hi (same binade, Sterbenz) is exact, so the split stays exact up to FLT_MAX.  An inf
// operand still splits into hi = 0x1.fep127, mid = inf, lo = NaN: its products come out non-finite
// (NaN where fp32 gives inf), as an inf input to the fp32 kernel does.
__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)__builtin_amdgcn_fmed3f(x, -0x1.fep127f, 0x1.fep127f);
  const float r1 = x - (float)h;  // exact
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);    // exact: at most 8 significand bits remain
}

// register tile -> the three bf16 planes of one LDS stage (plane stride PL elements)
template <int R, bool KC, int NT, int N4>
__device__ __forceinline__ void x6_store(const float4 (&r)[N4], __bf16* s) {
  constexpr int PL = R * BK;
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < N4; ++i) {
    const int idx = t + NT * i;
    const float v[4] = {r[i].x, r[i].y, r[i].z, r[i].w};
    if (KC) {  // 4 consecutive k of one row: 8 bytes per plane
      const int rr = idx / (BK / 4), k4 = (idx % (BK / 4)) * 4;
      bf16x4 h, m, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __bf16 a, b, c;
        split3(v[e], a, b, c);
        h[e] = a;
        m[e] = b;
        l[e] = c;
      }
      const int off = rr * BK + (((k4 >> 3) ^ x6_swz(rr)) << 3) + (k4 & 7);
      *reinterpret_cast<bf16x4*>(s + off) = h;
      *reinterpret_cast<bf16x4*>(s + PL + off) = m;
      *reinterpret_cast<bf16x4*>(s + 2 * PL + off) = l;
    } else {  // 4 consecutive rows at one k: one element per row and plane
      const int kk = idx / (R / 4), m4 = (idx % (R / 4)) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rr = m4 + e;
        const int off = rr * BK + (((kk >> 3) ^ x6_swz(rr)) << 3) + (kk & 7);
        __bf16 a, b, c;
        split3(v[e], a, b, c);
        s[off] = a;
        s[PL + off] = b;
        s[2 * PL + off] = c;
      }
    }
  }
}

// k-contiguous operand tile [R rows][BK k] in registers, loaded through per-granule element offsets
// computed once per workgroup: rows past the operand's end are clamped onto its last row (their
// products only reach C rows / columns the epilogue discards), so a full k tile loads with no
// bounds test at all; only the last, partial k tile zeroes k >= K (lda >= K rounded up to 4, so
// its float4 granules that start below K stay inside the row).
template <int R, int NT>
struct KcTile {
  static constexpr int N4 = R * BK / 4 / NT;
  static_assert(N4 * NT * 4 == R * BK, "tile rows x BK must split evenly over the block");
  int off[N4];
  float4 r[N4];

  __device__ __forceinline__ void init(int64_t r0, int64_t nrows, int64_t ld) {
#pragma unroll
    for (int i = 0; i < N4; ++i) {
      const int idx = threadIdx.x + NT * i;
      const int rr = idx / (BK / 4), k4 = (idx % (BK / 4)) * 4;
      const int64_t row = min(r0 + rr, nrows - 1) - r0;
      off[i] = (int)(row * ld) + k4;
    }
  }
  __device__ __forceinline__ void load(const float* __restrict__ base) {  // base = tile row 0, k0
#pragma unroll
    for (int i = 0; i < N4; ++i) r[i] = *reinterpret_cast<const float4*>(base + off[i]);
  }
  __device__ __forceinline__ void load_tail(const float* __restrict__ base, int kleft) {
#pragma unroll
    for (int i = 0; i < N4; ++i) {
      const int k4 = ((threadIdx.x + NT * i) % (BK / 4)) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k4 < kleft) {
        v = *reinterpret_cast<const float4*>(base + off[i]);
        if (k4 + 1 >= kleft) v.y = 0.f;
        if (k4 + 2 >= kleft) v.z = 0.f;
        if (k4 + 3 >= kleft) v.w = 0.f;
      }
      r[i] = v;
    }
  }
};

// m- / n-contiguous operand tile (A stored K x M of a TN call, B stored K x N of an NN / TN call) read in place:
// each thread owns one row of the tile and E = R x BK / NT consecutive k of it (8 or 16), loaded as single
// floats (the 64 lanes of a load read 64 consecutive rows at one k: 256 contiguous bytes), so after the split
// it writes 16-byte chunks of its own row: the same plane images as KcTile's, with no transposed copy in HBM,
// and consecutive lanes write consecutive 64-byte rows (the 4-row quads of a float4 mapping all hit one half
// of the banks and ran the TN gradients 8-10 % slower than copy + k-contiguous, profiles/r05zs_*).  Rows past
// the operand's end load its last row (any alignment) and only reach C rows / columns the epilogue discards;
// k past the slab's end is zeroed, never loaded.
template <int R, int NT>
struct MnTile {
  static constexpr int E = R * BK / NT;  // k per thread
  static_assert(E % 8 == 0 && NT % R == 0, "whole 8-k chunks of one row per thread");
  int off;  // element offset of (this thread's row, its first k) from the tile's (r0, k0)
  int rr;   // the row within the tile
  int kt;   // its first k
  int64_t ld;
  float v[E];

  __device__ __forceinline__ void init(int64_t r0, int64_t nrows, int64_t ld_) {
    ld = ld_;
    rr = threadIdx.x % R;
    kt = (threadIdx.x / R) * E;
    off = (int)(kt * ld + (min(r0 + rr, nrows - 1) - r0));
  }
  // base = element (row r0, k0); kleft = valid k of this tile (BK for a full one)
  __device__ __forceinline__ void load(const float* __restrict__ base, int kleft) {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = (kleft == BK || kt + e < kleft) ? base[off + e * ld] : 0.f;
  }
  // the three bf16 planes of one LDS stage (plane stride PL elements), KcTile / x6_store's image
  __device__ __forceinline__ void store(__bf16* s) const {
    constexpr int PL = R * BK;
#pragma unroll
    for (int c = 0; c < E / 8; ++c) {
      bf16x8 h, m, l;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        __bf16 a, b, d;
        split3(v[8 * c + e], a, b, d);
        h[e] = a;
        m[e] = b;
        l[e] = d;
      }
      const int o = rr * BK + ((((kt >> 3) + c) ^ x6_swz(rr)) << 3);
      *reinterpret_cast<bf16x8*>(s + o) = h;
      *reinterpret_cast<bf16x8*>(s + PL + o) = m;
      *reinterpret_cast<bf16x8*>(s + 2 * PL + o) = l;
    }
  }
};

// NT products (A [M][K], B [N][K], both k-contiguous, 16-byte aligned, lda / ldb multiples of 4)
// float4 granules [I0, I1) of a k-contiguous register tile -> the three bf16 planes (as x6_store)
template <int R, int NT, int N4, int I0, int I1>
__device__ __forceinline__ void x6_store_part(const float4 (&r)[N4], __bf16* s) {
  constexpr int PL = R * BK;
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    const int idx = threadIdx.x + NT * i;
    const int rr = idx / (BK / 4), k4 = (idx % (BK / 4)) * 4;
    const float v[4] = {r[i].x, r[i].y, r[i].z, r[i].w};
    bf16x4 h, m, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      __bf16 a, b, c;
      split3(v[e], a, b, c);
      h[e] = a;
      m[e] = b;
      l[e] = c;
    }
    const int off = rr * BK + (((k4 >> 3) ^ x6_swz(rr)) << 3) + (k4 & 7);
    *reinterpret_cast<bf16x4*>(s + off) = h;
    *reinterpret_cast<bf16x4*>(s + PL + off) = m;
    *reinterpret_cast<bf16x4*>(s + 2 * PL + off) = l;
  }
}

// one k tile of a k-contiguous operand straight into ring registers d (KcTile's offsets; full tile or the
// zero-padded last one): the loads of later ring slots stay in flight while earlier slots are split
template <int R, int NT, int N4>
__device__ __forceinline__ void kc_fetch(float4 (&d)[N4], const KcTile<R, NT>& tl, const float* __restrict__ base,
                                         bool full, int kleft) {
  if (full) {
#pragma unroll
    for (int i = 0; i < N4; ++i) d[i] = *reinterpret_cast<const float4*>(base + tl.off[i]);
  } else {
#pragma unroll
    for (int i = 0; i < N4; ++i) {
      const int k4 = ((threadIdx.x + NT * i) % (BK / 4)) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k4 < kleft) {
        v = *reinterpret_cast<const float4*>(base + tl.off[i]);
        if (k4 + 1 >= kleft) v.y = 0.f;
        if (k4 + 2 >= kleft) v.z = 0.f;
        if (k4 + 3 >= kleft) v.w = 0.f;
      }
      d[i] = v;
    }
  }
}

// instruction order of one pipelined MFMA step: its NR fragment reads, then NM MFMAs, each followed
// by NV VALU instructions of the next tile's split and, for the first NW, one of its LDS writes
// (sched_group_barrier masks: 0x008 MFMA, 0x002 VALU, 0x100 DS read, 0x200 DS write)
template <int NR, int NM, int NV, int NW>
__device__ __forceinline__ void x6_interleave() {
  __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
    if (i < NW) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
  }
}

template <int BM, int BN, int WGM, int WGN, int NBUF, int OCC, int PIPE, bool AKC = true, bool BKC = true>
__global__ void __launch_bounds__(64 * WGM * WGN, OCC) gemm_x6_kernel(int64_t M, int64_t N, int64_t K,
                                                                const float* __restrict__ A, int64_t lda,
                                                                const float* __restrict__ B, int64_t ldb,
                                                                float* __restrict__ C, int64_t ldc, Epi epi,
                                                                int tiles_n, int64_t k_per_split,
                                                                float* __restrict__ ws) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int APL = BM * BK, BPL = BN * BK;  // bf16 elements per plane
  constexpr int STAGE = 3 * (APL + BPL);
  __shared__ __attribute__((aligned(16))) __bf16 smem[NBUF * STAGE];

  const int nwg = gridDim.x;
  const int b = blockIdx.x;
  const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  int tmi, tni;
  tile_mn(tile, tiles_n, (int)((M + BM - 1) / BM), tmi, tni);
  const int64_t m0 = (int64_t)tmi * BM;
  const int64_t n0 = (int64_t)tni * BN;
  const int64_t kbeg = (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = min(K, kbeg + k_per_split);

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int wm = w / WGN, wn = w % WGN;
  const int h = lane >> 5, l32 = lane & 31;

  // Two accumulators per output tile (round 6): hi * hi alone into acc, the five small products into sml, added
  // once after the k loop.  The bf16 MFMA's fp32 accumulation is not unbiased when it adds products far below
  // the accumulator (it rounds toward -inf by ~0.03 ulp per x6 k step, both signs of the result alike:
  // scripts/micro/mfma_round.hip, profiles/r06j_mfma_rounding.txt); with the small products summed apart, at
  // 2^-8 of the magnitude, that bias shrinks 13x on one-sign sums (-0.185 -> -0.014 ulp of scale over 64 steps)
  // and the mean |error| halves (the gc term's Z = out @ feats sums the denoiser output's errors over 7,050 items,
  // where a bias adds up linearly: gc rows 1.1e-5 -> 1.5e-6 off fp64 at baby, profiles/r06j_*).  Cost: +4-7 % on
  // the p_sample products (the 128^2 three-blocks-per-CU tile no longer fits its registers), ~1 ms per epoch.
  floatx16 acc[TM][TN], sml[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = sml[i][j][e] = 0.f;

  // one 16-deep MFMA step s (k = 16 s + 8 h + j: chunk 2 s + h of the 32-deep rows) of a stage
  auto mstep = [&](const __bf16* a_s, int s) {
    const __bf16* b_s = a_s + 3 * APL;
    bf16x8 fb[3][TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn * WTN + j * 32 + l32;
      const int off = row * BK + (((2 * s + h) ^ x6_swz(row)) << 3);
#pragma unroll
      for (int p = 0; p < 3; ++p) fb[p][j] = *reinterpret_cast<const bf16x8*>(b_s + p * BPL + off);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {  // A fragments read per row block: 12 live registers, not 12 TM
      bf16x8 fa[3];
      const int row = wm * WTM + i * 32 + l32;
      const int off = row * BK + (((2 * s + h) ^ x6_swz(row)) << 3);
#pragma unroll
      for (int p = 0; p < 3; ++p) fa[p] = *reinterpret_cast<const bf16x8*>(a_s + p * APL + off);
#pragma unroll
      for (int j = 0; j < TN; ++j) {  // small terms first
        sml[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1][j], sml[i][j], 0, 0, 0);
        sml[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2][j], sml[i][j], 0, 0, 0);
        sml[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0][j], sml[i][j], 0, 0, 0);
        sml[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1][j], sml[i][j], 0, 0, 0);
        sml[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0][j], sml[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0][j], acc[i][j], 0, 0, 0);
      }
    }
  };

  static_assert((AKC && BKC) || PIPE == 0, "m- / n-contiguous operands: the PIPE 0 loop only");
  std::conditional_t<AKC, KcTile<BM, NT>, MnTile<BM, NT>> ra;
  std::conditional_t<BKC, KcTile<BN, NT>, MnTile<BN, NT>> rb;
  ra.init(m0, M, lda);
  rb.init(n0, N, ldb);
  const float* a0 = AKC ? A + m0 * lda : A + m0;
  const float* b0 = BKC ? B + n0 * ldb : B + n0;
  const int nk = kend > kbeg ? (int)((kend - kbeg + BK - 1) / BK) : 0;
  const int kl = (int)(kend - kbeg - (int64_t)(nk - 1) * BK);  // k in the last tile (1..32)
  auto fetch = [&](int t) {
    const int64_t k0 = kbeg + (int64_t)t * BK;
    if constexpr (AKC && BKC) {
      if (t + 1 < nk || kl == BK) {
        ra.load(a0 + k0);
        rb.load(b0 + k0);
      } else {
        ra.load_tail(a0 + k0, kl);
        rb.load_tail(b0 + k0, kl);
      }
    } else {
      const int kleft = t + 1 < nk ? BK : kl;
      if constexpr (AKC) {
        if (kleft == BK) ra.load(a0 + k0);
        else ra.load_tail(a0 + k0, kleft);
      } else {
        ra.load(a0 + k0 * lda, kleft);
      }
      rb.load(b0 + k0 * ldb, kleft);
    }
  };
  auto store = [&](__bf16* s) {  // the registers of one k tile -> the planes of one LDS stage
    if constexpr (AKC) x6_store<BM, true, NT>(ra.r, s);
    else ra.store(s);
    if constexpr (BKC) x6_store<BN, true, NT>(rb.r, s + 3 * APL);
    else rb.store(s + 3 * APL);
  };
  if constexpr (PIPE == 2) {
    // register ring of PF k tiles (the small 64^2 tiles: one 4-wave block per CU at the 2,048-row GenRecV1
    // products, 12 MFMAs per wave per k tile - one tile of prefetch left every k step waiting on its loads):
    // tile t is split into LDS buffer t & 1, then the slot refills with tile t + PF while t is computed.
    // One barrier per tile: a wave storing tile t has passed tile t - 1's barrier, which every wave reaches
    // only after its compute of tile t - 2 (the previous user of buffer t & 1).
    constexpr int PF = 4;
    constexpr int NA = KcTile<BM, NT>::N4, NB = KcTile<BN, NT>::N4;
    float4 qa[PF][NA], qb[PF][NB];
    auto fetch_slot = [&](float4 (&da)[NA], float4 (&db)[NB], int t) {
      if (t < nk) {
        const int64_t k0 = kbeg + (int64_t)t * BK;
        const bool full = t + 1 < nk || kl == BK;
        kc_fetch<BM, NT, NA>(da, ra, a0 + k0, full, kl);
        kc_fetch<BN, NT, NB>(db, rb, b0 + k0, full, kl);
      }
    };
#pragma unroll
    for (int q = 0; q < PF; ++q) fetch_slot(qa[q], qb[q], q);
    for (int t0 = 0; t0 < nk; t0 += PF) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int t = t0 + q;
        if (t < nk) {
          __bf16* buf = smem + (t & 1) * STAGE;
          x6_store<BM, true, NT>(qa[q], buf);
          x6_store<BN, true, NT>(qb[q], buf + 3 * APL);
          __syncthreads();
          fetch_slot(qa[q], qb[q], t + PF);
          mstep(buf, 0);
          mstep(buf, 1);
        }
      }
    }
    __syncthreads();  // every wave is done with the buffers before an LDS epilogue reuses them
  } else if constexpr (PIPE == 0) {
  int cur = 0;
  if (nk > 0) {
    fetch(0);
    store(smem);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const bool more = t + 1 < nk;
    if (more) fetch(t + 1);
    const __bf16* a_s = smem + cur * STAGE;
    mstep(a_s, 0);
    mstep(a_s, 1);
    if constexpr (NBUF == 2) {
      if (more) store(smem + (cur ^ 1) * STAGE);
      __syncthreads();
      cur ^= 1;
    } else {
      __syncthreads();
      if (more) store(smem);
      __syncthreads();
    }
  }
  } else {
    // PIPE = 1 (NBUF = 2): registers double-buffered; tile t+2 loads while tile t is computed and
    // tile t+1 (landed during t-1) is split into the free LDS buffer BETWEEN the MFMAs of tile t
    // (one basic block per step, x6_interleave orders it).  The split runs unconditionally: on the
    // last tile it fills the idle buffer with stale registers that are never read.
    static_assert(NBUF == 2, "the pipelined loop double-buffers LDS");
    constexpr int NA = KcTile<BM, NT>::N4, NB = KcTile<BN, NT>::N4, NF = NA + NB, H0 = (NF + 1) / 2;
    float4 qa[NA], qb[NB];  // tile t+1 while ra / rb take tile t+2
    auto fetch_next = [&](int t) {  // registers of tile t (clamped: past the end a tile is re-read)
      fetch(min(t, nk - 1));
    };
    if (nk > 0) {
      fetch(0);
      x6_store<BM, true, NT>(ra.r, smem);
      x6_store<BN, true, NT>(rb.r, smem + 3 * APL);
      fetch_next(1);
    }
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
#pragma unroll
      for (int i = 0; i < NA; ++i) qa[i] = ra.r[i];
#pragma unroll
      for (int i = 0; i < NB; ++i) qb[i] = rb.r[i];
      if (t + 2 < nk) fetch_next(t + 2);
      const __bf16* a_s = smem + (t & 1) * STAGE;
      __bf16* nxt = smem + ((t & 1) ^ 1) * STAGE;
      // granules [0, H0) of the A|B register list go with step 0, the rest with step 1
      mstep(a_s, 0);
      if constexpr (H0 <= NA) {
        x6_store_part<BM, NT, NA, 0, H0>(qa, nxt);
      } else {
        x6_store_part<BM, NT, NA, 0, NA>(qa, nxt);
        x6_store_part<BN, NT, NB, 0, H0 - NA>(qb, nxt + 3 * APL);
      }
      x6_interleave<6 * (TM + TN), 6 * TM * TN, 3, 3 * H0>();
      mstep(a_s, 1);
      if constexpr (H0 <= NA) {
        x6_store_part<BM, NT, NA, H0, NA>(qa, nxt);
        x6_store_part<BN, NT, NB, 0, NB>(qb, nxt + 3 * APL);
      } else {
        x6_store_part<BN, NT, NB, H0 - NA, NB>(qb, nxt + 3 * APL);
      }
      x6_interleave<6 * (TM + TN), 6 * TM * TN, 3, 3 * (NF - H0)>();
      __syncthreads();
    }
  }

#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] += sml[i][j];

  // epilogues that read an aux / C element per output leave through LDS as float4 row chunks (coalesced
  // C / aux traffic: the p_sample posterior product 870 -> 726 us at 8192 rows); the others store the
  // accumulator fragments directly (the row passes of the LDS epilogue cost the bias-only products)
  if (!ws && epi_reads_x(epi))
    gemm_epilogue_lds<BM, BN, WGM, WGN, NBUF * 3 * (BM + BN) * BK / 2>(acc, reinterpret_cast<float*>(smem), M, N, C,
                                                                     ldc, epi, m0, n0, ws);
  else
    gemm_epilogue<BM, BN, WGM, WGN, 32>(acc, M, N, C, ldc, epi, m0, n0, ws);
}

// 64 x 64 tiles through LDS (row pad 1: conflict-free column reads), 256 threads, 16 elements each;
// reads and writes are 256-byte row segments
__global__ void __launch_bounds__(256) x6_transpose_kernel(const float* __restrict__ src, int64_t ld_src,
                                                           int64_t rows, int64_t cols, float* __restrict__ dst,
                                                           int64_t ld_dst, int64_t tiles_c) {
  __shared__ float t[64][65];
  const int64_t tr = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int64_t r0 = tr * 64, c0 = tc * 64;
  const int x = threadIdx.x & 63, y = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t r = r0 + y + 4 * i, c = c0 + x;
    t[y + 4 * i][x] = (r < rows && c < cols) ? src[r * ld_src + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t c = c0 + y + 4 * i, r = r0 + x;
    if (c < cols && r < rows) dst[c * ld_dst + r] = t[x][y + 4 * i];
  }
}

}  // namespace

namespace gmr_gemm {

void x6_transpose(const float* src, int64_t ld_src, int64_t rows, int64_t cols, float* dst, int64_t ld_dst,
                  hipStream_t st) {
  const int64_t tr = (rows + 63) / 64, tc = (cols + 63) / 64;
  hipLaunchKernelGGL(x6_transpose_kernel, dim3((unsigned)(tr * tc)), dim3(256), 0, st, src, ld_src, rows, cols, dst,
                     ld_dst, tc);
}

// GMR_GEMM_X6_PIPE = 1: the double-buffered kernels split the next tile between the MFMAs (A/B)
static int x6_pipe() {
  static const int v = [] {
    const char* e = getenv("GMR_GEMM_X6_PIPE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// GMR_X6_RING = 0 turns off the register-ring 64^2 kernel (PIPE 2) and its unsplit plans (A/B)
int x6_ring() {
  static const int v = [] {
    const char* e = getenv("GMR_X6_RING");
    return e ? atoi(e) : 1;
  }();
  return v;
}

static int x6_nb128() {
  static const int v = [] {
    const char* e = getenv("GMR_GEMM_X6_NB128");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// GMR_X6_INPLACE = 0 (default): TN / NN split-bf16 calls copy their m- / n-contiguous operands k-contiguous
// first; 1: B read in place (MnTile), A copied; 2: both read in place.  Opt-in: the in-place kernels ran the
// denoiser gradient products 4-10 % slower than copy + k-contiguous kernel, epoch unchanged
// (profiles/r05zt_x6_inplace_*.txt)
int x6_inplace() {
  static const int v = [] {
    const char* e = getenv("GMR_X6_INPLACE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

int x6_launch(int bm, int bn, dim3 grid, hipStream_t st, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
              const float* B, int64_t ldb, float* C, int64_t ldc, const Epi& epi, int tiles_n, int64_t kps, float* ws,
              bool akc, bool bkc) {
#define GMR_X6(BM_, BN_, WGM_, WGN_, NBUF_, OCC_)                                                                \
  {                                                                                                                \
    if (!akc || !bkc) {                                                                                            \
      if (akc)                                                                                                     \
        hipLaunchKernelGGL((gemm_x6_kernel<BM_, BN_, WGM_, WGN_, NBUF_, OCC_, 0, true, false>), grid,              \
                           dim3(64 * WGM_ * WGN_), 0, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps, ws); \
      else if (!bkc)                                                                                               \
        hipLaunchKernelGGL((gemm_x6_kernel<BM_, BN_, WGM_, WGN_, NBUF_, OCC_, 0, false, false>), grid,             \
                           dim3(64 * WGM_ * WGN_), 0, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps, ws); \
      else                                                                                                         \
        return -1;                                                                                                 \
      return 0;                                                                                                    \
    }                                                                                                              \
    if (NBUF_ == 2 && x6_pipe())                                                                                   \
      hipLaunchKernelGGL((gemm_x6_kernel<BM_, BN_, WGM_, WGN_, NBUF_, OCC_, NBUF_ - 1>), grid, dim3(64 * WGM_ * WGN_), \
                         0, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps, ws);                           \
    else                                                                                                           \
      hipLaunchKernelGGL((gemm_x6_kernel<BM_, BN_, WGM_, WGN_, NBUF_, OCC_, 0>), grid, dim3(64 * WGM_ * WGN_), 0,   \
                         st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps, ws);                              \
    return 0;                                                                                                      \
  }
  // 256 x 128 / 128 x 256: one 8-wave block per CU, LDS double-buffered (144 KiB); 128^2: two or three
  // 4-wave blocks per CU, single-buffered (48 KiB each), so one block's split / barrier phase overlaps
  // the others' MFMA steps (GMR_GEMM_X6_NB128 = 1 / 3: always two / three single-buffered blocks,
  // = 2: one double-buffered block per CU; for A/B runs)
  // 64^2 (4 waves of 32^2, LDS double-buffered, 48 KiB: three blocks per CU) for the small products
  if (bm == 64 && bn == 64 && (!akc || !bkc)) return -1;  // 64^2 split tiles: NT calls only (make_plan)
  if (bm == 64 && bn == 64 && x6_ring()) {
    hipLaunchKernelGGL((gemm_x6_kernel<64, 64, 2, 2, 2, 3, 2>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C,
                       ldc, epi, tiles_n, kps, ws);
    return 0;
  }
  if (bm == 64 && bn == 64) GMR_X6(64, 64, 2, 2, 2, 3)
  if (bm == 256 && bn == 128) GMR_X6(256, 128, 4, 2, 2, 1)
  if (bm == 128 && bn == 256) GMR_X6(128, 256, 2, 4, 2, 1)
  if (bm == 128 && bn == 128) {
    // two blocks per CU.  (Three (168 VGPRs) won 4-8 % on the 19445-row p_sample products with one accumulator
    // set (profiles/r02x6_study.txt); with the two sets of round 6 it spills 392 bytes per lane, so it is
    // opt-in, GMR_GEMM_X6_NB128 = 3.)
    const int nb = x6_nb128();
    if (nb == 2) GMR_X6(128, 128, 2, 2, 2, 1)
    if (nb == 3) GMR_X6(128, 128, 2, 2, 1, 3)
    GMR_X6(128, 128, 2, 2, 1, 2)
  }
#undef GMR_X6
  return -1;
}

}  // namespace gmr_gemm
