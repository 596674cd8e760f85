// K3/K4/K6/K9 — fp32 GEMM on the gfx950 f32-input matrix cores (v_mfma_f32_32x32x2_f32).
//
// C[M,N] = epilogue(alpha * op(A)[M,K] * op(B)[K,N], ...), all row-major.
//   op(A): trans_a = 0 -> A stored M x K (lda >= K);  trans_a = 1 -> A stored K x M.
//   op(B): trans_b = 0 -> B stored K x N (ldb >= N);  trans_b = 1 -> B stored N x K.
// Replaces nn.Linear / torch.mm / matmul on the hot path: Denoise layers
// (models/diffmm.py:352-358), modal projections (:117,124), gc loss GEMMs (:472-473),
// full-catalog scoring (:277) and their backward products.
//
// Block: 256 threads = 4 waves in a 2x2 grid; tile BM x BN x 32; each wave owns
// (BM/64) x (BN/64) 32x32 accumulators.  The k order inside a 32-deep tile is
// permuted (MFMA step s, lane half h -> k = 16h + s) so a lane's A/B fragments for
// consecutive steps are contiguous in a k-contiguous LDS row: 4 x ds_read_b128 per
// tile per 16 MFMAs.  m/n-contiguous operands keep an [k][m] LDS image read with
// conflict-free ds_read_b32.  Register-staged double buffer, one barrier per k-tile.
// Split-K (grid.z) writes fp32 partial slabs that a second pass sums in slab order
// (deterministic) and then applies the epilogue.
#include <stdlib.h>

#include <type_traits>

#include "gemm_impl.h"

namespace {
using namespace gmr_gemm;

template <int BM, int BN, int WGM, int WGN, bool AKC, bool BKC, bool VEC, int MF>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_kernel(int64_t M, int64_t N, int64_t K,
                                                             const float* __restrict__ A, int64_t lda,
                                                             const float* __restrict__ B, int64_t ldb,
                                                             float* __restrict__ C, int64_t ldc, Epi epi, int tiles_n,
                                                             int64_t k_per_split, float* __restrict__ ws) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;  // wave tile
  constexpr int TM = WTM / MF, TN = WTN / MF;
  using AccT = typename std::conditional<MF == 32, floatx16, floatx4>::type;
  constexpr int NE = MF == 32 ? 16 : 4;
  using SA = Stage<BM, AKC, VEC, NT>;
  using SB = Stage<BN, BKC, VEC, NT>;
  __shared__ __attribute__((aligned(16))) float smem[2 * (SA::WORDS + SB::WORDS)];
  constexpr int STAGE_WORDS = SA::WORDS + SB::WORDS;

  // XCD-aware remap: blocks b and b+8 share an XCD; give each XCD a contiguous tile range.
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
  const int h = MF == 32 ? lane >> 5 : lane >> 4;     // k group of the lane
  const int l32 = MF == 32 ? lane & 31 : lane & 15;   // row / column of the lane inside a fragment

  AccT acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[i][j][e] = 0.f;

  SA ra;
  SB rb;
  int cur = 0;
  if (kbeg < kend) {
    ra.load(A, lda, m0, M, kbeg, kend);
    rb.load(B, ldb, n0, N, kbeg, kend);
    ra.store(smem);
    rb.store(smem + SA::WORDS);
  }
  __syncthreads();
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    const bool more = k0 + BK < kend;
    if (more) {
      ra.load(A, lda, m0, M, k0 + BK, kend);
      rb.load(B, ldb, n0, N, k0 + BK, kend);
    }
    const float* a_s = smem + cur * STAGE_WORDS;
    const float* b_s = a_s + SA::WORDS;
    if constexpr (MF == 32) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        float4 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag4<AKC, SA::LD>(a_s, wm * WTM + i * 32 + l32, h, qq);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag4<BKC, SB::LD>(b_s, wn * WTN + j * 32 + l32, h, qq);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].x, fb[j].x, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].y, fb[j].y, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].z, fb[j].z, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].w, fb[j].w, acc[i][j], 0, 0, 0);
          }
      }
    } else {
      // k = 8h + 4g + s: frag16 reads the 4 consecutive k of step group g
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        float4 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag16<AKC, SA::LD>(a_s, wm * WTM + i * 16 + l32, 8 * h + 4 * g);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag16<BKC, SB::LD>(b_s, wn * WTN + j * 16 + l32, 8 * h + 4 * g);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
      }
    }
    if (more) {
      ra.store(smem + (cur ^ 1) * STAGE_WORDS);
      rb.store(smem + (cur ^ 1) * STAGE_WORDS + SA::WORDS);
    }
    __syncthreads();
    cur ^= 1;
  }

  gemm_epilogue<BM, BN, WGM, WGN, MF>(acc, M, N, C, ldc, epi, m0, n0, ws);
}

// ---------------------------------------------------------------------------------------------
// glds variant (MF = 32, 16-byte aligned operands): global -> LDS by global_load_lds_dwordx4, no
// register staging and no ds_write pass before the barrier.  One glds wave-instruction writes
// 1 KiB of LDS lane-linearly (base + 16 * lane), so the LDS images are unpadded:
//   k-contiguous operand (KC): [R rows][32 k], the eight 16-byte k chunks of row r stored at
//     chunk c ^ ((r >> 1) & 7) (the XOR goes on the glds SOURCE address and on the read), which
//     keeps the 16-lane groups of a ds_read_b128 fragment read on distinct banks;
//   m-contiguous operand (MC): [32 k][R rows], read with conflict-free ds_read_b32.
// The full 32-deep k tiles go by glds; a partial last tile (K % 32) by zero-filled register loads
// + ds_write into the same images.  Same MFMA order per output as gemm_kernel: bit-identical.
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int kc_swz(int r) { return (r >> 1) & 7; }

// One global_load_lds_dwordx4 (lane -> lds + 16 * lane), issued in inline asm: hipcc treats its own
// glds as a pending LDS write and waits vmcnt(0) before the next ds_read of ANY buffer, which
// would drain the prefetch of tile t+1 before tile t is computed.  hipcc does not count asm loads:
// the kernel waits for them itself (glds_wait) before the barrier that publishes the buffer.
// M0 (the LDS destination base) is saved and restored inside the statement.
__device__ __forceinline__ void glds16(const float* src, float* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_void*)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}
__device__ __forceinline__ void glds_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int R, bool KC, int NW>
__device__ __forceinline__ void glds_tile(const float* __restrict__ p, int64_t ld, int64_t r0, int64_t nrows,
                                          int64_t k0, int64_t kend, float* img, int w, int lane) {
  constexpr int NI = R / 8;  // 1 KiB instructions per operand tile (32 x R floats)
  static_assert(NI % NW == 0, "glds instructions must split evenly over the waves");
#pragma unroll
  for (int i = 0; i < NI / NW; ++i) {
    const int j = w + NW * i;
    const float* src;
    if (KC) {
      const int r = 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ kc_swz(r);
      const int64_t row = min(r0 + r, nrows - 1);  // rows past the edge: any valid row (discarded)
      int64_t k = k0 + 4 * c;
      if (k >= kend) k = k0;  // chunks past K: any valid chunk, zeroed in LDS (glds_zero_tail)
      src = p + row * ld + k;
    } else {
      const int f = 256 * j + 4 * lane;
      const int k = f / R, m = f % R;
      const int64_t row = min(r0 + m, ((nrows - 1) >> 2) << 2);
      src = p + min(k0 + k, kend - 1) * ld + row;
    }
    glds16(src, img + 256 * j);
  }
}

// a partial last k tile (kend - k0 < 32) landed with junk past K: zero it in the LDS image (the
// chunk that straddles K was read whole: ld % 4 == 0 keeps that read inside the row)
template <int R, bool KC, int NT>
__device__ __forceinline__ void glds_zero_tail(float* img, int kvalid) {
  for (int idx = threadIdx.x; idx < R * BK; idx += NT) {
    if (KC) {
      const int r = idx / BK, kk = idx % BK;  // logical (row, k); stored at chunk (kk / 4) ^ swz(r)
      if (kk >= kvalid) img[r * BK + 4 * ((kk >> 2) ^ kc_swz(r)) + (kk & 3)] = 0.f;
    } else {
      const int kk = idx / R;
      if (kk >= kvalid) img[idx] = 0.f;
    }
  }
}

// Final epilogue of one float4 chunk (row m, columns n .. n + 3): bias / x reads and the C store
// are 16-byte where aligned, element-wise at the right edge.
template <bool KC, int R>
__device__ __forceinline__ float4 gfrag(const float* img, int row, int h, int q) {
  if (KC) return *reinterpret_cast<const float4*>(img + row * BK + 4 * ((4 * h + q) ^ kc_swz(row)));
  const int k = 16 * h + 4 * q;
  return make_float4(img[k * R + row], img[(k + 1) * R + row], img[(k + 2) * R + row], img[(k + 3) * R + row]);
}

// In-launch split-K reduction (glds kernel): each k slice stores its slab, publishes it (agent-
// scope release) and counts itself in the tile's counter; the slice that arrives last (acquire)
// sums the slabs in slab order z = 0, 1, ... (the reduce kernel's order: same bits), applies the
// epilogue and resets the counter to 0 for the next call.  Correct for any placement of a tile's
// slices over XCDs; no second launch, and the slabs are re-read while still in L2 / MALL.
template <int BM, int BN, int NT>
__device__ __forceinline__ void splitk_fixup(float* smem, int* cnt, int64_t M, int64_t N, float* __restrict__ C,
                                             int64_t ldc, const Epi& epi, int64_t m0, int64_t n0,
                                             const float* __restrict__ ws) {
  const int splits = (int)gridDim.z;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores are done
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);  // (the one LDS array: no second __shared__ object)
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == splits - 1;
    if (last) {
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    flag[0] = last;
  }
  __syncthreads();
  if (!flag[0]) return;
  const EpiCtx ctx = epi_ctx(epi, C, ldc);
  const bool v_ws = N % 4 == 0 && ((uintptr_t)ws & 15) == 0;
  const int64_t slab = M * N;
  constexpr int C4 = BN / 4;
  for (int idx = threadIdx.x; idx < BM * C4; idx += NT) {
    const int64_t m = m0 + idx / C4, n = n0 + (idx % C4) * 4;
    if (m >= M || n >= N) continue;
    const float* p = ws + m * N + n;
    float a4[4] = {0.f, 0.f, 0.f, 0.f};
    if (v_ws && n + 3 < N) {
      for (int z = 0; z < splits; ++z) {
        const float4 t = *reinterpret_cast<const float4*>(p + (int64_t)z * slab);
        a4[0] += t.x, a4[1] += t.y, a4[2] += t.z, a4[3] += t.w;
      }
    } else {
      for (int z = 0; z < splits; ++z)
        for (int q = 0; q < 4 && n + q < N; ++q) a4[q] += p[(int64_t)z * slab + q];
    }
    epi_store4(epi, C, ldc, N, m, n, a4, ctx);
  }
}

// ST-stage ring of LDS images: tile t + ST - 1 is issued while tile t is computed; each wave
// waits for its own glds with a counted vmcnt (the asm glds are invisible to hipcc's counters),
// then one barrier publishes the tile.  ST = 2 (ST = 3 optional for the 64^2 tiles).
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int WGM, int WGN, bool AKC, bool BKC, int ST>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_glds_kernel(int64_t M, int64_t N, int64_t K,
                                                                  const float* __restrict__ A, int64_t lda,
                                                                  const float* __restrict__ B, int64_t ldb,
                                                                  float* __restrict__ C, int64_t ldc, Epi epi,
                                                                  int tiles_n, int64_t k_per_split,
                                                                  float* __restrict__ ws, int* __restrict__ counters) {
  constexpr int NW = WGM * WGN, NT = 64 * NW;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int AW = BM * BK, STAGE = (BM + BN) * BK;
  constexpr int GPW = (BM + BN) / 8 / NW;  // glds instructions per wave per k tile
  static_assert(ST >= 2 && ST <= 4, "2 to 4 stages");
  __shared__ __attribute__((aligned(16))) float smem[ST * STAGE];

  const int nwg = gridDim.x;
  const int b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  int tmi, tni;
  tile_mn(tile, tiles_n, (int)((M + BM - 1) / BM), tmi, tni);
  const int64_t m0 = (int64_t)tmi * BM;
  const int64_t n0 = (int64_t)tni * BN;
  const int64_t kbeg = (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = min(K, kbeg + k_per_split);
  const int nk = kend > kbeg ? (int)((kend - kbeg + BK - 1) / BK) : 0;  // k tiles; only the last may be partial
  const int kv_last = (int)(kend - kbeg - (int64_t)(nk - 1) * BK);     // its valid k

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w / WGN, wn = w % WGN;
  const int h = lane >> 5, l32 = lane & 31;

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  auto issue = [&](int t) {  // glds of k tile t into ring slot t % ST
    float* img = smem + (t % ST) * STAGE;
    const int64_t k0 = kbeg + (int64_t)t * BK;
    glds_tile<BM, AKC, NW>(A, lda, m0, M, k0, kend, img, w, lane);
    glds_tile<BN, BKC, NW>(B, ldb, n0, N, k0, kend, img + AW, w, lane);
  };
  auto publish = [&](int t) {  // after this wave's glds of tile t landed: share it (zero the tail)
    __syncthreads();
    if (t == nk - 1 && kv_last < BK) {
      float* img = smem + (t % ST) * STAGE;
      glds_zero_tail<BM, AKC, NT>(img, kv_last);
      glds_zero_tail<BN, BKC, NT>(img + AW, kv_last);
      __syncthreads();
    }
  };

#pragma unroll
  for (int t = 0; t < ST - 1; ++t)
    if (t < nk) issue(t);
  if (nk > 0) {
    if (nk >= ST - 1) vm_wait<(ST - 2) * GPW>();  // tile 0 landed, tiles 1 .. ST-2 may be in flight
    else vm_wait<0>();
    publish(0);
  }
  for (int t = 0; t < nk; ++t) {
    const bool refill = t + ST - 1 < nk;
    if (refill) issue(t + ST - 1);  // the slot of tile t - 1, released by the last barrier
    const float* a_s = smem + (t % ST) * STAGE;
    const float* b_s = a_s + AW;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      float4 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = gfrag<AKC, BM>(a_s, wm * WTM + i * 32 + l32, h, qq);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = gfrag<BKC, BN>(b_s, wn * WTN + j * 32 + l32, h, qq);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].x, fb[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].y, fb[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].z, fb[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].w, fb[j].w, acc[i][j], 0, 0, 0);
        }
    }
    if (t + 1 < nk) {
      // tile t + 1 must have landed; tiles t + 2 .. t + ST - 1 (if issued) may stay in flight
      if (refill) vm_wait<(ST - 2) * GPW>();
      else vm_wait<0>();
      publish(t + 1);
    } else {
      __syncthreads();  // every wave is done with the ring before the epilogue reuses it
    }
  }
  if (nk == 0) __syncthreads();
  gemm_epilogue_lds<BM, BN, WGM, WGN>(acc, smem, M, N, C, ldc, epi, m0, n0, ws);
  if (ws && counters) splitk_fixup<BM, BN, NT>(smem, counters + tile, M, N, C, ldc, epi, m0, n0, ws);
}

__global__ void splitk_reduce_kernel(int64_t M, int64_t N, int splits, const float* __restrict__ ws,
                                     float* __restrict__ C, int64_t ldc, Epi epi) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  const int64_t m = idx / N, n = idx % N;
  const int64_t slab = M * N;
  float s = 0.f;
  int z = 0;
  for (; z + 4 <= splits; z += 4) {  // four independent slab loads in flight, summed in slab order
    const float a0 = ws[(int64_t)z * slab + idx], a1 = ws[(int64_t)(z + 1) * slab + idx];
    const float a2 = ws[(int64_t)(z + 2) * slab + idx], a3 = ws[(int64_t)(z + 3) * slab + idx];
    s += a0;
    s += a1;
    s += a2;
    s += a3;
  }
  for (; z < splits; ++z) s += ws[(int64_t)z * slab + idx];
  C[m * ldc + n] = epi_apply(epi, s, m, n, C, ldc);
}

// split-K reduce of an N = 64 product through the modality projection's epilogue and the row normalisation that
// follows it (GMR_EPI_LEAKY_NORM; models/diffmm.py:115-127 then F.normalize, :138-149): 16 lanes per row, each
// element's slabs summed in slab order (splitk_reduce_kernel's bits), C = leaky(alpha s + bias), then
// NF = C / max(|C|, 1e-12) and nrm as normalize_rows_kernel (diffmm.hip) computes them: the bits of the three
// separate passes in one launch
__global__ void splitk_reduce_leaky_norm_kernel(int64_t M, int splits, const float* __restrict__ ws,
                                                float* __restrict__ C, int64_t ldc, Epi epi, float* __restrict__ NF,
                                                int64_t ldnf, float* __restrict__ nrm) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t m = gid >> 4;
  if (m >= M) return;  // (whole 16-lane rows)
  const int c = (int)(gid & 15) * 4;
  const int64_t slab = M * 64, idx = m * 64 + c;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  int z = 0;
  for (; z + 4 <= splits; z += 4) {
    float4 a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = *reinterpret_cast<const float4*>(ws + (int64_t)(z + q) * slab + idx);
#pragma unroll
    for (int q = 0; q < 4; ++q) s = gmr::f4_add(s, a[q]);
  }
  for (; z < splits; ++z) s = gmr::f4_add(s, *reinterpret_cast<const float4*>(ws + (int64_t)z * slab + idx));
  Epi e = epi;
  e.kind = GMR_EPI_LEAKY;
  const float v[4] = {epi_apply(e, s.x, m, c, C, ldc), epi_apply(e, s.y, m, c + 1, C, ldc),
                      epi_apply(e, s.z, m, c + 2, C, ldc), epi_apply(e, s.w, m, c + 3, C, ldc)};
  const float4 f = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(C + m * ldc + c) = f;
  float ss = f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
#pragma unroll
  for (int q = 8; q >= 1; q >>= 1) ss += __shfl_xor(ss, q);
  const float nv = fmaxf(sqrtf(ss), 1e-12f);
  *reinterpret_cast<float4*>(NF + m * ldnf + c) = gmr::f4_scale(1.f / nv, f);
  if (c == 0) nrm[m] = nv;
}

// tile order inside each XCD's contiguous range: G > 1 walks G tile rows per column (the workgroups
// resident on one XCD then share G A-panels and ~resident/G B-panels of each k slab in its L2 instead
// of one A-panel and ~resident B-panels); 0/1 = row-major.  Default: G = 8 for products at least 32
// tiles wide, row-major below (measured, profiles/r03t_*: 19445 x 7050 x 1000 fetches 4.8 -> 1.7 GB per
// launch, the 2048-row diffusion product 457 -> 136 MB, time unchanged; the 8-tile-wide p_sample hidden
// layer fetches more grouped, 1.9 -> 2.4 GB).  GMR_GEMM_GROUP = G forces G for every product.
int tile_group(int64_t tn) {
  static const int g = [] {
    const char* e = getenv("GMR_GEMM_GROUP");
    const int v = e ? atoi(e) : -1;
    return v < 0 ? -1 : (v > 64 ? 64 : v);
  }();
  if (g >= 0) return g;
  return tn >= 32 ? 8 : 0;
}

bool inkernel_fixup() {
  static const bool f = [] {
    const char* e = getenv("GMR_GEMM_FIXUP");
    return e && atoi(e) == 1;
  }();
  return f;
}

// ring depth of the 64^2 glds tiles (GMR_GEMM_STAGES64 = 3 for a 3-slot ring; default 2: the
// 3-slot ring measured no faster on the N = 64 projections, profiles/r02r_gemm.txt)
int stages64() {
  static const int s = [] {
    const char* e = getenv("GMR_GEMM_STAGES64");
    return (e && atoi(e) == 3) ? 3 : 2;
  }();
  return s;
}

template <int BM, int BN, int WGM, int WGN, bool AKC, bool BKC, int MF>
int launch_t(bool vec, bool glds, dim3 grid, hipStream_t st, int64_t M, int64_t N, int64_t K, const float* A,
              int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, const Epi& epi, int tiles_n,
              int64_t kps, float* ws, int* counters) {
  const dim3 blk(64 * WGM * WGN);
  if constexpr (MF == 6) {  // split-bf16 kernel (gemm_x6.hip): NT products, 16-byte aligned (make_plan)
    // -1: no split-bf16 kernel for this tile / operand layout (the caller reports GMR_ERR_ARG)
    return x6_launch(BM, BN, grid, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps, ws, AKC, BKC);
  } else {
  if constexpr (MF == 32) {
    if (vec && glds) {
      if constexpr (BM == 64 && BN == 64) {
        if (stages64() == 3) {
          hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WGM, WGN, AKC, BKC, 3>), grid, blk, 0, st, M, N, K, A, lda, B,
                             ldb, C, ldc, epi, tiles_n, kps, ws, counters);
          return 0;
        }
      }
      hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WGM, WGN, AKC, BKC, 2>), grid, blk, 0, st, M, N, K, A, lda, B, ldb,
                         C, ldc, epi, tiles_n, kps, ws, counters);
      return 0;
    }
  }
  if (vec)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WGM, WGN, AKC, BKC, true, MF>), grid, blk, 0, st, M, N, K, A, lda, B, ldb,
                       C, ldc, epi, tiles_n, kps, ws);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WGM, WGN, AKC, BKC, false, MF>), grid, blk, 0, st, M, N, K, A, lda, B, ldb,
                       C, ldc, epi, tiles_n, kps, ws);
  return 0;
  }
}

template <int BM, int BN, int WGM, int WGN, int MF>
int launch_mf(int ta, int tb, bool vec, bool glds, dim3 grid, hipStream_t st, int64_t M, int64_t N, int64_t K,
               const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, const Epi& epi,
               int tiles_n, int64_t kps, float* ws, int* counters) {
  // AKC = A is k-contiguous (not transposed); BKC = B is k-contiguous (transposed)
  if (!ta && tb)
    return launch_t<BM, BN, WGM, WGN, true, true, MF>(vec, glds, grid, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps,
                                               ws, counters);
  else if (!ta && !tb)
    return launch_t<BM, BN, WGM, WGN, true, false, MF>(vec, glds, grid, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps,
                                                ws, counters);
  else if (ta && !tb)
    return launch_t<BM, BN, WGM, WGN, false, false, MF>(vec, glds, grid, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n,
                                                 kps, ws, counters);
  else
    return launch_t<BM, BN, WGM, WGN, false, true, MF>(vec, glds, grid, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps,
                                                ws, counters);
}

template <int BM, int BN, int WGM, int WGN>
int launch_tile(int mf, bool glds, int ta, int tb, bool vec, dim3 grid, hipStream_t st, int64_t M, int64_t N,
                 int64_t K, const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                 const Epi& epi, int tiles_n, int64_t kps, float* ws, int* counters) {
  if (mf == 6)
    return launch_mf<BM, BN, WGM, WGN, 6>(ta, tb, vec, false, grid, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps, ws,
                                   counters);
  else if (mf == 16)
    return launch_mf<BM, BN, WGM, WGN, 16>(ta, tb, vec, false, grid, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps,
                                    ws, counters);
  else
    return launch_mf<BM, BN, WGM, WGN, 32>(ta, tb, vec, glds, grid, st, M, N, K, A, lda, B, ldb, C, ldc, epi, tiles_n, kps,
                                    ws, counters);
}

// Tile, MFMA shape and split-K choice of gmr_gemm_f32 (tile / split_k = 0: automatic).
// tile | GMR_GEMM_MFMA16 / GMR_GEMM_MFMA32 forces the MFMA shape; otherwise the environment variable
// GMR_GEMM_MFMA (16 or 32, read once) or the built-in default.
// Staging: global_load_lds (gemm_glds_kernel) unless tile | GMR_GEMM_REGSTAGE, or the environment
// variable GMR_GEMM_GLDS = 0 (read once), asks for register staging (gemm_kernel); MFMA16 plans and
// operands that are not 16-byte aligned always take register staging.
struct Plan {
  int tile, bm, bn, splits, mf;
  bool glds;
  int64_t tm, tn, kps;
  int xpose;  // split-bf16 plans of TN / NN / TT calls: 1 = A, 2 = B copied k-contiguous into the workspace
};

int default_mfma() {
  static int mf = [] {
    const char* e = getenv("GMR_GEMM_MFMA");
    return (e && atoi(e) == 16) ? 16 : 32;
  }();
  return mf;
}

// NT products on >= 128^2 tiles take the split-bf16 kernel (fp32-accurate, gemm_x6.hip) unless the call
// passes GMR_GEMM_F32 or the environment sets GMR_GEMM_X6=0 (every product on the fp32-input MFMA)
bool default_x6() {
  static bool x = [] {
    const char* e = getenv("GMR_GEMM_X6");
    return !(e && atoi(e) == 0);
  }();
  return x;
}

// NT products planned on 64^2 tiles also take the split-bf16 kernel (64^2 split tiles, three blocks per CU):
// measured (profiles/r03j_gemm64.txt) 2048 x 512 x 512 19.7 -> 17.1 us, 2048 x 6710 x 256 86.5 -> 68.5,
// 2048 x 7050 x 64 43.6 -> 34.1; the TN / NN forms lose to their operand transposes there (4096 x 64 x
// 7050 TN 49 -> 86 us), so only plain NT calls use it (make_plan).  GMR_GEMM_X6_64=0 turns it off.
bool default_x6_64() {
  static bool x = [] {
    const char* e = getenv("GMR_GEMM_X6_64");
    return !(e && atoi(e) == 0);
  }();
  return x;
}

bool default_glds() {
  static bool g = [] {
    const char* e = getenv("GMR_GEMM_GLDS");
    return !(e && atoi(e) == 0);
  }();
  return g;
}

// automatic split-K: aim for >= 512 workgroups on 256 CUs; skinny 64^2 products (one tile row or
// column: the N = 64 projections) split down to ~192-deep K slabs (measured: 384 x 64 x 7050 TN
// 34 -> 16 us at 32 slabs); the rest keep slabs >= 512 deep, and 128^2 long-K products keep
// splitting while they would run fewer than 8 waves of workgroups or leave the last wave < 90 %
// full (19445 x 1000 x 7050: 2.42 ms unsplit, 2.30 ms at 4 slabs, profiles/r02q_split.txt)
int auto_splits(int64_t tm, int64_t tn, int bm, int64_t K) {
  const bool skinny = bm == 64 && (tm == 1 || tn == 1);
  const int64_t min_k = skinny ? 192 : 512;
  const int max_s = skinny ? 64 : 16;
  int s = 1;
  while (tm * tn * s < 512 && K / (s * 2) >= min_k && s < max_s) s *= 2;
  if (bm == 128) {
    const int64_t slots = 512;  // two 128^2 workgroups per CU
    auto waves = [&](int q) { return (double)(tm * tn * q) / (double)slots; };
    auto fill = [&](int q) {
      const int64_t w = tm * tn * q;
      return (double)w / (double)(((w + slots - 1) / slots) * slots);
    };
    while ((waves(s) < 8.0 || fill(s) < 0.9) && K / (s * 2) >= min_k && s < max_s) s *= 2;
  }
  return s;
}

Plan make_plan_core(int ta, int tb, int64_t M, int64_t N, int64_t K, int tile, int split_k, bool allow_x6) {
  int mf = default_mfma();
  if (tile & GMR_GEMM_MFMA16) mf = 16;
  if (tile & GMR_GEMM_MFMA32) mf = 32;
  bool glds = default_glds();
  if (tile & GMR_GEMM_GLDS) glds = true;
  if (tile & GMR_GEMM_REGSTAGE) glds = false;
  // (the staging and MFMA-shape flags name fp32-kernel variants, so they select the fp32 kernel too)
  const bool x6 = allow_x6 && ((tile & GMR_GEMM_X6) || default_x6()) &&
                  !(tile & (GMR_GEMM_F32 | GMR_GEMM_MFMA16 | GMR_GEMM_MFMA32 | GMR_GEMM_GLDS | GMR_GEMM_REGSTAGE));
  const bool x6_64 = x6 && ((tile & GMR_GEMM_X6) || default_x6_64());
  tile &= ~(GMR_GEMM_MFMA16 | GMR_GEMM_MFMA32 | GMR_GEMM_GLDS | GMR_GEMM_REGSTAGE | GMR_GEMM_X6 | GMR_GEMM_F32);
  if (tile == 0) {
    // measured on MI355X (scripts/gemm_bench.py): 256^2 tiles win the long-K products of the
    // denoiser (M >= 2048, N >= 1000, K >= 4096; one 16-wave block per CU), 128^2 the wide
    // K ~ 1000 ones, 64^2 (with split-K) the skinny N = 64 / K = 64 products and the TN updates.
    // The 2048 x 512 x 512 transformer products (GenRecV1) run best on 64^2 tiles without split-K,
    // their K = 6710 input projection on 128^2, the K = 256 output projection on 256^2.
    // Wide products with 256 <= K <= 1024 take 256^2 unless its last wave is much emptier than
    // 128^2's (a 256^2 tile runs ~8% faster per flop; one 256^2 block or two 128^2 blocks per CU).
    const bool tnm = ta && !tb;
    auto fill = [](int64_t tiles, int64_t slots) { return (double)tiles / (double)(((tiles + slots - 1) / slots) * slots); };
    const bool wide256 = M >= 2048 && N >= 4096 && K >= 256 && K <= 1024 &&
                         fill(((M + 255) / 256) * ((N + 255) / 256), 256) >=
                             0.92 * fill(((M + 127) / 128) * ((N + 127) / 128), 512);
    // Long-K products: 256^2 vs 128^2 by the fill of the last wave of workgroups (one 256^2 or
    // two 128^2 blocks per CU), the split-K slabs each needs (-5 % per doubling) and the 256^2
    // tile's ~3 % per-flop edge: 19445 x 1000 x 7050 (the whole-user p_sample) runs 2.29 ms on
    // 128^2 vs 2.67 on 256^2 with two slabs (profiles/r02l_gemm_g1.txt).  With glds staging the
    // NN form (dh = G W1) is faster on 128^2.
    auto score = [&](int t) {
      const int64_t tm = (M + t - 1) / t, tn = (N + t - 1) / t;
      const int s = auto_splits(tm, tn, t, K);
      double pen = 1.0;
      for (int q = s; q > 1; q >>= 1) pen *= 0.95;
      return fill(tm * tn * s, t == 256 ? 256 : 512) * pen * (t == 256 ? 1.03 : 1.0);
    };
    if (!tnm && M >= 2048 && N >= 1000 && K >= 4096)
      tile = (tb || !glds) && score(256) >= score(128) ? 256 : 128;
    else if (!tnm && wide256) tile = 256;
    else if (!tnm && M * N >= (int64_t)8 << 20 && K >= 512) tile = 128;
    else if (!tnm && M * N >= (int64_t)1 << 20 && K >= 4096) tile = 128;
    // N <= 64 NN products of many rows and long K (the item-feature projections, 7050 x 64 x 4096): 128 x 64
    // tiles, four 64 x 32 wave tiles with two accumulator chains each, 8 slabs: 54.1 -> 49.7 us
    // (profiles/r05zp_tile12864.txt; the TN gradient moves < 1 %, so it keeps 64^2)
    else if (!ta && !tb && N <= 64 && M >= 4096 && K >= 2048) tile = 12864;
    else tile = 64;
  }
  // split-bf16 plans take 128^2 instead of 64^2 for products of >= 4M outputs (the denoiser weight
  // gradients 7050 x 1000 x 2048, TN, run as NT on transposed copies: two 128^2 blocks per CU)
  if (x6 && tile == 64 && M * N >= ((int64_t)4 << 20) && K >= 256) tile = 128;
  // the split-bf16 kernel (gemm_x6.hip): NT products on 128^2, 256 x 128, 128 x 256 and 256^2 tiles
  // (the 256^2 tile maps to 256 x 128: a 2-wave-per-SIMD 256^2 block spills its prefetch registers)
  if (x6 && (tile != 64 || x6_64) && tile != 12864 && !ta && tb) {  // (no 128 x 64 split-bf16 tile)
    mf = 6;
    // products with >= 768 128^2 tiles run three 128^2 blocks per CU (gemm_x6.hip), which beat
    // 256 x 128 there (19445 x 1000 x 7050: 1852 -> 1605 us); smaller ones keep 256 x 128
    if (tile == 256) tile = ((M + 127) / 128) * ((N + 127) / 128) >= 768 ? 128 : 256128;
  }
  Plan p;
  p.mf = mf;
  p.glds = glds && mf == 32;
  p.tile = tile;
  p.bm = tile == 256128 ? 256 : tile == 128256 || tile == 12864 ? 128 : tile;
  p.bn = tile == 256128 ? 128 : tile == 128256 ? 256 : tile == 12864 ? 64 : tile;
  p.tm = (M + p.bm - 1) / p.bm;
  p.tn = (N + p.bn - 1) / p.bn;
  int splits = split_k;
  if (splits <= 0 && mf == 6) {
    // split-bf16 plans: the slabs cost more next to the faster product; split only while the tiles
    // fill < 80 % of the resident slots (256 x 128: one block per CU; 128^2: two) and slabs stay >= 512
    // deep (measured: the 7050 x 1000 x 2048 weight gradients 253 -> 222 us unsplit, the 2048-row
    // diffusion products best at 4 slabs; profiles/r02x6_study.txt)
    // 64^2 plans split down to 256-deep slabs (the GenRecV1 2048 x 512 x 512 decoder products: one tile per
    // CU and a latency-bound 512-deep k loop unsplit; epoch 118.0 -> 114.5 ms, profiles/r04u_ab.txt),
    // the larger tiles to 512 (GMR_X6_MIN_SLAB overrides both, for A/B runs)
    static const int64_t min_slab_env = [] {
      const char* e = getenv("GMR_X6_MIN_SLAB");
      const int v = e ? atoi(e) : 0;
      return (int64_t)(v >= 64 ? v : 0);
    }();
    // with the register-ring 64^2 kernel (gemm_x6.hip PIPE 2) 64^2 products of K <= 1024 run unsplit (the
    // 2048 x 512 x 512 decoder products: no partial slabs, no reduce launch); longer ones keep 256-deep slabs
    // (their sums - e.g. VBPR's K = 4,480 item projection - stay the ones the parity tests pinned)
    const int64_t min_slab = min_slab_env ? min_slab_env : p.bm == 64 ? (x6_ring() && K <= 1024 ? K : 256) : 512;
    const int64_t slots = p.bm == 64 ? 768 : p.bm * p.bn == 128 * 128 ? 512 : 256;
    splits = 1;
    while (p.tm * p.tn * splits * 5 < slots * 4 && K / (splits * 2) >= min_slab && splits < 16) splits *= 2;
  }
  if (splits <= 0) splits = auto_splits(p.tm, p.tn, p.bm, K);
  int64_t kps = (K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  p.splits = (int)((K + kps - 1) / kps);
  p.kps = kps;
  p.xpose = 0;
  return p;
}

// TN / NN / TT calls whose NT form takes the split-bf16 kernel copy their m- / n-contiguous operands
// k-contiguous into the workspace (gemm_x6.hip x6_transpose: 2 x 4 bytes per element, a few percent of
// the product's time at the denoiser shapes) and run as NT; otherwise the fp32-input MFMA plan
Plan make_plan(int ta, int tb, int64_t M, int64_t N, int64_t K, int tile, int split_k) {
  if (ta || !tb) {
    Plan q = make_plan_core(0, 1, M, N, K, tile, split_k, true);
    if (q.mf == 6 && q.bm != 64) {  // 64^2 split tiles: plain NT calls only (the copies cost more there)
      q.xpose = (ta ? 1 : 0) | (tb ? 0 : 2);
      return q;
    }
    return make_plan_core(ta, tb, M, N, K, tile, split_k, false);
  }
  return make_plan_core(ta, tb, M, N, K, tile, split_k, true);
}

// workspace layout of a plan: [tile counters | split slabs (split-K) | A^T (M x Kp) | B^T (N x Kp)],
// segments 16-byte aligned, Kp = K rounded up to 4.  The counter words lead EVERY layout that uses
// the workspace (a shared per-stream scratch whose counters must stay zero between calls), so a
// transposed-operand plan never writes over them.
struct WsLayout {
  int64_t slabs, at, bt, total, kp;
};
WsLayout ws_layout(const Plan& p, int64_t M, int64_t N, int64_t K) {
  auto r4 = [](int64_t v) { return (v + 3) / 4 * 4; };
  WsLayout w;
  w.kp = r4(K);
  const bool uses = p.splits > 1 || p.xpose;
  w.slabs = GMR_GEMM_COUNTER_WORDS;
  w.at = uses ? r4(GMR_GEMM_COUNTER_WORDS + (p.splits > 1 ? (int64_t)p.splits * M * N : 0)) : 0;
  w.bt = w.at + ((p.xpose & 1) ? r4(M * w.kp) : 0);
  w.total = w.bt + ((p.xpose & 2) ? r4(N * w.kp) : 0);
  return w;
}

}  // namespace

extern "C" int32_t gmr_gemm_kernel_kind(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                                        int32_t tile, int32_t split_k, int32_t aligned) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const Plan p = make_plan(trans_a, trans_b, M, N, K, tile, split_k);
  if (p.mf == 6 && !aligned && p.xpose != 3)  // gmr_gemm_f32: k-contiguous operands used in place need alignment
    return make_plan_core(trans_a, trans_b, M, N, K, tile, split_k, false).mf;
  return p.mf;
}

extern "C" int64_t gmr_gemm_workspace_floats(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                                             int32_t tile, int32_t split_k) {
  // exact scratch of gmr_gemm_f32 with the same arguments: the tile-counter words + splits * M * N
  // partial sums, 0 without split-K
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const Plan p = make_plan(trans_a, trans_b, M, N, K, tile, split_k);
  int64_t need = ws_layout(p, M, N, K).total;
  if (p.mf == 6) {  // gmr_gemm_f32 falls back to the fp32 plan when the operands are not 16-byte aligned
    const Plan q = make_plan_core(trans_a, trans_b, M, N, K, tile, split_k, false);
    need = std::max(need, ws_layout(q, M, N, K).total);
  }
  return need;
}

extern "C" int gmr_gemm_f32(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K, float alpha,
                            const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                            int64_t ldc, int32_t epilogue, const float* bias, const int32_t* bias_row, int64_t ld_bias,
                            const float* aux, int64_t ld_aux, const float* rowvec1, const float* rowvec2, float slope,
                            int32_t tile, int32_t split_k, float* workspace, int64_t workspace_floats, void* stream) {
  GMR_ARG(A && B && C, "null operand");
  GMR_ARG(M > 0 && N > 0 && K > 0, "empty GEMM");
  GMR_ARG(lda >= (trans_a ? M : K) && ldb >= (trans_b ? K : N) && ldc >= N, "leading dimension too small");
  GMR_ARG(epilogue >= GMR_EPI_NONE && epilogue <= GMR_EPI_SCALE_BIAS, "bad epilogue");
  GMR_ARG(epilogue != GMR_EPI_LEAKY_NORM ||
              (N == 64 && aux && rowvec1 && ld_aux >= 64 && ld_aux % 4 == 0 && ldc % 4 == 0 &&
               (((uintptr_t)aux | (uintptr_t)C) & 15) == 0),
          "GMR_EPI_LEAKY_NORM: N = 64, 16-byte aligned C and aux (the normalised rows), rowvec1 (the norms)");
  GMR_ARG(!(epilogue == GMR_EPI_POSTERIOR || epilogue == GMR_EPI_DTANH || epilogue == GMR_EPI_ROWSCALE_AUX ||
            epilogue == GMR_EPI_DRELU) || aux,
          "epilogue needs aux");
  GMR_ARG(epilogue != GMR_EPI_ROWSCALE_AUX || rowvec1, "epilogue needs rowvec1");
  {
    const int t = tile & ~(GMR_GEMM_MFMA16 | GMR_GEMM_MFMA32 | GMR_GEMM_GLDS | GMR_GEMM_REGSTAGE | GMR_GEMM_X6 |
                           GMR_GEMM_F32);
    GMR_ARG(t == 0 || t == 64 || t == 128 || t == 256 || t == 256128 || t == 128256 || t == 12864,
            "tile must be 0 (auto), 64, 128, 256, 256128, 128256 or 12864 (| GMR_GEMM_MFMA16 / GMR_GEMM_MFMA32)");
  }
  Epi e;
  e.kind = epilogue;
  e.alpha = alpha;
  e.beta = beta;
  e.slope = slope;
  e.bias = bias;
  e.bias_row = bias_row;
  e.ld_bias = ld_bias;
  e.aux = aux;
  e.ld_aux = ld_aux;
  e.rv1 = rowvec1;
  e.rv2 = rowvec2;
  const bool a16 = ((uintptr_t)A % 16 == 0) && lda % 4 == 0, b16 = ((uintptr_t)B % 16 == 0) && ldb % 4 == 0;
  bool vec = a16 && b16;
  Plan pl = make_plan(trans_a, trans_b, M, N, K, tile, split_k);
  // the split-bf16 kernel loads float4 granules: operands it reads in place must be 16-byte aligned
  if (pl.mf == 6 && !(((pl.xpose & 1) || a16) && ((pl.xpose & 2) || b16)))
    pl = make_plan_core(trans_a, trans_b, M, N, K, tile, split_k, false);
  // GMR_X6_INPLACE = 1 / 2 (opt-in, gemm_x6.hip x6_inplace): TN / NN split-bf16 plans read their n- (and
  // m-) contiguous operands in place (MnTile, single-float loads: any alignment) instead of copying them
  // k-contiguous.  TT calls (A m-contiguous, B k-contiguous) always copy.
  if ((pl.xpose & 2) && x6_inplace()) pl.xpose &= ~2;
  if (pl.xpose == 1 && !trans_b && x6_inplace() == 2) pl.xpose = 0;
  const WsLayout wl = ws_layout(pl, M, N, K);
  if (pl.xpose) {
    GMR_ARG(workspace && workspace_floats >= wl.total, "needs workspace of gmr_gemm_workspace_floats(...) floats");
    GMR_ARG(((uintptr_t)workspace & 15) == 0, "workspace must be 16-byte aligned");
    if (pl.xpose & 1) {  // A stored K x M -> A^T (M x Kp)
      x6_transpose(A, lda, K, M, workspace + wl.at, wl.kp, (hipStream_t)stream);
      GMR_LAUNCHED();
      A = workspace + wl.at;
      lda = wl.kp;
    }
    if (pl.xpose & 2) {  // B stored K x N -> B^T (N x Kp)
      x6_transpose(B, ldb, K, N, workspace + wl.bt, wl.kp, (hipStream_t)stream);
      GMR_LAUNCHED();
      B = workspace + wl.bt;
      ldb = wl.kp;
    }
    if (pl.xpose & 1) trans_a = 0;
    if (pl.xpose & 2) trans_b = 1;
    vec = (pl.xpose & 1 ? true : a16) && (pl.xpose & 2 ? true : b16);
  }
  tile = pl.tile;
  const int64_t tm = pl.tm, tn = pl.tn, kps = pl.kps;
  const int splits = pl.splits;
  GMR_ARG(tm * tn < (1ll << 31), "too many tiles");
  float* ws = nullptr;
  int* counters = nullptr;
  if (splits > 1) {
    GMR_ARG(workspace && workspace_floats >= GMR_GEMM_COUNTER_WORDS + (int64_t)splits * M * N,
            "split-K needs workspace of gmr_gemm_workspace_floats(...) floats");
    ws = workspace + GMR_GEMM_COUNTER_WORDS;
    // GMR_GEMM_FIXUP=1: the glds kernel reduces in-launch through per-tile counters (words
    // [0, tiles) of the workspace, zero on entry and on exit).  Off by default: each slice's
    // agent-scope release writes back its XCD's L2, and that cost more than the reduce launch it
    // saves (projections 15 -> 48 us, 19445 x 1000 x 7050 2.30 -> 2.59 ms; profiles/r02u_fixup.txt)
    if (pl.glds && vec && tm * tn <= GMR_GEMM_COUNTER_WORDS && inkernel_fixup() && epilogue != GMR_EPI_LEAKY_NORM)
      counters = reinterpret_cast<int*>(workspace);
  }
  GMR_ARG(epilogue != GMR_EPI_LEAKY_NORM || splits > 1, "GMR_EPI_LEAKY_NORM needs a split-K plan");
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)(tm * tn), 1, (unsigned)splits);
  const int tnp = (int)tn | (tile_group(tn) << 20);
  int lrc = 0;
  switch (tile) {
    case 256:
      lrc = launch_tile<256, 256, 4, 4>(pl.mf, pl.glds, trans_a, trans_b, vec, grid, st, M, N, K, A, lda, B, ldb, C, ldc, e, tnp, kps, ws, counters);
      break;
    case 256128:
      lrc = launch_tile<256, 128, 4, 2>(pl.mf, pl.glds, trans_a, trans_b, vec, grid, st, M, N, K, A, lda, B, ldb, C, ldc, e, tnp, kps, ws, counters);
      break;
    case 128256:
      lrc = launch_tile<128, 256, 2, 4>(pl.mf, pl.glds, trans_a, trans_b, vec, grid, st, M, N, K, A, lda, B, ldb, C, ldc, e, tnp, kps, ws, counters);
      break;
    case 12864:
      lrc = launch_tile<128, 64, 2, 2>(pl.mf, pl.glds, trans_a, trans_b, vec, grid, st, M, N, K, A, lda, B, ldb, C, ldc, e, tnp, kps, ws, counters);
      break;
    case 128:
      lrc = launch_tile<128, 128, 2, 2>(pl.mf, pl.glds, trans_a, trans_b, vec, grid, st, M, N, K, A, lda, B, ldb, C, ldc, e, tnp, kps, ws, counters);
      break;
    default:
      lrc = launch_tile<64, 64, 2, 2>(pl.mf, pl.glds, trans_a, trans_b, vec, grid, st, M, N, K, A, lda, B, ldb, C, ldc, e, tnp, kps, ws, counters);
  }
  GMR_ARG(lrc == 0, "no split-bf16 kernel for this tile and operand layout");
  GMR_LAUNCHED();
  if (ws && !counters && epilogue == GMR_EPI_LEAKY_NORM) {
    hipLaunchKernelGGL(splitk_reduce_leaky_norm_kernel, dim3(gmr::grid_for(M * 16, 256)), dim3(256), 0, st, M, splits,
                       ws, C, ldc, e, const_cast<float*>(aux), ld_aux, const_cast<float*>(rowvec1));
    GMR_LAUNCHED();
  } else if (ws && !counters) {
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(gmr::grid_for(M * N, 256)), dim3(256), 0, st, M, N, splits, ws, C,
                       ldc, e);
    GMR_LAUNCHED();
  }
  return GMR_OK;
}
