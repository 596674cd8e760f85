// K3/K4 — fp32 GEMM on the bf16 matrix cores from PRE-SPLIT operands (the p_sample products of the
// graph rebuild: models/diffmm.py:352-358, 408-451; common/trainer.py:529-546).
//
// gemm_x6.hip splits every fp32 operand element into three bf16 terms on its way into LDS; per 32-deep
// k tile a 128^2 block spends ~280 VALU instructions per wave and 48 KiB of LDS writes on that split for
// 48 MFMAs, which is where its time goes.  Here the PRODUCERS write the operands
// once as three bf16 planes (x = hi + mid + lo exactly, the split3 of gemm_x6.hip): the rebuild's
// denoiser weights once per rebuild (gmr_split3_planes), the p_sample state x and the hidden layer h by
// the epilogues of the products that make them.  The k loop is then a plain bf16 GEMM: each 32-deep k
// tile goes global -> LDS by global_load_lds_dwordx4 (16 rows x 64 B of one plane per wave
// instruction, no staging registers, no VALU), and the waves run the same six bf16 MFMA products per
// 32x32x16 block as gemm_x6 (hi.hi + hi.mid + mid.hi + hi.lo + lo.hi + mid.mid, small terms first):
// the same fp32 accuracy (test_kernels_gpu.py::test_gemm_p3_*).
//
// Plane layout (caller-owned, bf16 as uint16): [3][rows][ld] with plane stride ps, k contiguous,
// ld a multiple of 32 and the columns [K, ld) ZERO (the split kernel writes them; a planes epilogue
// never touches them), so every k tile is full: no tail, no bounds test in the loop.  Rows past the
// operand's end are clamped onto its last row (their products only reach discarded outputs).
// LDS: per stage 3 (BM + BN) rows x 64 B; chunk c of row r stored at c ^ ((r >> 2) & 3) (the XOR goes on
// the glds SOURCE address and on the ds_read_b128 fragment read: conflict-free, as gemm_x6).
// Epilogue through LDS as float4 row chunks (gemm_epilogue_lds form): fp32 C and/or output planes;
// the POSTERIOR aux may be given as planes (x = (hi + mid) + lo, exact).
#include <stdlib.h>

#include "gemm_impl.h"

namespace {
using namespace gmr_gemm;

typedef __bf16 p3bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 p3bf4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void p3_lds_void;

__device__ __forceinline__ int p3_swz(int r) { return (r >> 2) & 3; }

// x = hi + mid + lo exactly (clamped into bf16 range first: gemm_x6.hip split3)
__device__ __forceinline__ void p3_split(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)__builtin_amdgcn_fmed3f(x, -0x1.fep127f, 0x1.fep127f);
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

// one global_load_lds_dwordx4 (lane -> lds + 16 * lane); asm so hipcc does not wait vmcnt(0) before the next
// ds_read (gemm.hip glds16); M0 saved and restored inside the statement
__device__ __forceinline__ void p3_glds16(const void* src, void* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(p3_lds_void*)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}
__device__ __forceinline__ void p3_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// 3 planes x R rows x 32 k of one operand -> LDS [plane][row][4 chunks]
template <int R, int NW>
__device__ __forceinline__ void p3_tile(const __bf16* __restrict__ p, int64_t ld, int64_t ps, int64_t r0, int64_t nrows,
                                        int64_t k0, __bf16* img, int w, int lane) {
  constexpr int NI = 3 * R / 16;  // 1 KiB wave instructions
  static_assert(NI % NW == 0, "glds instructions must split evenly over the waves");
#pragma unroll
  for (int i = 0; i < NI / NW; ++i) {
    const int j = w + NW * i;
    const int plane = j / (R / 16), rb = (j % (R / 16)) * 16;
    const int r = rb + (lane >> 2);
    const int c = (lane & 3) ^ p3_swz(r);
    const int64_t row = min(r0 + r, nrows - 1);
    p3_glds16(p + plane * ps + row * ld + k0 + 8 * c, img + (plane * R + rb) * BK);
  }
}

struct P3Out {
  float* C;                 // fp32 output (or null)
  int64_t ldc;
  __bf16* P;                // output planes (or null)
  int64_t ldp, psp;
  const __bf16* auxp;       // POSTERIOR aux as planes (or null: epi.aux, fp32)
  int64_t ld_auxp, ps_auxp;
};

__device__ __forceinline__ float4 p3_ld_planes4(const __bf16* p, int64_t ps) {
  const p3bf4 h = *reinterpret_cast<const p3bf4*>(p);
  const p3bf4 m = *reinterpret_cast<const p3bf4*>(p + ps);
  const p3bf4 l = *reinterpret_cast<const p3bf4*>(p + 2 * ps);
  float v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = ((float)h[q] + (float)m[q]) + (float)l[q];  // exact
  return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void p3_st_planes4(__bf16* p, int64_t ps, const float (&o)[4]) {
  p3bf4 h, m, l;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    __bf16 a, b, c;
    p3_split(o[q], a, b, c);
    h[q] = a;
    m[q] = b;
    l[q] = c;
  }
  *reinterpret_cast<p3bf4*>(p) = h;
  *reinterpret_cast<p3bf4*>(p + ps) = m;
  *reinterpret_cast<p3bf4*>(p + 2 * ps) = l;
}

__device__ __forceinline__ const float* p3_xptr(const Epi& epi, const P3Out& o, int64_t m, int64_t n) {
  return (epi.kind == GMR_EPI_NONE || epi.kind == GMR_EPI_BIAS) ? o.C + m * o.ldc + n : epi.aux + m * epi.ld_aux + n;
}

// fragments -> LDS (fp32 rows of BN) -> float4 row chunks -> epi_fin -> fp32 C and / or planes
template <int BM, int BN, int WGM, int WGN, int AVAIL>
__device__ __forceinline__ void p3_epilogue(const floatx16 (&acc)[BM / WGM / 32][BN / WGN / 32], float* smem,
                                            int64_t M, int64_t N, const Epi& epi, const P3Out& o, int64_t m0,
                                            int64_t n0) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN, TM = WTM / 32, TN = WTN / 32;
  constexpr int HR0 = (AVAIL / BN) / 32 * 32;
  constexpr int HR = HR0 < BM ? HR0 : BM;
  static_assert(HR >= 32, "LDS too small for one 32-row pass");
  constexpr int C4 = BN / 4;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w / WGN, wn = w % WGN, h = lane >> 5, l32 = lane & 31;
  const bool rx = epi_reads_x(epi);
#pragma unroll
  for (int r0 = 0; r0 < BM; r0 += HR) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rb = wm * WTM + i * 32;
      if (rb < r0 || rb >= r0 + HR) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WTN + j * 32 + l32;
#pragma unroll
        for (int e = 0; e < 16; ++e) smem[(rb - r0 + (e & 3) + 8 * (e >> 2) + 4 * h) * BN + col] = acc[i][j][e];
      }
    }
    __syncthreads();
    const int rows = BM - r0 < HR ? BM - r0 : HR;
    for (int idx = threadIdx.x; idx < rows * C4; idx += NT) {
      const int rr = idx / C4, c = (idx % C4) * 4;
      const int64_t m = m0 + r0 + rr, n = n0 + c;
      if (m >= M || n >= N) continue;
      const float4 v = *reinterpret_cast<const float4*>(smem + rr * BN + c);
      const float a4[4] = {v.x, v.y, v.z, v.w};
      const bool full = n + 3 < N;  // the right edge (N % 4 != 0) goes element by element
      float b4[4] = {0.f, 0.f, 0.f, 0.f}, x4[4] = {0.f, 0.f, 0.f, 0.f};
      if (full) {
        if (epi.bias) {
          const float4 t = *reinterpret_cast<const float4*>(epi.bias + n);
          b4[0] = t.x, b4[1] = t.y, b4[2] = t.z, b4[3] = t.w;
        }
        if (rx) {
          float4 x;
          if (o.auxp) x = p3_ld_planes4(o.auxp + m * o.ld_auxp + n, o.ps_auxp);
          else x = *reinterpret_cast<const float4*>(p3_xptr(epi, o, m, n));
          x4[0] = x.x, x4[1] = x.y, x4[2] = x.z, x4[3] = x.w;
        }
      } else {
        for (int q = 0; q < 4 && n + q < N; ++q) {
          if (epi.bias) b4[q] = epi.bias[n + q];
          if (rx) {
            if (o.auxp) {
              const __bf16* ap = o.auxp + m * o.ld_auxp + n + q;
              x4[q] = ((float)ap[0] + (float)ap[o.ps_auxp]) + (float)ap[2 * o.ps_auxp];
            } else {
              x4[q] = p3_xptr(epi, o, m, n)[q];
            }
          }
        }
      }
      const float r1 = epi_r1(epi, m), r2 = epi_r2(epi, m);
      float o4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o4[q] = epi_fin(epi, a4[q], b4[q], x4[q], r1, r2);
      if (full) {
        if (o.C) *reinterpret_cast<float4*>(o.C + m * o.ldc + n) = make_float4(o4[0], o4[1], o4[2], o4[3]);
        if (o.P) p3_st_planes4(o.P + m * o.ldp + n, o.psp, o4);
      } else {
        for (int q = 0; q < 4 && n + q < N; ++q) {
          if (o.C) o.C[m * o.ldc + n + q] = o4[q];
          if (o.P) {
            __bf16 a, b, cc;
            p3_split(o4[q], a, b, cc);
            __bf16* pp = o.P + m * o.ldp + n + q;
            pp[0] = a;
            pp[o.psp] = b;
            pp[2 * o.psp] = cc;
          }
        }
      }
    }
  }
}

// NBUF = 2: LDS double-buffered, tile t + 1 loads while tile t is computed (one barrier per k tile);
// NBUF = 1: one buffer, OCC blocks per CU overlap one another's loads and MFMA steps
template <int BM, int BN, int WGM, int WGN, int NBUF, int OCC>
__global__ void __launch_bounds__(64 * WGM * WGN, OCC) gemm_p3_kernel(int64_t M, int64_t N, int64_t Kp,
                                                                   const __bf16* __restrict__ A, int64_t lda,
                                                                   int64_t psa, const __bf16* __restrict__ B,
                                                                   int64_t ldb, int64_t psb, Epi epi, P3Out out,
                                                                   int tiles_n) {
  constexpr int NW = WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN, TM = WTM / 32, TN = WTN / 32;
  constexpr int APL = BM * BK, BPL = BN * BK, STAGE = 3 * (APL + BPL);
  __shared__ __attribute__((aligned(16))) __bf16 smem[NBUF * STAGE];
  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  int tmi, tni;
  tile_mn(tile, tiles_n, (int)((M + BM - 1) / BM), tmi, tni);
  const int64_t m0 = (int64_t)tmi * BM, n0 = (int64_t)tni * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w / WGN, wn = w % WGN, h = lane >> 5, l32 = lane & 31;
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int nk = (int)(Kp / BK);
  auto issue = [&](int t) {
    __bf16* img = smem + (NBUF == 2 ? (t & 1) * STAGE : 0);
    p3_tile<BM, NW>(A, lda, psa, m0, M, (int64_t)t * BK, img, w, lane);
    p3_tile<BN, NW>(B, ldb, psb, n0, N, (int64_t)t * BK, img + 3 * APL, w, lane);
  };
  if (nk > 0) {
    issue(0);
    p3_wait_all();
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const bool more = t + 1 < nk;
    if (NBUF == 2 && more) issue(t + 1);  // the buffer of tile t - 1, released by the last barrier
    const __bf16* a_s = smem + (NBUF == 2 ? (t & 1) * STAGE : 0);
    const __bf16* b_s = a_s + 3 * APL;
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // 16-deep MFMA step s: k = 16 s + 8 h + 0..7 (chunk 2 s + h)
      p3bf8 fb[3][TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WTN + j * 32 + l32;
        const int off = row * BK + (((2 * s + h) ^ p3_swz(row)) << 3);
#pragma unroll
        for (int p = 0; p < 3; ++p) fb[p][j] = *reinterpret_cast<const p3bf8*>(b_s + p * BPL + off);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        p3bf8 fa[3];
        const int row = wm * WTM + i * 32 + l32;
        const int off = row * BK + (((2 * s + h) ^ p3_swz(row)) << 3);
#pragma unroll
        for (int p = 0; p < 3; ++p) fa[p] = *reinterpret_cast<const p3bf8*>(a_s + p * APL + off);
#pragma unroll
        for (int j = 0; j < TN; ++j) {  // small terms first (gemm_x6.hip order)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0][j], acc[i][j], 0, 0, 0);
        }
      }
    }
    if (NBUF == 2) {
      if (more) p3_wait_all();  // this wave's glds of tile t + 1 landed
      __syncthreads();          // ... and everyone's: publish it; the buffer of tile t is free
    } else {
      __syncthreads();  // every wave is done reading the one buffer
      if (more) {
        issue(t + 1);
        p3_wait_all();
        __syncthreads();
      }
    }
  }
  p3_epilogue<BM, BN, WGM, WGN, NBUF * STAGE / 2>(acc, reinterpret_cast<float*>(smem), M, N, epi, out, m0, n0);
}

// fp32 [rows][cols] (ld_src) -> three bf16 planes [rows][ld_dst] (plane stride ps), columns [cols, ld_dst)
// zeroed; one thread per 4 columns (cols % 4 == 0 not required: the edge chunk is masked)
__global__ void __launch_bounds__(256) split3_planes_kernel(int64_t rows, int64_t cols, const float* __restrict__ src,
                                                            int64_t ld_src, __bf16* __restrict__ dst, int64_t ld_dst,
                                                            int64_t ps) {
  const int64_t c4n = ld_dst / 4;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < rows * c4n;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = g / c4n, c = (g % c4n) * 4;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = c + q < cols ? src[r * ld_src + c + q] : 0.f;
    p3_st_planes4(dst + r * ld_dst + c, ps, v);
  }
}

template <int BM, int BN, int WGM, int WGN, int NBUF, int OCC>
void p3_launch(hipStream_t st, int64_t M, int64_t N, int64_t Kp, const __bf16* A, int64_t lda, int64_t psa,
               const __bf16* B, int64_t ldb, int64_t psb, const Epi& epi, const P3Out& o, int group) {
  const int tm = (int)((M + BM - 1) / BM), tn = (int)((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_p3_kernel<BM, BN, WGM, WGN, NBUF, OCC>), dim3((unsigned)(tm * tn)), dim3(64 * WGM * WGN), 0,
                     st, M, N, Kp, A, lda, psa, B, ldb, psb, epi, o, tn | (group << 20));
}

// tile: 0 = by shape; GMR_GEMM_P3_TILE = 1 (256 x 128, double-buffered), 2 (128^2 double-buffered),
// 3 (128^2, single-buffered, three blocks per CU) for A/B runs
int p3_tile_env() {
  static const int v = [] {
    const char* e = getenv("GMR_GEMM_P3_TILE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

}  // namespace

extern "C" int gmr_split3_planes(int64_t rows, int64_t cols, const float* src, int64_t ld_src, uint16_t* dst,
                                 int64_t ld_dst, int64_t plane_stride, void* stream) {
  GMR_ARG(src && dst && rows >= 0 && cols >= 0 && ld_src >= cols, "bad arguments");
  GMR_ARG(ld_dst >= cols && ld_dst % 32 == 0 && plane_stride >= rows * ld_dst, "ld_dst: multiple of 32 >= cols");
  GMR_ARG(((uintptr_t)dst & 7) == 0 && plane_stride % 4 == 0, "planes must be 8-byte aligned");
  if (rows == 0) return GMR_OK;
  hipLaunchKernelGGL(split3_planes_kernel, dim3(gmr::grid_for(rows * (ld_dst / 4), 256, 16384)), dim3(256), 0,
                     (hipStream_t)stream, rows, cols, src, ld_src, reinterpret_cast<__bf16*>(dst), ld_dst, plane_stride);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_gemm_p3_f32(int64_t M, int64_t N, int64_t Kp, float alpha, const uint16_t* A, int64_t lda,
                               int64_t psa, const uint16_t* B, int64_t ldb, int64_t psb, float* C, int64_t ldc,
                               uint16_t* C_planes, int64_t ldcp, int64_t pscp, int32_t epilogue, const float* bias,
                               const float* aux, int64_t ld_aux, const uint16_t* aux_planes, int64_t ld_auxp,
                               int64_t ps_auxp, float slope, float beta, int32_t tile, void* stream) {
  GMR_ARG(A && B && (C || C_planes), "null operand / no output");
  GMR_ARG(M > 0 && N > 0 && Kp > 0 && Kp % 32 == 0, "M, N > 0; Kp a positive multiple of 32");
  GMR_ARG(lda >= Kp && ldb >= Kp && lda % 8 == 0 && ldb % 8 == 0, "plane leading dimensions: multiples of 8, >= Kp");
  GMR_ARG(psa >= M * lda && psb >= N * ldb && psa % 8 == 0 && psb % 8 == 0, "plane strides");
  GMR_ARG((((uintptr_t)A | (uintptr_t)B) & 15) == 0, "operand planes must be 16-byte aligned");
  GMR_ARG(!C || (ldc >= N && ldc % 4 == 0 && ((uintptr_t)C & 15) == 0), "C: 16-byte aligned, ldc % 4 == 0");
  GMR_ARG(!C_planes || (ldcp >= N && ldcp % 4 == 0 && pscp >= M * ldcp && ((uintptr_t)C_planes & 7) == 0),
          "output planes: 8-byte aligned, ld % 4 == 0");
  GMR_ARG(epilogue == GMR_EPI_NONE || epilogue == GMR_EPI_BIAS || epilogue == GMR_EPI_BIAS_TANH ||
              epilogue == GMR_EPI_POSTERIOR,
          "epilogue: NONE, BIAS, BIAS_TANH or POSTERIOR");
  GMR_ARG(!(epilogue == GMR_EPI_BIAS || epilogue == GMR_EPI_BIAS_TANH || epilogue == GMR_EPI_POSTERIOR) ||
              (bias && ((uintptr_t)bias & 15) == 0),
          "this epilogue needs a 16-byte aligned bias");
  GMR_ARG(epilogue != GMR_EPI_POSTERIOR ||
              (aux_planes ? (ld_auxp % 4 == 0 && ps_auxp >= M * ld_auxp && ((uintptr_t)aux_planes & 7) == 0)
                          : (aux && ld_aux % 4 == 0 && ((uintptr_t)aux & 15) == 0)),
          "POSTERIOR needs aux (fp32, 16-byte aligned) or aux planes");
  GMR_ARG(!((epilogue == GMR_EPI_NONE || epilogue == GMR_EPI_BIAS) && beta != 0.f && !C), "beta != 0 reads C");
  Epi e{};
  e.kind = epilogue;
  e.alpha = alpha;
  e.beta = beta;
  e.slope = slope;
  e.bias = bias;
  e.aux = aux;
  e.ld_aux = ld_aux;
  P3Out o{C, ldc, reinterpret_cast<__bf16*>(C_planes), ldcp, pscp, reinterpret_cast<const __bf16*>(aux_planes),
          ld_auxp, ps_auxp};
  const __bf16* a = reinterpret_cast<const __bf16*>(A);
  const __bf16* b = reinterpret_cast<const __bf16*>(B);
  const hipStream_t st = (hipStream_t)stream;
  int t = tile > 0 ? tile : p3_tile_env();
  // by shape (scripts/micro/p3_micro.hip at the rebuild products, profiles/r04c_p3_micro.txt): 256 x 128 for
  // wide products (19445 x 7050 x 1000: 1.53 ms vs 1.79 / 1.69 on the 128^2 tiles), three single-buffered
  // 128^2 blocks per CU for narrow ones (19445 x 1000 x 7050: 1.63 ms vs 1.71 on 256 x 128)
  if (t <= 0) t = (N > 1024 && ((M + 255) / 256) * ((N + 127) / 128) >= 512) ? 1 : 3;
  const int tn = (int)((N + 127) / 128);
  const int group = tn >= 32 ? 8 : 0;  // gemm.hip tile_group: G tile rows per column on wide products
  if (t == 1) p3_launch<256, 128, 4, 2, 2, 1>(st, M, N, Kp, a, lda, psa, b, ldb, psb, e, o, group);
  else if (t == 2) p3_launch<128, 128, 2, 2, 2, 1>(st, M, N, Kp, a, lda, psa, b, ldb, psb, e, o, group);
  else p3_launch<128, 128, 2, 2, 1, 3>(st, M, N, Kp, a, lda, psa, b, ldb, psb, e, o, group);
  GMR_LAUNCHED();
  return GMR_OK;
}
