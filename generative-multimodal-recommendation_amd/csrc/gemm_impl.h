// Shared parts of the fp32-operand GEMM kernels (gemm.hip: fp32 MFMA; gemm_x6.hip: split-bf16 MFMA):
// epilogue descriptor and its per-element math, register staging of operand tiles, the MFMA-layout
// epilogue and the tile order.  See gemm.hip for the operand conventions.
#pragma once
#include <type_traits>

#include "gmr_common.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace gmr_gemm {

constexpr int BK = 32;

struct Epi {
  int kind;
  float alpha, beta, slope;
  const float* bias;
  const int* bias_row;
  int64_t ld_bias;
  const float* aux;
  int64_t ld_aux;
  const float* rv1;
  const float* rv2;
};

// Per-element inputs of the epilogue, loaded in one batch before any store (the p_sample
// posterior runs in place, C == aux, so a load/compute/store chain per element would make every
// element a dependent memory round trip).
__device__ __forceinline__ bool epi_reads_x(const Epi& e) {
  return e.kind == GMR_EPI_POSTERIOR || e.kind == GMR_EPI_DTANH || e.kind == GMR_EPI_ROWSCALE_AUX ||
         e.kind == GMR_EPI_DRELU || ((e.kind == GMR_EPI_NONE || e.kind == GMR_EPI_BIAS) && e.beta != 0.f);
}
__device__ __forceinline__ const float* epi_x_ptr(const Epi& e, float* C, int64_t ldc, int64_t m, int64_t n) {
  return (e.kind == GMR_EPI_NONE || e.kind == GMR_EPI_BIAS) ? C + m * ldc + n : e.aux + m * e.ld_aux + n;
}
// r1 / r2: the POSTERIOR row coefficients (rv1[m] or slope, rv2[m] or beta), ROWSCALE_AUX's rv1[m]
__device__ __forceinline__ float epi_fin(const Epi& e, float acc, float b, float x, float r1, float r2) {
  float v = e.alpha * acc;
  switch (e.kind) {
    case GMR_EPI_NONE:
      return e.beta != 0.f ? fmaf(e.beta, x, v) : v;
    case GMR_EPI_BIAS:
      v += b;
      return e.beta != 0.f ? fmaf(e.beta, x, v) : v;
    case GMR_EPI_BIAS_TANH:
      return tanhf(v + b);
    case GMR_EPI_LEAKY:
      v += b;
      return v > 0.f ? v : v * e.slope;
    case GMR_EPI_POSTERIOR:
      return r1 * (v + b) + r2 * x;
    case GMR_EPI_DTANH:
      return v * (1.f - x * x);
    case GMR_EPI_ROWSCALE_AUX:
      return v + b + r1 * x;
    case GMR_EPI_BIAS_RELU:
      return fmaxf(v + b, 0.f);
    case GMR_EPI_DRELU:
      return x > 0.f ? v : 0.f;
    case GMR_EPI_SCALE_BIAS:  // = POSTERIOR with c2 = 0: c1 (v + b) + 0 x rounds once, like c1 (v + b)
      return e.slope * (v + b);
    default:
      return v;
  }
}
__device__ __forceinline__ float epi_r1(const Epi& e, int64_t m) {
  if (e.kind == GMR_EPI_POSTERIOR) return e.rv1 ? e.rv1[m] : e.slope;
  if (e.kind == GMR_EPI_ROWSCALE_AUX) return e.rv1[m];
  return 0.f;
}
__device__ __forceinline__ float epi_r2(const Epi& e, int64_t m) {
  return e.kind == GMR_EPI_POSTERIOR ? (e.rv2 ? e.rv2[m] : e.beta) : 0.f;
}
// scalar form (split-K reduce)
__device__ __forceinline__ float epi_apply(const Epi& e, float acc, int64_t m, int64_t n, float* C, int64_t ldc) {
  const float b = e.bias ? e.bias[(e.bias_row ? (int64_t)e.bias_row[m] : 0) * e.ld_bias + n] : 0.f;
  const float x = epi_reads_x(e) ? *epi_x_ptr(e, C, ldc, m, n) : 0.f;
  return epi_fin(e, acc, b, x, epi_r1(e, m), epi_r2(e, m));
}

// Loads a BK-deep tile slice of an operand into registers (float4 granules).
// KC: operand stored [rows][k] (k contiguous), tile = R rows x BK.
// MC: operand stored [k][rows] (rows contiguous), tile = BK x R.
template <int R, bool KC, bool VEC, int NT>
struct Stage {
  static constexpr int N4 = R * BK / 4 / NT;  // float4 per thread
  static_assert(N4 * NT * 4 == R * BK, "tile rows x BK must split evenly over the block");
  float4 r[N4];

  __device__ __forceinline__ void load(const float* __restrict__ p, int64_t ld, int64_t r0, int64_t nrows,
                                       int64_t k0, int64_t K) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < N4; ++i) {
      const int idx = t + NT * i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (KC) {
        const int rr = idx / (BK / 4), k4 = (idx % (BK / 4)) * 4;
        const int64_t row = r0 + rr, k = k0 + k4;
        if (row < nrows) {
          const float* q = p + row * ld + k;
          if (VEC && k + 3 < K) {
            v = *reinterpret_cast<const float4*>(q);
          } else {
            if (k < K) v.x = q[0];
            if (k + 1 < K) v.y = q[1];
            if (k + 2 < K) v.z = q[2];
            if (k + 3 < K) v.w = q[3];
          }
        }
      } else {
        const int kk = idx / (R / 4), m4 = (idx % (R / 4)) * 4;
        const int64_t k = k0 + kk, row = r0 + m4;
        if (k < K) {
          const float* q = p + k * ld + row;
          if (VEC && row + 3 < nrows) {
            v = *reinterpret_cast<const float4*>(q);
          } else {
            if (row < nrows) v.x = q[0];
            if (row + 1 < nrows) v.y = q[1];
            if (row + 2 < nrows) v.z = q[2];
            if (row + 3 < nrows) v.w = q[3];
          }
        }
      }
      r[i] = v;
    }
  }

  // LDS images: KC -> [R][BK + 4] ; MC -> [BK][R + 4]
  static constexpr int LD = KC ? BK + 4 : R + 4;
  static constexpr int WORDS = KC ? R * (BK + 4) : BK * (R + 4);

  __device__ __forceinline__ void store(float* s) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < N4; ++i) {
      const int idx = t + NT * i;
      if (KC) {
        const int rr = idx / (BK / 4), k4 = (idx % (BK / 4)) * 4;
        *reinterpret_cast<float4*>(s + rr * LD + k4) = r[i];
      } else {
        const int kk = idx / (R / 4), m4 = (idx % (R / 4)) * 4;
        *reinterpret_cast<float4*>(s + kk * LD + m4) = r[i];
      }
    }
  }
};

// fragment for rows [row] and k = 16h + 4q .. +3 (four consecutive MFMA steps)
template <bool KC, int LD>
__device__ __forceinline__ float4 frag4(const float* s, int row, int h, int q) {
  if (KC) {
    return *reinterpret_cast<const float4*>(s + row * LD + h * 16 + q * 4);
  } else {
    const int k = h * 16 + q * 4;
    return make_float4(s[(k + 0) * LD + row], s[(k + 1) * LD + row], s[(k + 2) * LD + row], s[(k + 3) * LD + row]);
  }
}

// MF = 32: v_mfma_f32_32x32x2_f32 (lane l: row l&31, k half l>>5);
// MF = 16: v_mfma_f32_16x16x4_f32 (lane l: row l&15, k quarter l>>4; k = 8*(l>>4) + step, so a
// lane's 8 steps of a 32-deep tile are two float4 LDS reads).  Same tiles, loads and epilogue.
// 16x16x4 fragment: rows [row], k = k0 .. k0 + 3
template <bool KC, int LD>
__device__ __forceinline__ float4 frag16(const float* s, int row, int k0) {
  if (KC) return *reinterpret_cast<const float4*>(s + row * LD + k0);
  return make_float4(s[(k0 + 0) * LD + row], s[(k0 + 1) * LD + row], s[(k0 + 2) * LD + row], s[(k0 + 3) * LD + row]);
}

// epilogue: acc element e of lane -> row (e&3) + 8(e>>2) + 4h, col l32 (MF = 32) / row 4h + e (MF = 16)
template <int BM, int BN, int WGM, int WGN, int MF, typename AccT>
__device__ __forceinline__ void gemm_epilogue(const AccT (&acc)[BM / WGM / MF][BN / WGN / MF], int64_t M, int64_t N,
                                              float* __restrict__ C, int64_t ldc, const Epi& epi, int64_t m0,
                                              int64_t n0, float* __restrict__ ws) {
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / MF, TN = WTN / MF;
  constexpr int NE = MF == 32 ? 16 : 4;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int wm = w / WGN, wn = w % WGN;
  const int h = MF == 32 ? lane >> 5 : lane >> 4;
  const int l32 = MF == 32 ? lane & 31 : lane & 15;
  if (ws) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int64_t n = n0 + wn * WTN + j * MF + l32;
        if (n >= N) continue;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const int64_t m = m0 + wm * WTM + i * MF + (MF == 32 ? (e & 3) + 8 * (e >> 2) + 4 * h : 4 * h + e);
          if (m < M) ws[((int64_t)blockIdx.z * M + m) * N + n] = acc[i][j][e];
        }
      }
    return;
  }
  const bool rx = epi_reads_x(epi);
  if (!rx && !epi.bias_row && !epi.rv1 && !epi.rv2) {
    // no per-element inputs: one bias value per column at most
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int64_t n = n0 + wn * WTN + j * MF + l32;
        if (n >= N) continue;
        const float b = epi.bias ? epi.bias[n] : 0.f;
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const int64_t m = m0 + wm * WTM + i * MF + (MF == 32 ? (e & 3) + 8 * (e >> 2) + 4 * h : 4 * h + e);
          if (m < M) C[m * ldc + n] = epi_fin(epi, acc[i][j][e], b, 0.f, 0.f, 0.f);
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t n = n0 + wn * WTN + j * MF + l32;
      if (n >= N) continue;
      float bv[NE], xv[NE];
#pragma unroll
      for (int e = 0; e < NE; ++e) {  // all loads of the 16 elements first (no store in between)
        const int64_t m = m0 + wm * WTM + i * MF + (MF == 32 ? (e & 3) + 8 * (e >> 2) + 4 * h : 4 * h + e);
        const bool ok = m < M;
        bv[e] = (epi.bias && ok) ? epi.bias[(epi.bias_row ? (int64_t)epi.bias_row[m] : 0) * epi.ld_bias + n] : 0.f;
        xv[e] = (rx && ok) ? *epi_x_ptr(epi, C, ldc, m, n) : 0.f;
      }
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const int64_t m = m0 + wm * WTM + i * MF + (MF == 32 ? (e & 3) + 8 * (e >> 2) + 4 * h : 4 * h + e);
        if (m < M) C[m * ldc + n] = epi_fin(epi, acc[i][j][e], bv[e], xv[e], epi_r1(epi, m), epi_r2(epi, m));
      }
    }
}

// (tile row, tile column) of linear tile `tile`; tn_packed = tiles_n | group << 20 (tile_group())
__device__ __forceinline__ void tile_mn(int tile, int tn_packed, int tiles_m, int& tmi, int& tni) {
  const int tiles_n = tn_packed & 0xFFFFF, G = tn_packed >> 20;
  if (G <= 1) {
    tmi = tile / tiles_n;
    tni = tile - tmi * tiles_n;
    return;
  }
  const int per = G * tiles_n, g = tile / per, first = g * G;
  const int gs = min(tiles_m - first, G), rem = tile - g * per;
  tni = rem / gs;
  tmi = first + rem - tni * gs;
}


struct EpiCtx {
  const float* xb;
  int64_t ldx;
  bool rx, pure, v_in, v_out;
};
__device__ __forceinline__ EpiCtx epi_ctx(const Epi& epi, const float* C, int64_t ldc) {
  EpiCtx c;
  c.rx = epi_reads_x(epi);
  c.pure = !c.rx && !epi.bias_row && !epi.rv1 && !epi.rv2;
  c.xb = (epi.kind == GMR_EPI_NONE || epi.kind == GMR_EPI_BIAS) ? C : epi.aux;
  c.ldx = (epi.kind == GMR_EPI_NONE || epi.kind == GMR_EPI_BIAS) ? ldc : epi.ld_aux;
  c.v_out = ldc % 4 == 0 && ((uintptr_t)C & 15) == 0;
  c.v_in = (!epi.bias || (((uintptr_t)epi.bias & 15) == 0 && (!epi.bias_row || epi.ld_bias % 4 == 0))) &&
           (!c.rx || (((uintptr_t)c.xb & 15) == 0 && c.ldx % 4 == 0));
  return c;
}
__device__ __forceinline__ void epi_store4(const Epi& epi, float* __restrict__ C, int64_t ldc, int64_t N, int64_t m,
                                           int64_t n, const float (&a4)[4], const EpiCtx& ctx) {
  const bool full = n + 3 < N;
  float b4[4] = {0.f, 0.f, 0.f, 0.f}, x4[4] = {0.f, 0.f, 0.f, 0.f};
  const float* bp = epi.bias ? epi.bias + (epi.bias_row ? (int64_t)epi.bias_row[m] * epi.ld_bias : 0) + n : nullptr;
  const float* xp = ctx.rx ? ctx.xb + m * ctx.ldx + n : nullptr;
  if (full && ctx.v_in) {
    if (bp) {
      const float4 t = *reinterpret_cast<const float4*>(bp);
      b4[0] = t.x, b4[1] = t.y, b4[2] = t.z, b4[3] = t.w;
    }
    if (xp) {
      const float4 t = *reinterpret_cast<const float4*>(xp);
      x4[0] = t.x, x4[1] = t.y, x4[2] = t.z, x4[3] = t.w;
    }
  } else {
    for (int q = 0; q < 4 && n + q < N; ++q) {
      if (bp) b4[q] = bp[q];
      if (xp) x4[q] = xp[q];
    }
  }
  const float r1 = ctx.pure ? 0.f : epi_r1(epi, m), r2 = ctx.pure ? 0.f : epi_r2(epi, m);
  float o4[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) o4[q] = epi_fin(epi, a4[q], b4[q], x4[q], r1, r2);
  float* o = C + m * ldc + n;
  if (full && ctx.v_out) {
    *reinterpret_cast<float4*>(o) = make_float4(o4[0], o4[1], o4[2], o4[3]);
  } else {
    for (int q = 0; q < 4 && n + q < N; ++q) o[q] = o4[q];
  }
}

// Epilogue through LDS (glds and split-bf16 kernels): after the k loop the staging buffers are free, so the tile
// goes to LDS in row blocks of HR rows (fragment element stores: 32 consecutive columns per half
// wave, conflict-free) and comes back as float4 row chunks: the bias / aux / C traffic and the
// output stores are 16-byte, coalesced, and no per-element arrays are held in registers (the
// register epilogue of a 1,024-thread 256^2 tile spills).  Same per-element arithmetic (epi_fin).
// AVAIL: floats of LDS the caller's buffers give (default: the glds kernel's two staging buffers)
template <int BM, int BN, int WGM, int WGN, int AVAIL = 2 * (BM + BN) * BK>
__device__ __forceinline__ void gemm_epilogue_lds(const floatx16 (&acc)[BM / WGM / 32][BN / WGN / 32], float* smem,
                                                  int64_t M, int64_t N, float* __restrict__ C, int64_t ldc,
                                                  const Epi& epi, int64_t m0, int64_t n0, float* __restrict__ ws) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int HR0 = (AVAIL / BN) / 32 * 32;
  constexpr int HR = HR0 < BM ? HR0 : BM;                   // rows per pass
  constexpr int C4 = BN / 4;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int wm = w / WGN, wn = w % WGN;
  const int h = lane >> 5, l32 = lane & 31;
  const EpiCtx ctx = epi_ctx(epi, C, ldc);
  const bool v_out = ws ? (N % 4 == 0 && ((uintptr_t)ws & 15) == 0) : ctx.v_out;
#pragma unroll
  for (int r0 = 0; r0 < BM; r0 += HR) {
    __syncthreads();  // the buffers (first pass: the k loop's last reads; later: the previous pass) are free
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
      const bool full = n + 3 < N;
      if (ws) {
        float* o = ws + ((int64_t)blockIdx.z * M + m) * N + n;
        if (full && v_out) {
          *reinterpret_cast<float4*>(o) = v;
        } else {
          for (int q = 0; q < 4 && n + q < N; ++q) o[q] = a4[q];
        }
        continue;
      }
      epi_store4(epi, C, ldc, N, m, n, a4, ctx);
    }
  }
}

// split-bf16 products (gemm_x6.hip) with 16-byte aligned operands (lda / ldb multiples of 4) on a BM x BN tile
// (64^2, 128 x 128, 256 x 128 or 128 x 256); same grid, workspace and epilogue conventions as gemm.hip.
// akc / bkc: A / B k-contiguous (A [M][K], B [N][K]) or m- / n-contiguous (A stored K x M, B stored K x N),
// the latter read in place by the 128^2 / 256 x 128 / 128 x 256 tiles (NN: bkc = 0; TN: both 0); -1 = no kernel
int x6_ring();  // gemm_x6.hip: the register-ring 64^2 split-bf16 kernel is on (GMR_X6_RING, default 1)
int x6_inplace();  // gemm_x6.hip: TN / NN operands read in place, no transposed copies (GMR_X6_INPLACE, default 0: opt-in, measured slower)
int x6_launch(int bm, int bn, dim3 grid, hipStream_t st, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
              const float* B, int64_t ldb, float* C, int64_t ldc, const Epi& epi, int tiles_n, int64_t kps, float* ws,
              bool akc = true, bool bkc = true);

// dst[c * ld_dst + r] = src[r * ld_src + c] for r < rows, c < cols (the k-contiguous copy of an m- or
// n-contiguous operand for the split-bf16 kernel)
void x6_transpose(const float* src, int64_t ld_src, int64_t rows, int64_t cols, float* dst, int64_t ld_dst,
                  hipStream_t st);

}  // namespace gmr_gemm
