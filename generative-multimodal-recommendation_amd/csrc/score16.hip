// Opt-in fp16 MFMA full-catalog scoring (BASELINE config 5: "fp16 MFMA scoring GEMM").
//
// Replaces the fp32 product of GenRecV1.full_sort_predict (reference models/genrecv1.py:419-427,
// scores = u_emb[user] @ i_emb^T) when `scoring_dtype: fp16` is configured:
//   C (E x I, fp32) = fp16(A) (E x 64) . fp16(B)^T (64 x I), fp32 accumulation.
// The fp32 embeddings are rounded to fp16 as they are loaded (no conversion pass), so the
// only HBM traffic is A and B once per tile plus the fp32 score write, which dominates
// (E*I*4 bytes): the kernel is write-bound, the MFMA work (2*E*I*64 flop) is small.
// Tile: a 256-thread workgroup writes a 64 x 64 score tile; each wave owns a 32 x 32 block and
// runs 4 v_mfma_f32_32x32x16_f16 over K = 64.  A lane holds row (lane & 31) of A and column
// (lane & 31) of B, k = 16 s + 8 (lane >> 5) + 0..7 for step s.  Output element j of a lane is
// row 8 (j >> 2) + 4 (lane >> 5) + (j & 3), column lane & 31.
// The default fp32 path (gmr_gemm_f32) stays the one that gives bit-exact top-K indices.
#include "gmr_common.h"

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16x __attribute__((ext_vector_type(16)));

__device__ __forceinline__ h8 load_h8(const float* __restrict__ p, bool ok) {
  h8 r;
  if (ok) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    r[0] = (_Float16)a.x; r[1] = (_Float16)a.y; r[2] = (_Float16)a.z; r[3] = (_Float16)a.w;
    r[4] = (_Float16)b.x; r[5] = (_Float16)b.y; r[6] = (_Float16)b.z; r[7] = (_Float16)b.w;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = (_Float16)0.f;
  }
  return r;
}

__global__ void __launch_bounds__(256) score16_kernel(int64_t E, int64_t I, const float* __restrict__ A,
                                                      int64_t lda, const float* __restrict__ B, int64_t ldb,
                                                      float* __restrict__ C, int64_t ldc, int64_t tiles_n) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int64_t tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int64_t r0 = tm * 64 + (wid >> 1) * 32, c0 = tn * 64 + (wid & 1) * 32;
  const int64_t ra = r0 + l32, cb = c0 + l32;
  f16x acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 16 * s + 8 * h;
    const h8 a = load_h8(A + ra * lda + k, ra < E);
    const h8 b = load_h8(B + cb * ldb + k, cb < I);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  }
  if (cb < I) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t r = r0 + 8 * (j >> 2) + 4 * h + (j & 3);
      if (r < E) C[r * ldc + cb] = acc[j];
    }
  }
}

}  // namespace

extern "C" int gmr_score_f16(int64_t E, int64_t I, int64_t d, const float* A, int64_t lda, const float* B,
                             int64_t ldb, float* C, int64_t ldc, void* stream) {
  GMR_ARG(A && B && C, "null pointer");
  GMR_ARG(d == 64, "fp16 scoring takes 64-wide embeddings");
  GMR_ARG(E > 0 && I > 0 && lda >= 64 && ldb >= 64 && ldc >= I, "bad shape");
  GMR_ARG(lda % 4 == 0 && ldb % 4 == 0 && (((uintptr_t)A | (uintptr_t)B) & 15) == 0,
          "A and B rows must be 16-byte aligned");
  const int64_t tiles_m = (E + 63) / 64, tiles_n = (I + 63) / 64;
  GMR_ARG(tiles_m * tiles_n < (1ll << 31), "too many tiles");
  hipLaunchKernelGGL(score16_kernel, dim3((unsigned)(tiles_m * tiles_n)), dim3(256), 0, (hipStream_t)stream, E, I, A,
                     lda, B, ldb, C, ldc, tiles_n);
  GMR_LAUNCHED();
  return GMR_OK;
}
