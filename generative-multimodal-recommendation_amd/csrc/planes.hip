// bf16 plane sets: an fp32 matrix held as three bf16 matrices x = hi + mid + lo EXACTLY (round-to-nearest
// splits: 3 x 8 significand bits hold fp32's 24, the split of gemm_x6.hip).  The split-bf16 form of the
// fused eval (gmr_score_topk_x6, GMR_EVAL_X6=1) reads its item table as such a plane set; the planes are
// written once per eval pass by gmr_split3_planes.
//
// Layout (caller-owned, bf16 as uint16): [3][rows][ld] with plane stride ps, columns contiguous, ld a
// multiple of 32 and the columns [cols, ld) ZERO.
#include "gmr_common.h"

namespace {

typedef __bf16 pl_bf4 __attribute__((ext_vector_type(4)));

// x = hi + mid + lo exactly (clamped into bf16 range first: gemm_x6.hip split3)
__device__ __forceinline__ void pl_split(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)__builtin_amdgcn_fmed3f(x, -0x1.fep127f, 0x1.fep127f);
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

// fp32 [rows][cols] (ld_src) -> three bf16 planes [rows][ld_dst] (plane stride ps), columns [cols, ld_dst)
// zeroed; one thread per 4 columns (the edge chunk is masked), one 8-byte store per plane
__global__ void __launch_bounds__(256) split3_planes_kernel(int64_t rows, int64_t cols, const float* __restrict__ src,
                                                            int64_t ld_src, __bf16* __restrict__ dst, int64_t ld_dst,
                                                            int64_t ps) {
  const int64_t c4n = ld_dst / 4;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < rows * c4n;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = g / c4n, c = (g % c4n) * 4;
    pl_bf4 h, m, l;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __bf16 a, b, e;
      pl_split(c + q < cols ? src[r * ld_src + c + q] : 0.f, a, b, e);
      h[q] = a;
      m[q] = b;
      l[q] = e;
    }
    __bf16* p = dst + r * ld_dst + c;
    *reinterpret_cast<pl_bf4*>(p) = h;
    *reinterpret_cast<pl_bf4*>(p + ps) = m;
    *reinterpret_cast<pl_bf4*>(p + 2 * ps) = l;
  }
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
