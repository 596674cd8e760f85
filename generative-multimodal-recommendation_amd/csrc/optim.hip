// Fused Adam over flat fp32 parameter slabs (replaces torch.optim.Adam on the hot path:
// common/trainer.py:125-142, 413-415).  Same update as torch's single-tensor Adam:
//   g += wd * p ; m = m + (1 - b1) (g - m) ; v = b2 v + (1 - b2) g^2
//   p -= step_size * m / (sqrt(v) / bc2_sqrt + eps),  step_size = lr / (1 - b1^t)
// Bias corrections are computed by the caller in fp64 and passed as fp32 scalars,
// exactly as torch passes Python scalars into its fp32 kernels.
#include "gmr_common.h"

namespace {

// one element's update (torch.optim.Adam's arithmetic, every product and sum rounded on its own): FMA
// contraction is off here because the float4 kernel's packed instructions (v_pk_fma_f32) would otherwise
// contract differently from the scalar kernel's, and the two paths must agree bit for bit
__device__ __forceinline__ float adam_one(float gi, float pi, float& mi, float& vi, float b1, float b2, float eps,
                                          float wd, float step_size, float bc2_sqrt) {
#pragma clang fp contract(off)
  if (wd != 0.f) gi = gi + wd * pi;
  mi = mi + (1.f - b1) * (gi - mi);
  vi = vi * b2 + (1.f - b2) * gi * gi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  return pi - step_size * (mi / denom);
}
__global__ void adam_kernel(int64_t n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, float b1, float b2, float eps, float wd, float step_size,
                            float bc2_sqrt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float mi = m[i], vi = v[i];
  const float po = adam_one(g[i], p[i], mi, vi, b1, b2, eps, wd, step_size, bc2_sqrt);
  m[i] = mi;
  v[i] = vi;
  p[i] = po;
}

// the same update, four elements per thread (16-byte aligned slabs; each lane's arithmetic is the scalar
// kernel's, so the results are bit-identical): one 16-byte load / store per operand instead of four
__global__ void adam4_kernel(int64_t n4, float4* __restrict__ p, const float4* __restrict__ g, float4* __restrict__ m,
                             float4* __restrict__ v, float b1, float b2, float eps, float wd, float step_size,
                             float bc2_sqrt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const float4 gi = g[i], pi = p[i];
  float4 mi = m[i], vi = v[i], po;
  po.x = adam_one(gi.x, pi.x, mi.x, vi.x, b1, b2, eps, wd, step_size, bc2_sqrt);
  po.y = adam_one(gi.y, pi.y, mi.y, vi.y, b1, b2, eps, wd, step_size, bc2_sqrt);
  po.z = adam_one(gi.z, pi.z, mi.z, vi.z, b1, b2, eps, wd, step_size, bc2_sqrt);
  po.w = adam_one(gi.w, pi.w, mi.w, vi.w, b1, b2, eps, wd, step_size, bc2_sqrt);
  m[i] = mi;
  v[i] = vi;
  p[i] = po;
}

}  // namespace

extern "C" int gmr_adam_f32(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, float beta1,
                            float beta2, float eps, float weight_decay, float step_size, float bias_correction2_sqrt,
                            void* stream) {
  GMR_ARG(param && grad && exp_avg && exp_avg_sq && n >= 0, "bad args");
  if (n == 0) return GMR_OK;
  hipStream_t st = (hipStream_t)stream;
  const bool al = (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15) == 0;
  const int64_t n4 = al ? n / 4 : 0;
  if (n4 > 0) {
    hipLaunchKernelGGL(adam4_kernel, dim3(gmr::grid_for(n4, 256)), dim3(256), 0, st, n4,
                       reinterpret_cast<float4*>(param), reinterpret_cast<const float4*>(grad),
                       reinterpret_cast<float4*>(exp_avg), reinterpret_cast<float4*>(exp_avg_sq), beta1, beta2, eps,
                       weight_decay, step_size, bias_correction2_sqrt);
    GMR_LAUNCHED();
  }
  const int64_t t0 = 4 * n4;  // scalar tail (or the whole range when a pointer is not 16-byte aligned)
  if (t0 < n) {
    hipLaunchKernelGGL(adam_kernel, dim3(gmr::grid_for(n - t0, 256)), dim3(256), 0, st, n - t0, param + t0, grad + t0,
                       exp_avg + t0, exp_avg_sq + t0, beta1, beta2, eps, weight_decay, step_size, bias_correction2_sqrt);
    GMR_LAUNCHED();
  }
  return GMR_OK;
}

extern "C" int gmr_zero(void* ptr, int64_t bytes, void* stream) {
  GMR_ARG(ptr || bytes == 0, "null pointer");
  if (bytes == 0) return GMR_OK;
  hipError_t e = hipMemsetAsync(ptr, 0, (size_t)bytes, (hipStream_t)stream);
  if (e != hipSuccess) return gmr::hip_status(__func__, e);
  return GMR_OK;
}

// Stream-timing probe for the ordering tests (gmr.kernels.Streams.PERTURB): one wave that sleeps about `us`
// microseconds (s_sleep 127 = 8,128 clocks, ~3.4 us at 2.4 GHz) and touches no memory, so whatever is queued
// behind it on `stream` starts that much later while the other streams run on.
__global__ void delay_kernel(int iters) {
  for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
}

extern "C" int gmr_delay(int32_t us, void* stream) {
  GMR_ARG(us >= 0 && us <= 1000000, "us must be in [0, 1e6]");
  if (us == 0) return GMR_OK;
  hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (us + 2) / 3);
  GMR_LAUNCHED();
  return GMR_OK;
}
