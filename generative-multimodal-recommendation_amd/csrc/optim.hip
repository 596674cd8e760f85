// Fused Adam over flat fp32 parameter slabs (replaces torch.optim.Adam on the hot path:
// common/trainer.py:125-142, 413-415).  Same update as torch's single-tensor Adam:
//   g += wd * p ; m = m + (1 - b1) (g - m) ; v = b2 v + (1 - b2) g^2
//   p -= step_size * m / (sqrt(v) / bc2_sqrt + eps),  step_size = lr / (1 - b1^t)
// Bias corrections are computed by the caller in fp64 and passed as fp32 scalars,
// exactly as torch passes Python scalars into its fp32 kernels.
#include "gmr_common.h"

namespace {

__global__ void adam_kernel(int64_t n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, float b1, float b2, float eps, float wd, float step_size,
                            float bc2_sqrt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float gi = g[i];
  const float pi = p[i];
  if (wd != 0.f) gi = gi + wd * pi;
  const float mi = m[i] + (1.f - b1) * (gi - m[i]);
  const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] = pi - step_size * (mi / denom);
}

}  // namespace

extern "C" int gmr_adam_f32(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, float beta1,
                            float beta2, float eps, float weight_decay, float step_size, float bias_correction2_sqrt,
                            void* stream) {
  GMR_ARG(param && grad && exp_avg && exp_avg_sq && n >= 0, "bad args");
  if (n == 0) return GMR_OK;
  hipLaunchKernelGGL(adam_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, param, grad, exp_avg,
                     exp_avg_sq, beta1, beta2, eps, weight_decay, step_size, bias_correction2_sqrt);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_zero(void* ptr, int64_t bytes, void* stream) {
  GMR_ARG(ptr || bytes == 0, "null pointer");
  if (bytes == 0) return GMR_OK;
  hipError_t e = hipMemsetAsync(ptr, 0, (size_t)bytes, (hipStream_t)stream);
  if (e != hipSuccess) return gmr::hip_status(__func__, e);
  return GMR_OK;
}
