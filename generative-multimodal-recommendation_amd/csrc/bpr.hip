// K7 — BPR + EmbLoss for the VBPR model (models/vbpr.py:76-97; common/loss.py BPRLoss, EmbLoss).
//
// loss = mean_b -log(1e-10 + sigmoid(<u_b, p_b> - <u_b, n_b>))
//        + reg_weight * (||U||_F + ||P||_F + ||N||_F) / B      (U, P, N: the gathered B x D rows)
// Three launches, all deterministic: per-row scores and squared norms (one wave per row), a
// single-workgroup fp64 reduction in fixed order (loss + the three norm coefficients), and the
// per-row gradient contributions [dU; dP; dN] (3B x D) that the sorted scatter adds to the
// user / item tables.  The rows live in one (U + I) x D table: users first, then items.
#include "gmr_common.h"

namespace {

__global__ void __launch_bounds__(256) vbpr_rows_kernel(int B, int D, const float* __restrict__ T, int64_t ldt,
                                                        const int* __restrict__ users, const int* __restrict__ pos,
                                                        const int* __restrict__ neg, int64_t item_off,
                                                        float* __restrict__ x, double* __restrict__ sq) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const float* u = T + (int64_t)users[b] * ldt;
  const float* p = T + (item_off + pos[b]) * ldt;
  const float* n = T + (item_off + neg[b]) * ldt;
  float dp = 0.f, dn = 0.f, su = 0.f, sp = 0.f, sn = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float uu = u[c], pp = p[c], nn = n[c];
    dp = fmaf(uu, pp, dp);
    dn = fmaf(uu, nn, dn);
    su = fmaf(uu, uu, su);
    sp = fmaf(pp, pp, sp);
    sn = fmaf(nn, nn, sn);
  }
  dp = gmr::wave_sum(dp);
  dn = gmr::wave_sum(dn);
  su = gmr::wave_sum(su);
  sp = gmr::wave_sum(sp);
  sn = gmr::wave_sum(sn);
  if (lane == 0) {
    x[b] = dp - dn;
    sq[b] = su;
    sq[B + b] = sp;
    sq[2 * B + b] = sn;
  }
}

// coef[0..2] = reg_weight / (B ||.||) for U, P, N;  loss[0] = total (fp32)
__global__ void __launch_bounds__(1024) vbpr_reduce_kernel(int B, const float* __restrict__ x,
                                                           const double* __restrict__ sq, float reg_weight,
                                                           float* __restrict__ loss, float* __restrict__ coef) {
  __shared__ double s[4][1024];
  const int t = threadIdx.x;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  for (int b = t; b < B; b += 1024) {
    const double sg = 1.0 / (1.0 + exp(-(double)x[b]));
    a[0] += -log(1e-10 + sg);
    a[1] += sq[b];
    a[2] += sq[B + b];
    a[3] += sq[2 * B + b];
  }
  for (int k = 0; k < 4; ++k) s[k][t] = a[k];
  __syncthreads();
  for (int off = 512; off > 0; off >>= 1) {
    if (t < off)
      for (int k = 0; k < 4; ++k) s[k][t] += s[k][t + off];
    __syncthreads();
  }
  if (t == 0) {
    const double nu = sqrt(s[1][0]), np = sqrt(s[2][0]), nn = sqrt(s[3][0]);
    loss[0] = (float)(s[0][0] / B + (double)reg_weight * (nu + np + nn) / B);
    coef[0] = nu > 0.0 ? (float)(reg_weight / (B * nu)) : 0.f;
    coef[1] = np > 0.0 ? (float)(reg_weight / (B * np)) : 0.f;
    coef[2] = nn > 0.0 ? (float)(reg_weight / (B * nn)) : 0.f;
  }
}

// contrib rows: [0, B) users, [B, 2B) positives, [2B, 3B) negatives
__global__ void __launch_bounds__(256) vbpr_contrib_kernel(int B, int D, const float* __restrict__ T, int64_t ldt,
                                                           const int* __restrict__ users,
                                                           const int* __restrict__ pos, const int* __restrict__ neg,
                                                           int64_t item_off, const float* __restrict__ x,
                                                           const float* __restrict__ coef,
                                                           float* __restrict__ contrib, int64_t ldc) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const float sg = 1.f / (1.f + expf(-x[b]));
  const float g = -(sg * (1.f - sg)) / (1e-10f + sg) / (float)B;  // d/dx of mean -log(1e-10 + sigmoid)
  const float cu = coef[0], cp = coef[1], cn = coef[2];
  const float* u = T + (int64_t)users[b] * ldt;
  const float* p = T + (item_off + pos[b]) * ldt;
  const float* n = T + (item_off + neg[b]) * ldt;
  float* du = contrib + (int64_t)b * ldc;
  float* dp = contrib + (int64_t)(B + b) * ldc;
  float* dn = contrib + (int64_t)(2 * B + b) * ldc;
  for (int c = lane; c < D; c += 64) {
    const float uu = u[c], pp = p[c], nn = n[c];
    du[c] = fmaf(g, pp - nn, cu * uu);
    dp[c] = fmaf(g, uu, cp * pp);
    dn[c] = fmaf(-g, uu, cn * nn);
  }
}

__global__ void fill2d_kernel(int64_t rows, int64_t cols, float* __restrict__ p, int64_t ld, float v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols) return;
  p[(i / cols) * ld + i % cols] = v;
}

}  // namespace

extern "C" int gmr_vbpr_loss_fwd_bwd(int32_t B, int32_t D, const float* table, int64_t ldt, const int32_t* users,
                                     const int32_t* pos, const int32_t* neg, int64_t item_off, float reg_weight,
                                     float* x_ws, double* sq_ws, float* coef_ws, float* loss, float* contrib,
                                     int64_t ldc, void* stream) {
  GMR_ARG(table && users && pos && neg && x_ws && sq_ws && coef_ws && loss && contrib && B > 0 && D > 0, "bad args");
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)((B + 3) / 4));
  hipLaunchKernelGGL(vbpr_rows_kernel, g, dim3(256), 0, st, B, D, table, ldt, users, pos, neg, item_off, x_ws, sq_ws);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(vbpr_reduce_kernel, dim3(1), dim3(1024), 0, st, B, x_ws, sq_ws, reg_weight, loss, coef_ws);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(vbpr_contrib_kernel, g, dim3(256), 0, st, B, D, table, ldt, users, pos, neg, item_off, x_ws,
                     coef_ws, contrib, ldc);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_fill2d_f32(int64_t rows, int64_t cols, float* p, int64_t ld, float value, void* stream) {
  GMR_ARG(p && rows >= 0 && cols >= 0 && ld >= cols, "bad args");
  if (rows == 0 || cols == 0) return GMR_OK;
  hipLaunchKernelGGL(fill2d_kernel, dim3(gmr::grid_for(rows * cols, 256)), dim3(256), 0, (hipStream_t)stream, rows,
                     cols, p, ld, value);
  GMR_LAUNCHED();
  return GMR_OK;
}
