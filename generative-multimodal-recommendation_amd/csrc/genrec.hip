// GenRecV1 recommendation step (models/genrecv1.py:225-427): fused column/row kernels.
//
// Every activation table of the step is N x 64 or I x 64 fp32, row-major (ld given); a row is
// covered by 16 lanes x float4.  BatchNorm1d runs in three deterministic passes (per-block fp64
// column partials, a fixed-order 64-thread finalise that also updates the running statistics
// exactly like nn.BatchNorm1d, an apply pass fused with the activation, the Dropout keep mask
// and the consumer's elementwise op).  The backward recomputes x_hat from the saved input.
#include "gmr_common.h"

namespace {

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float4 f4(float a, float b, float c, float d) { return make_float4(a, b, c, d); }
__device__ __forceinline__ float g4(float4 v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
__device__ __forceinline__ void s4(float4& v, int k, float x) {
  if (k == 0) v.x = x; else if (k == 1) v.y = x; else if (k == 2) v.z = x; else v.w = x;
}
__device__ __forceinline__ float row16_sum(float v) {
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// activation codes: 0 identity, 1 leaky-ReLU(slope), 2 sigmoid, 3 tanh
__device__ __forceinline__ float act_f(int act, float v, float slope) {
  switch (act) {
    case 1: return v > 0.f ? v : v * slope;
    case 2: return 1.f / (1.f + expf(-v));
    case 3: return tanhf(v);
    default: return v;
  }
}
__device__ __forceinline__ float act_d(int act, float v, float a, float slope) {
  switch (act) {
    case 1: return v > 0.f ? 1.f : slope;
    case 2: return a * (1.f - a);
    case 3: return 1.f - a * a;
    default: return 1.f;
  }
}

constexpr int kRows = 16;   // row slots per 256-thread block
constexpr int kMaxParts = 256;

__host__ __device__ inline int parts_for(int64_t rows) {
  int64_t p = (rows + kRows - 1) / kRows;
  return (int)(p < kMaxParts ? p : kMaxParts);
}

// ----------------------------------------------------------------- BatchNorm1d (64 columns)
__global__ void __launch_bounds__(256) bn_stats_kernel(int64_t rows, const float* __restrict__ z, int64_t ldz,
                                                       double* __restrict__ part) {
  __shared__ double red[kRows][128];
  const int slot = threadIdx.x >> 4, l = threadIdx.x & 15, c = l * 4;
  double s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
  for (int64_t r = (int64_t)blockIdx.x * kRows + slot; r < rows; r += (int64_t)gridDim.x * kRows) {
    const float4 v = ld4(z + r * ldz + c);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double x = g4(v, k);
      s[k] += x;
      q[k] += x * x;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[slot][c + k] = s[k];
    red[slot][64 + c + k] = q[k];
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    double a = 0.0;
    for (int j = 0; j < kRows; ++j) a += red[j][threadIdx.x];
    part[(int64_t)blockIdx.x * 128 + threadIdx.x] = a;
  }
}

// 1024 threads: column c = t & 63 summed by 16 groups (parts g, g+16, ...) then the 16 group sums in
// order — a fixed reduction order with a 16-long dependent chain instead of P
__global__ void __launch_bounds__(1024) bn_finalize_kernel(int P, const double* __restrict__ part, int64_t rows,
                                                           float eps, float momentum, int train,
                                                           float* __restrict__ run_mean, float* __restrict__ run_var,
                                                           float* __restrict__ mean_out, float* __restrict__ invstd_out) {
  __shared__ double rs[16][64], rq[16][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  if (!train) {
    if (g == 0) {
      mean_out[c] = run_mean[c];
      invstd_out[c] = 1.f / sqrtf(run_var[c] + eps);
    }
    return;
  }
  double s = 0.0, q = 0.0;
  for (int p = g; p < P; p += 16) {
    s += part[(int64_t)p * 128 + c];
    q += part[(int64_t)p * 128 + 64 + c];
  }
  rs[g][c] = s;
  rq[g][c] = q;
  __syncthreads();
  if (g != 0) return;
  s = q = 0.0;
  for (int j = 0; j < 16; ++j) {
    s += rs[j][c];
    q += rq[j][c];
  }
  const double n = (double)rows;
  const double mean = s / n;
  double var = q / n - mean * mean;
  if (var < 0.0) var = 0.0;
  mean_out[c] = (float)mean;
  invstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) {
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)(rows > 1 ? var * n / (n - 1.0) : var);
  }
}

// y = act(w (z - mean) invstd + b) [* keep * mscale]; post: 0 none, 1 out2 = rs * aux + y,
// 2 out2 = aux * y, 3 rowdot[r] = <y_r, aux[0:64]>
__global__ void __launch_bounds__(256) bn_apply_kernel(int64_t rows, const float* __restrict__ z, int64_t ldz,
                                                       const float* __restrict__ mean, const float* __restrict__ invstd,
                                                       const float* __restrict__ w, const float* __restrict__ b, int act,
                                                       float slope, const uint8_t* __restrict__ mask, int64_t ldm,
                                                       float mscale, float* __restrict__ y, int64_t ldy, int post,
                                                       const float* __restrict__ aux, int64_t ldaux,
                                                       const float* __restrict__ rs, float* __restrict__ out2,
                                                       int64_t ld2, float* __restrict__ rowdot) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = gid >> 4;
  const bool ok = r < rows;
  const int c = (gid & 15) * 4;
  float4 a = f4(0, 0, 0, 0);
  if (ok) {
    const float4 zz = ld4(z + r * ldz + c), mu = ld4(mean + c), is = ld4(invstd + c), ww = ld4(w + c), bb = ld4(b + c);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = (g4(zz, k) - g4(mu, k)) * g4(is, k);
      float v = act_f(act, xh * g4(ww, k) + g4(bb, k), slope);
      if (mask) v = mask[r * ldm + c + k] ? v * mscale : 0.f;
      s4(a, k, v);
    }
    if (y) st4(y + r * ldy + c, a);
  }
  if (post == 3) {
    float d = ok ? (a.x * aux[c] + a.y * aux[c + 1] + a.z * aux[c + 2] + a.w * aux[c + 3]) : 0.f;
    d = row16_sum(d);
    if (ok && (gid & 15) == 0) rowdot[r] = d;
    return;
  }
  if (!ok || post == 0) return;
  const float4 x = ld4(aux + r * ldaux + c);
  float4 o;
  if (post == 1) {
    const float s = rs[0];
    o = f4(s * x.x + a.x, s * x.y + a.y, s * x.z + a.z, s * x.w + a.w);
  } else {
    o = f4(x.x * a.x, x.y * a.y, x.z * a.z, x.w * a.w);
  }
  st4(out2 + r * ld2 + c, o);
}

struct BnBwdIn {
  const float* z; int64_t ldz;
  const float* mean; const float* invstd; const float* w; const float* b;
  int act; float slope;
  const uint8_t* mask; int64_t ldm; float mscale;
  const float* dy; int64_t lddy;
  const float* mul; int64_t ldmul;
  const float* da; const float* v;
};

// upstream gradient of the BN output (pre-activation): dv, plus x_hat and the activation output
__device__ __forceinline__ void bn_bwd_elem(const BnBwdIn& p, int64_t r, int c, float4& dv, float4& xh, float4& av) {
  const float4 zz = ld4(p.z + r * p.ldz + c), mu = ld4(p.mean + c), is = ld4(p.invstd + c), ww = ld4(p.w + c),
               bb = ld4(p.b + c);
  float4 g;
  if (p.da) {
    const float d = p.da[r];
    g = f4(d * p.v[c], d * p.v[c + 1], d * p.v[c + 2], d * p.v[c + 3]);
  } else {
    g = ld4(p.dy + r * p.lddy + c);
    if (p.mul) {
      const float4 m = ld4(p.mul + r * p.ldmul + c);
      g = f4(g.x * m.x, g.y * m.y, g.z * m.z, g.w * m.w);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float x = (g4(zz, k) - g4(mu, k)) * g4(is, k);
    const float v = x * g4(ww, k) + g4(bb, k);
    const float a = act_f(p.act, v, p.slope);
    float gg = g4(g, k);
    if (p.mask) gg = p.mask[r * p.ldm + c + k] ? gg * p.mscale : 0.f;
    s4(dv, k, gg * act_d(p.act, v, a, p.slope));
    s4(xh, k, x);
    s4(av, k, a);
  }
}

// per-block fp64 column partials: [sum dv | sum dv*xhat | sum da*a] (3 x 64)
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(int64_t rows, BnBwdIn p, double* __restrict__ part) {
  __shared__ double red[kRows][192];
  const int slot = threadIdx.x >> 4, c = (threadIdx.x & 15) * 4;
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  for (int64_t r = (int64_t)blockIdx.x * kRows + slot; r < rows; r += (int64_t)gridDim.x * kRows) {
    float4 dv, xh, av;
    bn_bwd_elem(p, r, c, dv, xh, av);
    const float d = p.da ? p.da[r] : 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s0[k] += (double)g4(dv, k);
      s1[k] += (double)g4(dv, k) * (double)g4(xh, k);
      s2[k] += (double)d * (double)g4(av, k);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[slot][c + k] = s0[k];
    red[slot][64 + c + k] = s1[k];
    red[slot][128 + c + k] = s2[k];
  }
  __syncthreads();
  if (threadIdx.x < 192) {
    double a = 0.0;
    for (int j = 0; j < kRows; ++j) a += red[j][threadIdx.x];
    part[(int64_t)blockIdx.x * 192 + threadIdx.x] = a;
  }
}

// dw += sum dv*xhat; db += sum dv; dvec += sum da*a; sums = [mean dv | mean dv*xhat]
// (1024 threads, 16 part groups per column, fixed order)
__global__ void __launch_bounds__(1024) bn_bwd_finalize_kernel(int P, const double* __restrict__ part, int64_t rows,
                                                               float* __restrict__ dw, float* __restrict__ db,
                                                               float* __restrict__ dvec, float* __restrict__ sums,
                                                               int accumulate) {
  __shared__ double r0[16][64], r1[16][64], r2[16][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  for (int p = g; p < P; p += 16) {
    s0 += part[(int64_t)p * 192 + c];
    s1 += part[(int64_t)p * 192 + 64 + c];
    s2 += part[(int64_t)p * 192 + 128 + c];
  }
  r0[g][c] = s0;
  r1[g][c] = s1;
  r2[g][c] = s2;
  __syncthreads();
  if (g != 0) return;
  s0 = s1 = s2 = 0.0;
  for (int j = 0; j < 16; ++j) {
    s0 += r0[j][c];
    s1 += r1[j][c];
    s2 += r2[j][c];
  }
  if (dw) dw[c] = (float)s1 + (accumulate ? dw[c] : 0.f);
  if (db) db[c] = (float)s0 + (accumulate ? db[c] : 0.f);
  if (dvec) dvec[c] = (float)s2 + (accumulate ? dvec[c] : 0.f);
  sums[c] = (float)(s0 / (double)rows);
  sums[64 + c] = (float)(s1 / (double)rows);
}

// dz = w invstd (dv - mean(dv) - xhat mean(dv xhat))
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(int64_t rows, BnBwdIn p, const float* __restrict__ sums,
                                                           float* __restrict__ dz, int64_t lddz, int accumulate) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = gid >> 4;
  if (r >= rows) return;
  const int c = (gid & 15) * 4;
  float4 dv, xh, av;
  bn_bwd_elem(p, r, c, dv, xh, av);
  const float4 m0 = ld4(sums + c), m1 = ld4(sums + 64 + c), ww = ld4(p.w + c), is = ld4(p.invstd + c);
  float4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    s4(o, k, g4(ww, k) * g4(is, k) * (g4(dv, k) - g4(m0, k) - g4(xh, k) * g4(m1, k)));
  float* q = dz + r * lddz + c;
  if (accumulate) {
    const float4 old = ld4(q);
    o = f4(o.x + old.x, o.y + old.y, o.z + old.z, o.w + old.w);
  }
  st4(q, o);
}

// ----------------------------------------------------------------- content (user_item_GCN x 2 + weights)
__device__ __forceinline__ void softmax2v(const float* a, const float* b, float& w0, float& w1) {
  const float x = a[0], y = b[0];
  const float m = fmaxf(x, y);
  const float ex = expf(x - m), ey = expf(y - m);
  w0 = ex / (ex + ey);
  w1 = ey / (ex + ey);
}

// C = w0 (E + A1)/2 + w1 (E + A2)/2, w = softmax([origin_weight, generation_weight]) (genrecv1.py:332-336)
__global__ void content_fwd_kernel(int64_t n, const float* __restrict__ E, const float* __restrict__ A1,
                                   const float* __restrict__ A2, const float* __restrict__ ow,
                                   const float* __restrict__ gw, float* __restrict__ C) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * 16) return;
  const int64_t o = (gid >> 4) * 64 + (gid & 15) * 4;
  float w0, w1;
  softmax2v(ow, gw, w0, w1);
  const float4 e = ld4(E + o), a1 = ld4(A1 + o), a2 = ld4(A2 + o);
  float4 r;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    s4(r, k, w0 * ((g4(e, k) + g4(a1, k)) * 0.5f) + w1 * ((g4(e, k) + g4(a2, k)) * 0.5f));
  st4(C + o, r);
}

// partial sums of <dC, c1> and <dC, c2> (c_k = (E + A_k)/2) per block -> part[2 * block]
__global__ void __launch_bounds__(256) content_bwd_part_kernel(int64_t n, const float* __restrict__ E,
                                                               const float* __restrict__ A1,
                                                               const float* __restrict__ A2,
                                                               const float* __restrict__ dC, double* __restrict__ part) {
  __shared__ double red[2][4];
  double s1 = 0.0, s2 = 0.0;
  for (int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < n * 16;
       gid += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = (gid >> 4) * 64 + (gid & 15) * 4;
    const float4 e = ld4(E + o), a1 = ld4(A1 + o), a2 = ld4(A2 + o), d = ld4(dC + o);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s1 += (double)g4(d, k) * (double)((g4(e, k) + g4(a1, k)) * 0.5f);
      s2 += (double)g4(d, k) * (double)((g4(e, k) + g4(a2, k)) * 0.5f);
    }
  }
  s1 = gmr::wave_sum_d(s1);
  s2 = gmr::wave_sum_d(s2);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x < 2)
    part[(int64_t)blockIdx.x * 2 + threadIdx.x] =
        (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
}

// fixed-order block reduction of P doubles (stride st, offset o): thread t sums t, t+256, ...; tree in LDS
__device__ __forceinline__ double block_sum_parts(int P, const double* __restrict__ part, int st, int o,
                                                  double* red) {
  double s = 0.0;
  for (int p = threadIdx.x; p < P; p += 256) s += part[(int64_t)p * st + o];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// softmax backward onto the two weight parameters (accumulated into their grads)
__global__ void __launch_bounds__(256) content_bwd_weights_kernel(int P, const double* __restrict__ part,
                                                                  const float* __restrict__ ow,
                                                                  const float* __restrict__ gw,
                                                                  float* __restrict__ dow, float* __restrict__ dgw) {
  __shared__ double red[256];
  const double s1 = block_sum_parts(P, part, 2, 0, red);
  const double s2 = block_sum_parts(P, part, 2, 1, red);
  if (threadIdx.x != 0) return;
  float w0, w1;
  softmax2v(ow, gw, w0, w1);
  const double dot = w0 * s1 + w1 * s2;
  dow[0] += (float)(w0 * (s1 - dot));
  dgw[0] += (float)(w1 * (s2 - dot));
}

// dE += ((w0 + w1) dC + w0 T1 + w1 T2) / 2  (T1 = A1^T dC, T2 = A2^T dC) + reg2 * E
__global__ void content_bwd_combine_kernel(int64_t n, const float* __restrict__ dC, const float* __restrict__ T1,
                                           const float* __restrict__ T2, const float* __restrict__ ow,
                                           const float* __restrict__ gw, const float* __restrict__ E, float reg2,
                                           float* __restrict__ dE) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * 16) return;
  const int64_t o = (gid >> 4) * 64 + (gid & 15) * 4;
  float w0, w1;
  softmax2v(ow, gw, w0, w1);
  const float4 d = ld4(dC + o), t1 = ld4(T1 + o), t2 = ld4(T2 + o), e = ld4(E + o), old = ld4(dE + o);
  float4 r;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    s4(r, k, g4(old, k) + 0.5f * (w0 * (g4(d, k) + g4(t1, k)) + w1 * (g4(d, k) + g4(t2, k))) + reg2 * g4(e, k));
  st4(dE + o, r);
}

// ----------------------------------------------------------------- gate_attention_fusion (genrecv1.py:309-353)
// alpha = softmax(aI, aT)[0]; COM = alpha IMG + (1-alpha) TXT;
// SIDE = (PI (IMG - COM) + PT (TXT - COM) + COM) / 4
__global__ void fusion_fwd_kernel(int64_t n, const float* __restrict__ IMG, const float* __restrict__ TXT,
                                  const float* __restrict__ aI, const float* __restrict__ aT,
                                  const float* __restrict__ PI, const float* __restrict__ PT,
                                  float* __restrict__ SIDE, float* __restrict__ alpha) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * 16) return;
  const int64_t r = gid >> 4;
  const int64_t o = r * 64 + (gid & 15) * 4;
  float w0, w1;
  softmax2v(aI + r, aT + r, w0, w1);
  if ((gid & 15) == 0) alpha[r] = w0;
  const float4 im = ld4(IMG + o), tx = ld4(TXT + o), pi = ld4(PI + o), pt = ld4(PT + o);
  float4 s;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float com = w0 * g4(im, k) + w1 * g4(tx, k);
    s4(s, k, (g4(pi, k) * (g4(im, k) - com) + g4(pt, k) * (g4(tx, k) - com) + com) / 4.f);
  }
  st4(SIDE + o, s);
}

__global__ void fusion_bwd_kernel(int64_t n, const float* __restrict__ IMG, const float* __restrict__ TXT,
                                  const float* __restrict__ alpha, const float* __restrict__ PI,
                                  const float* __restrict__ PT, const float* __restrict__ dSIDE,
                                  float* __restrict__ dIMG, float* __restrict__ dTXT, float* __restrict__ daI,
                                  float* __restrict__ daT, float* __restrict__ dPI, float* __restrict__ dPT) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = gid >> 4;
  const bool ok = r < n;
  const int64_t o = r * 64 + (gid & 15) * 4;
  float dal = 0.f;
  if (ok) {
    const float a = alpha[r];
    const float4 im = ld4(IMG + o), tx = ld4(TXT + o), pi = ld4(PI + o), pt = ld4(PT + o), ds = ld4(dSIDE + o);
    float4 di, dt, dpi, dpt;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float g = g4(ds, k) * 0.25f;
      const float com = a * g4(im, k) + (1.f - a) * g4(tx, k);
      const float dcom = g * (1.f - g4(pi, k) - g4(pt, k));
      s4(dpi, k, g * (g4(im, k) - com));
      s4(dpt, k, g * (g4(tx, k) - com));
      s4(di, k, g * g4(pi, k) + a * dcom);
      s4(dt, k, g * g4(pt, k) + (1.f - a) * dcom);
      dal += dcom * (g4(im, k) - g4(tx, k));
    }
    st4(dIMG + o, di);
    st4(dTXT + o, dt);
    st4(dPI + o, dpi);
    st4(dPT + o, dpt);
  }
  dal = row16_sum(dal);
  if (ok && (gid & 15) == 0) {
    const float a = alpha[r];
    const float d = dal * a * (1.f - a);
    daI[r] = d;
    daT[r] = -d;
  }
}

// ----------------------------------------------------------------- small elementwise / reductions
// out (+)= a * b over n4 float4 groups (rows of 64, lds given)
__global__ void mul_kernel(int64_t rows, const float* __restrict__ a, int64_t lda, const float* __restrict__ b,
                           int64_t ldb, float* __restrict__ out, int64_t ldo, float scale, int accumulate) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= rows * 16) return;
  const int64_t r = gid >> 4;
  const int c = (gid & 15) * 4;
  const float4 x = ld4(a + r * lda + c), y = ld4(b + r * ldb + c);
  float4 v = f4(scale * x.x * y.x, scale * x.y * y.y, scale * x.z * y.z, scale * x.w * y.w);
  float* q = out + r * ldo + c;
  if (accumulate) {
    const float4 o = ld4(q);
    v = f4(v.x + o.x, v.y + o.y, v.z + o.z, v.w + o.w);
  }
  st4(q, v);
}

// per-block fp64 partials of sum(a * b) over rows x 64
__global__ void __launch_bounds__(256) dot_part_kernel(int64_t rows, const float* __restrict__ a, int64_t lda,
                                                       const float* __restrict__ b, int64_t ldb,
                                                       double* __restrict__ part) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < rows * 16;
       gid += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = gid >> 4;
    const int c = (gid & 15) * 4;
    const float4 x = ld4(a + r * lda + c), y = ld4(b + r * ldb + c);
    s += (double)x.x * y.x + (double)x.y * y.y + (double)x.z * y.z + (double)x.w * y.w;
  }
  s = gmr::wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) sum_parts_kernel(int P, const double* __restrict__ part, float scale,
                                                        float* __restrict__ out, int accumulate) {
  __shared__ double red[256];
  const double s = block_sum_parts(P, part, 1, 0, red);
  if (threadIdx.x == 0) out[0] = (float)(s * scale) + (accumulate ? out[0] : 0.f);
}

// ----------------------------------------------------------------- losses
// InfoNCE rows (genrecv1.py:407-414) on logits L = v1 v2^T / temp (B x B, in place):
//   loss[r] = logsumexp(L[r]) - L[r][r];  L[r][j] <- coef (softmax_rj - [j == r])
// rows of an in-batch InfoNCE logit block L (rows x cols, already scaled by 1/tau): row r's positive
// sits at column diag_off + r (diag_off = 0, cols = rows: the square B x B block of one process; a
// data-parallel rank holds rows [diag_off, diag_off + rows) of the global batch against all cols keys).
// loss[r] = logsumexp_j L[r, j] - L[r, diag_off + r]; with coef != 0, L is overwritten by its gradient
// coef * (softmax_r - e_{diag_off + r}).
__global__ void __launch_bounds__(256) nce_rows_kernel(int64_t cols, float* __restrict__ L, int64_t ld,
                                                       int64_t diag_off, float coef, float* __restrict__ loss) {
  const int64_t r = blockIdx.x;
  float* p = L + r * ld;
  __shared__ float red[4];
  float m = -INFINITY;
  for (int64_t j = threadIdx.x; j < cols; j += 256) m = fmaxf(m, p[j]);
  m = gmr::wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int64_t j = threadIdx.x; j < cols; j += 256) s += expf(p[j] - m);
  s = gmr::wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float S = (red[0] + red[1]) + (red[2] + red[3]);
  const float lse = m + logf(S);
  const int64_t dj = diag_off + r;
  const float diag = p[dj];
  __syncthreads();
  if (threadIdx.x == 0 && loss) loss[r] = lse - diag;
  if (coef != 0.f)
    for (int64_t j = threadIdx.x; j < cols; j += 256) p[j] = coef * expf(p[j] - lse) - (j == dj ? coef : 0.f);
}

// BPR with log-sigmoid (genrecv1.py:377-380): x = <u,p> - <u,n>; loss_b = softplus(-x);
// contrib = [dU; dP; dN] (3B x 64), dx = -sigmoid(-x) * inv_norm
__global__ void bpr_ls_kernel(int B, int64_t U, const float* __restrict__ C, const int* __restrict__ users,
                              const int* __restrict__ pos, const int* __restrict__ neg, float* __restrict__ loss,
                              float* __restrict__ contrib, float inv_norm) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = (int)(gid >> 4);
  const bool ok = b < B;
  const int c = (gid & 15) * 4;
  float4 u = f4(0, 0, 0, 0), p = u, q = u;
  if (ok) {
    u = ld4(C + (int64_t)users[b] * 64 + c);
    p = ld4(C + (U + pos[b]) * 64 + c);
    q = ld4(C + (U + neg[b]) * 64 + c);
  }
  float x = (u.x * p.x + u.y * p.y + u.z * p.z + u.w * p.w) - (u.x * q.x + u.y * q.y + u.z * q.z + u.w * q.w);
  x = row16_sum(x);
  if (!ok) return;
  if ((gid & 15) == 0) loss[b] = fmaxf(-x, 0.f) + log1pf(expf(-fabsf(x)));
  const float dx = -inv_norm / (1.f + expf(x));
  st4(contrib + (int64_t)b * 64 + c, f4(dx * (p.x - q.x), dx * (p.y - q.y), dx * (p.z - q.z), dx * (p.w - q.w)));
  st4(contrib + (int64_t)(B + b) * 64 + c, f4(dx * u.x, dx * u.y, dx * u.z, dx * u.w));
  st4(contrib + (int64_t)(2 * B + b) * 64 + c, f4(-dx * u.x, -dx * u.y, -dx * u.z, -dx * u.w));
}

// y += alpha[0] * x (alpha on the device)
__global__ void axpy_dev_kernel(int64_t n, const float* __restrict__ alpha, const float* __restrict__ x,
                                float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] += alpha[0] * x[i];
}

// out = a * b (flat)
__global__ void mul_flat_kernel(int64_t n, const float* __restrict__ a, const float* __restrict__ b,
                                float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] * b[i];
}

// Bernoulli(p_keep) keep bytes (nn.Dropout masks of the modal projections)
__global__ void keep_mask_kernel(int64_t n, float p_keep, uint64_t seed, uint64_t step, uint64_t ctr0,
                                 uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 r = gmr::Philox::gen(seed, step, ctr0 + (uint64_t)i);
  out[i] = (float)(r.x >> 8) * (1.0f / 16777216.0f) < p_keep ? 1 : 0;
}

// GenRecV1's four in-batch InfoNCE terms (genrecv1.py:389-397) through the fused contrast kernel
// (gmr_contrast_fused_f32): each term k pairs query table i1[k] with key table i2[k] of the nv tables
// [4][Bg][64]; a rank's queries are rows [row0, row0 + B) of the step, the keys all Bg rows.
struct NceTerms {
  int i1[4], i2[4];
};

// CLN_k[i] = [nv[i1_k][row0 + i] | nv[i2_k][row0 + i]]: the (query, positive) pair rows the contrast reads
// (nv tables tab rows apart, CLN terms ct rows apart)
__global__ void nce_pairs_kernel(int nterms, int64_t B, int64_t tab, int64_t ct, int64_t row0, NceTerms t,
                                 const float* __restrict__ nv, float* __restrict__ cln) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (k, row, 128 columns / 4)
  if (i >= nterms * B * 32) return;
  const int k = (int)(i / (B * 32));
  const int64_t r = (i / 32) % B;
  const int c4 = (int)(i % 32) * 4;
  const int src = c4 < 64 ? t.i1[k] : t.i2[k];
  const float4 v = *reinterpret_cast<const float4*>(nv + ((int64_t)src * tab + row0 + r) * 64 + (c4 & 63));
  *reinterpret_cast<float4*>(cln + ((int64_t)k * ct + r) * 128 + c4) = v;
}

// g[j][r] = the terms' gradients of nv[j][r], summed in term order: a query block's dP (contrib
// columns 0..63) where j = i1_k, and where j = i2_k the logsumexp part dT_k[r] plus, on the rank's rows,
// the positive part (contrib columns 64..127)
__global__ void nce_combine_kernel(int nterms, int64_t B, int64_t Bg, int64_t tab, int64_t ct, int64_t dts,
                                   int64_t row0, NceTerms t, const float* __restrict__ contrib,
                                   const float* __restrict__ dT, float* __restrict__ g) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (j, r, c)
  if (i >= 4 * Bg * 64) return;
  const int j = (int)(i / (Bg * 64));
  const int64_t r = (i / 64) % Bg;
  const int c = (int)(i % 64);
  const bool mine = r >= row0 && r < row0 + B;
  float s = 0.f;
  for (int k = 0; k < nterms; ++k) {
    if (t.i1[k] == j && mine) s += contrib[((int64_t)k * ct + r - row0) * 128 + c];
    if (t.i2[k] == j) {
      s += dT[((int64_t)k * dts + r) * 64 + c];
      if (mine) s += contrib[((int64_t)k * ct + r - row0) * 128 + 64 + c];
    }
  }
  g[((int64_t)j * tab + r) * 64 + c] = s;
}

dim3 rows16(int64_t n) { return dim3((unsigned)gmr::grid_for(n * 16, 256)); }

}  // namespace

#define GR_CHECK_ROWS(rows) GMR_ARG((rows) > 0 && (rows) < (1ll << 31), "bad row count")

extern "C" int64_t gmr_bn_parts_doubles(int64_t rows) { return (int64_t)192 * parts_for(rows); }

extern "C" int gmr_bn_fwd_f32(int64_t rows, const float* z, int64_t ldz, int32_t train, float eps, float momentum,
                              float* run_mean, float* run_var, double* parts, float* mean, float* invstd,
                              const float* w, const float* b, int32_t act, float slope, const uint8_t* keep,
                              int64_t ld_keep, float keep_scale, float* y, int64_t ldy, int32_t post, const float* aux,
                              int64_t ld_aux, const float* rs, float* out2, int64_t ld2, float* rowdot, void* stream) {
  GR_CHECK_ROWS(rows);
  GMR_ARG(z && mean && invstd && w && b && parts, "null pointer");
  GMR_ARG(ldz % 4 == 0 && ldz >= 64, "z must be rows x 64 with ld % 4 == 0");
  GMR_ARG(act >= 0 && act <= 3 && post >= 0 && post <= 3, "bad act/post");
  GMR_ARG(train || (run_mean && run_var), "eval mode needs the running statistics");
  GMR_ARG(post == 0 || aux, "post op needs aux");
  GMR_ARG(post != 1 || (rs && out2), "post RES needs rs and out2");
  GMR_ARG(post != 2 || out2, "post MUL needs out2");
  GMR_ARG(post != 3 || rowdot, "post ROWDOT needs rowdot");
  GMR_ARG(y || post != 0, "nothing to write");
  hipStream_t st = (hipStream_t)stream;
  const int P = parts_for(rows);
  if (train) {
    hipLaunchKernelGGL(bn_stats_kernel, dim3(P), dim3(256), 0, st, rows, z, ldz, parts);
    GMR_LAUNCHED();
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(1), dim3(1024), 0, st, P, parts, rows, eps, momentum, (int)train, run_mean,
                     run_var, mean, invstd);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(bn_apply_kernel, rows16(rows), dim3(256), 0, st, rows, z, ldz, mean, invstd, w, b, (int)act, slope,
                     keep, ld_keep, keep_scale, y, ldy, (int)post, aux, ld_aux, rs, out2, ld2, rowdot);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_bn_bwd_f32(int64_t rows, const float* z, int64_t ldz, const float* mean, const float* invstd,
                              const float* w, const float* b, int32_t act, float slope, const uint8_t* keep,
                              int64_t ld_keep, float keep_scale, const float* dy, int64_t lddy, const float* mul,
                              int64_t ld_mul, const float* da, const float* v, double* parts, float* sums, float* dw,
                              float* db, float* dv, int32_t accumulate_params, float* dz, int64_t lddz,
                              int32_t accumulate_dz, void* stream) {
  GR_CHECK_ROWS(rows);
  GMR_ARG(z && mean && invstd && w && b && parts && sums && dz, "null pointer");
  GMR_ARG((dy != nullptr) != (da != nullptr), "exactly one of dy / da");
  GMR_ARG(!da || (v && dv), "rowdot backward needs v and dv");
  hipStream_t st = (hipStream_t)stream;
  BnBwdIn p{z, ldz, mean, invstd, w, b, (int)act, slope, keep, ld_keep, keep_scale, dy, lddy, mul, ld_mul, da, v};
  const int P = parts_for(rows);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(P), dim3(256), 0, st, rows, p, parts);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(1), dim3(1024), 0, st, P, parts, rows, dw, db, dv, sums,
                     (int)accumulate_params);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(bn_bwd_apply_kernel, rows16(rows), dim3(256), 0, st, rows, p, sums, dz, lddz, (int)accumulate_dz);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_gr_content_fwd(int64_t n, const float* E, const float* A1, const float* A2, const float* ow,
                                  const float* gw, float* C, void* stream) {
  GR_CHECK_ROWS(n);
  GMR_ARG(E && A1 && A2 && ow && gw && C, "null pointer");
  hipLaunchKernelGGL(content_fwd_kernel, rows16(n), dim3(256), 0, (hipStream_t)stream, n, E, A1, A2, ow, gw, C);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int64_t gmr_gr_parts(int64_t n) { return 2 * 1024; }

extern "C" int gmr_gr_content_bwd(int64_t n, const float* E, const float* A1, const float* A2, const float* dC,
                                  const float* T1, const float* T2, const float* ow, const float* gw, float reg2,
                                  double* parts, float* dE, float* dow, float* dgw, void* stream) {
  GR_CHECK_ROWS(n);
  GMR_ARG(E && A1 && A2 && dC && T1 && T2 && ow && gw && parts && dE && dow && dgw, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int P = gmr::grid_for(n * 16, 256, 1024);
  hipLaunchKernelGGL(content_bwd_part_kernel, dim3(P), dim3(256), 0, st, n, E, A1, A2, dC, parts);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(content_bwd_weights_kernel, dim3(1), dim3(256), 0, st, P, parts, ow, gw, dow, dgw);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(content_bwd_combine_kernel, rows16(n), dim3(256), 0, st, n, dC, T1, T2, ow, gw, E, reg2, dE);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_gr_fusion_fwd(int64_t n, const float* IMG, const float* TXT, const float* aI, const float* aT,
                                 const float* PI, const float* PT, float* SIDE, float* alpha, void* stream) {
  GR_CHECK_ROWS(n);
  GMR_ARG(IMG && TXT && aI && aT && PI && PT && SIDE && alpha, "null pointer");
  hipLaunchKernelGGL(fusion_fwd_kernel, rows16(n), dim3(256), 0, (hipStream_t)stream, n, IMG, TXT, aI, aT, PI, PT,
                     SIDE, alpha);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_gr_fusion_bwd(int64_t n, const float* IMG, const float* TXT, const float* alpha, const float* PI,
                                 const float* PT, const float* dSIDE, float* dIMG, float* dTXT, float* daI, float* daT,
                                 float* dPI, float* dPT, void* stream) {
  GR_CHECK_ROWS(n);
  GMR_ARG(IMG && TXT && alpha && PI && PT && dSIDE && dIMG && dTXT && daI && daT && dPI && dPT, "null pointer");
  hipLaunchKernelGGL(fusion_bwd_kernel, rows16(n), dim3(256), 0, (hipStream_t)stream, n, IMG, TXT, alpha, PI, PT,
                     dSIDE, dIMG, dTXT, daI, daT, dPI, dPT);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_mul64_f32(int64_t rows, const float* a, int64_t lda, const float* b, int64_t ldb, float* out,
                             int64_t ldo, float scale, int32_t accumulate, void* stream) {
  GR_CHECK_ROWS(rows);
  GMR_ARG(a && b && out && lda % 4 == 0 && ldb % 4 == 0 && ldo % 4 == 0, "bad args");
  hipLaunchKernelGGL(mul_kernel, rows16(rows), dim3(256), 0, (hipStream_t)stream, rows, a, lda, b, ldb, out, ldo,
                     scale, (int)accumulate);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dot64_f32(int64_t rows, const float* a, int64_t lda, const float* b, int64_t ldb, double* parts,
                             float scale, float* out, int32_t accumulate, void* stream) {
  GR_CHECK_ROWS(rows);
  GMR_ARG(a && b && parts && out, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int P = gmr::grid_for(rows * 16, 256, 1024);
  hipLaunchKernelGGL(dot_part_kernel, dim3(P), dim3(256), 0, st, rows, a, lda, b, ldb, parts);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(256), 0, st, P, parts, scale, out, (int)accumulate);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_nce_rows_f32(int64_t B, float* L, int64_t ld, float coef, float* loss, void* stream) {
  GMR_ARG(L && B > 0 && ld >= B, "bad args");
  hipLaunchKernelGGL(nce_rows_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, B, L, ld, (int64_t)0, coef,
                     loss);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_nce_rows_off_f32(int64_t rows, int64_t cols, float* L, int64_t ld, int64_t diag_off, float coef,
                                    float* loss, void* stream) {
  GMR_ARG(L && rows > 0 && cols > 0 && ld >= cols && diag_off >= 0 && diag_off + rows <= cols, "bad args");
  hipLaunchKernelGGL(nce_rows_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, cols, L, ld, diag_off,
                     coef, loss);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_bpr_logsigmoid_f32(int32_t B, int64_t U, const float* C, const int32_t* users, const int32_t* pos,
                                      const int32_t* neg, float* loss, float* contrib, float inv_norm, void* stream) {
  GMR_ARG(C && users && pos && neg && loss && contrib && B > 0, "bad args");
  hipLaunchKernelGGL(bpr_ls_kernel, rows16(B), dim3(256), 0, (hipStream_t)stream, B, U, C, users, pos, neg, loss,
                     contrib, inv_norm);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_axpy_dev_f32(int64_t n, const float* alpha, const float* x, float* y, void* stream) {
  GMR_ARG(alpha && x && y && n > 0, "bad args");
  hipLaunchKernelGGL(axpy_dev_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, alpha, x, y);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_mul_f32(int64_t n, const float* a, const float* b, float* out, void* stream) {
  GMR_ARG(a && b && out && n > 0, "bad args");
  hipLaunchKernelGGL(mul_flat_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, a, b, out);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_nce_pairs_f32(int32_t nterms, int64_t B, int64_t Bg, int64_t row0, const int32_t* i1,
                                 const int32_t* i2, const float* nv, int64_t tab, float* cln, int64_t ct, void* stream) {
  GMR_ARG(nv && cln && i1 && i2 && nterms > 0 && nterms <= 4 && B > 0 && Bg >= B && row0 >= 0 && row0 + B <= Bg &&
              tab >= Bg && ct >= B,
          "bad args");
  NceTerms t{};
  for (int k = 0; k < nterms; ++k) {
    GMR_ARG(i1[k] >= 0 && i1[k] < 4 && i2[k] >= 0 && i2[k] < 4, "term tables index the 4 nv tables");
    t.i1[k] = i1[k];
    t.i2[k] = i2[k];
  }
  hipLaunchKernelGGL(nce_pairs_kernel, dim3(gmr::grid_for((int64_t)nterms * B * 32, 256)), dim3(256), 0,
                     (hipStream_t)stream, nterms, B, tab, ct, row0, t, nv, cln);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_nce_combine_f32(int32_t nterms, int64_t B, int64_t Bg, int64_t row0, const int32_t* i1,
                                   const int32_t* i2, const float* contrib, int64_t ct, const float* dT, int64_t dts,
                                   float* g, int64_t tab, void* stream) {
  GMR_ARG(contrib && dT && g && i1 && i2 && nterms > 0 && nterms <= 4 && B > 0 && Bg >= B && row0 >= 0 &&
              row0 + B <= Bg && ct >= B && dts >= Bg && tab >= Bg,
          "bad args");
  NceTerms t{};
  for (int k = 0; k < nterms; ++k) {
    GMR_ARG(i1[k] >= 0 && i1[k] < 4 && i2[k] >= 0 && i2[k] < 4, "term tables index the 4 nv tables");
    t.i1[k] = i1[k];
    t.i2[k] = i2[k];
  }
  hipLaunchKernelGGL(nce_combine_kernel, dim3(gmr::grid_for(4 * Bg * 64, 256)), dim3(256), 0, (hipStream_t)stream,
                     nterms, B, Bg, tab, ct, dts, row0, t, contrib, dT, g);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_keep_mask_u8(int64_t n, float p_keep, uint64_t seed, uint64_t step, uint64_t ctr0, uint8_t* out,
                                void* stream) {
  GMR_ARG(out && n > 0 && p_keep > 0.f && p_keep <= 1.f, "bad args");
  hipLaunchKernelGGL(keep_mask_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, p_keep, seed,
                     step, ctr0, out);
  GMR_LAUNCHED();
  return GMR_OK;
}
