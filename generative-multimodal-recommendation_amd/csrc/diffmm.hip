// Fused row-wise kernels of the DiffMM recommendation step (forward + hand-derived backward).
//
// Layout in HBM (N = U + I nodes, d = 64):
//   E0      = [uEmbeds; iEmbeds]            N x 64   (one contiguous parameter slab)
//   NF      = [norm(imgF) | norm(txtF)]     I x 128
//   G, H    = adj @ [...] for image|text    N x 128
//   Q_img   = iadj @ [E0 | S_img]           N x 128  (ris-adj term | contrastive view)
//   E       = G + H + lambda * [IA | TA]    N x 128  (written over G)
//   M       = w0 * E_img + w1 * E_txt       N x 64
//   Emb     = M + adj@M + ris * norm(M)     N x 64   (forward_MM output)
// Reference: models/diffmm.py:129-258.
#include <algorithm>

#include <cstdlib>

#include "gmr_common.h"

namespace {

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
__device__ __forceinline__ float4 f4(float a, float b, float c, float d) { return make_float4(a, b, c, d); }
__device__ __forceinline__ float4 sub4(float4 a, float4 b) { return f4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
__device__ __forceinline__ float4 mul4(float4 a, float4 b) { return f4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }

// reduce across the 16 lanes that hold one 64-float row
__device__ __forceinline__ float row16_sum(float v) {
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

__device__ __forceinline__ void softmax2(const float* mw, float& w0, float& w1) {
  float a = mw[0], b = mw[1];
  float mx = fmaxf(a, b);
  float ea = expf(a - mx), eb = expf(b - mx);
  float s = ea + eb;
  w0 = ea / s;
  w1 = eb / s;
}

// normalize backward of one 64-column row held by 16 lanes (4 columns each): (g - y <y,g>) / nrm, the projection
// term dropped when the norm was clamped, then the leaky-ReLU backward on sign(y) (slope 1: none); the
// expression of normalize_bwd_kernel, so the fused callers give its bits
__device__ __forceinline__ float4 nbwd_leaky(float4 g, float4 y, float nv, float slope) {
  float dp = row16_sum(dot4(y, g));
  if (nv <= 1e-12f) dp = 0.f;
  float4 o = gmr::f4_scale(1.f / nv, sub4(g, gmr::f4_scale(dp, y)));
  if (slope != 1.f) {
    o.x *= y.x > 0.f ? 1.f : slope;
    o.y *= y.y > 0.f ? 1.f : slope;
    o.z *= y.z > 0.f ? 1.f : slope;
    o.w *= y.w > 0.f ? 1.f : slope;
  }
  return o;
}

// E = G + H + lam * [Qi[:, :64] | Qt[:, :64]] (in place over G);  M = w0*E_img + w1*E_txt
__global__ void combine_fwd_kernel(int64_t n, float* __restrict__ G, const float* __restrict__ H,
                                   const float* __restrict__ Qi, const float* __restrict__ Qt,
                                   const float* __restrict__ mw, float lam, float* __restrict__ M) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * 16) return;
  const int64_t r = gid >> 4;
  const int c = (gid & 15) * 4;
  float w0, w1;
  softmax2(mw, w0, w1);
  float4 gi = ld4(G + r * 128 + c), gt = ld4(G + r * 128 + 64 + c);
  float4 hi = ld4(H + r * 128 + c), ht = ld4(H + r * 128 + 64 + c);
  float4 ai = ld4(Qi + r * 128 + c), at = ld4(Qt + r * 128 + c);
  float4 ei = gmr::f4_fma(lam, ai, gmr::f4_add(gi, hi));
  float4 et = gmr::f4_fma(lam, at, gmr::f4_add(gt, ht));
  st4(G + r * 128 + c, ei);
  st4(G + r * 128 + 64 + c, et);
  st4(M + r * 64 + c, gmr::f4_fma(w1, et, gmr::f4_scale(w0, ei)));
}

// Emb = M + L + ris * M / max(|M|, 1e-12); nrm[r] = max(|M_r|, 1e-12)
__global__ void final_fwd_kernel(int64_t n, const float* __restrict__ M, const float* __restrict__ L, float ris,
                                 float* __restrict__ Emb, float* __restrict__ nrm) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = gid >> 4;
  const bool ok = r < n;
  const int c = (gid & 15) * 4;
  float4 m = ok ? ld4(M + r * 64 + c) : f4(0, 0, 0, 0);
  float ss = row16_sum(dot4(m, m));
  if (!ok) return;
  float nv = fmaxf(sqrtf(ss), 1e-12f);
  float4 l = ld4(L + r * 64 + c);
  st4(Emb + r * 64 + c, gmr::f4_fma(ris / nv, m, gmr::f4_add(m, l)));
  if ((gid & 15) == 0) nrm[r] = nv;
}

// contrastive views: K = C + K2 (C = Q[:, 64:]); CLN = normalize(K + 1e-8) for image|text -> N x 128
__global__ void cl_fwd_kernel(int64_t n, const float* __restrict__ Qi, const float* __restrict__ Qt,
                              const float* __restrict__ K2, float* __restrict__ CLN, float* __restrict__ nrm) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = gid >> 5;  // 32 threads per row: 16 image + 16 text
  const bool ok = r < n;
  const int half = (gid >> 4) & 1;
  const int c = (gid & 15) * 4;
  const float* Q = half ? Qt : Qi;
  float4 k = ok ? gmr::f4_add(ld4(Q + r * 128 + 64 + c), ld4(K2 + r * 128 + half * 64 + c)) : f4(0, 0, 0, 0);
  k = f4(k.x + 1e-8f, k.y + 1e-8f, k.z + 1e-8f, k.w + 1e-8f);
  float ss = row16_sum(dot4(k, k));
  if (!ok) return;
  float nv = fmaxf(sqrtf(ss), 1e-12f);
  st4(CLN + r * 128 + half * 64 + c, gmr::f4_scale(1.f / nv, k));
  if ((gid & 15) == 0) nrm[half * n + r] = nv;  // [img norms | txt norms]
}

// Row L2-normalisation of a column block: y = x / max(|x|, eps). 16 lanes per 64 columns.
__global__ void normalize_rows_kernel(int64_t n, int cols, const float* __restrict__ x, int64_t ldx, float* __restrict__ y,
                                      int64_t ldy, float* __restrict__ nrm) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = gid >> 4;
  const bool ok = r < n;
  const int l = gid & 15;
  float ss = 0.f;
  if (ok)
    for (int c = l * 4; c < cols; c += 64) {
      float4 v = ld4(x + r * ldx + c);
      ss += dot4(v, v);
    }
  ss = row16_sum(ss);
  if (!ok) return;
  float nv = fmaxf(sqrtf(ss), 1e-12f);
  for (int c = l * 4; c < cols; c += 64) st4(y + r * ldy + c, gmr::f4_scale(1.f / nv, ld4(x + r * ldx + c)));
  if (l == 0 && nrm) nrm[r] = nv;
}

// normalize backward: dx = (dy - y <y,dy>) / nrm   (y = output, nrm = clamped norm);
// if nrm was clamped (== eps) the projection term vanishes.  Optional leaky-ReLU backward
// on the pre-normalised input (sign(x) == sign(y)).  dx may alias dy.
__global__ void normalize_bwd_kernel(int64_t n, int cols, const float* __restrict__ y, int64_t ldy,
                                     const float* __restrict__ nrm, const float* dy, int64_t lddy, float* dx,
                                     int64_t lddx, float slope, int accumulate) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = gid >> 4;
  const bool ok = r < n;
  const int l = gid & 15;
  float dp = 0.f;
  if (ok)
    for (int c = l * 4; c < cols; c += 64) dp += dot4(ld4(y + r * ldy + c), ld4(dy + r * lddy + c));
  dp = row16_sum(dp);
  if (!ok) return;
  const float nv = nrm[r];
  if (nv <= 1e-12f) dp = 0.f;
  const float inv = 1.f / nv;
  for (int c = l * 4; c < cols; c += 64) {
    float4 yy = ld4(y + r * ldy + c);
    float4 g = gmr::f4_scale(inv, sub4(ld4(dy + r * lddy + c), gmr::f4_scale(dp, yy)));
    if (slope != 1.f) {
      g.x *= yy.x > 0.f ? 1.f : slope;
      g.y *= yy.y > 0.f ? 1.f : slope;
      g.z *= yy.z > 0.f ? 1.f : slope;
      g.w *= yy.w > 0.f ? 1.f : slope;
    }
    float* o = dx + r * lddx + c;
    if (accumulate) g = gmr::f4_add(g, ld4(o));
    st4(o, g);
  }
}

// BPR with gathers: x = <a,p> - <a,n>;  loss_b = -log(1e-10 + sigmoid(x));
// contributions (scaled by 1/B): slot b -> d a, slot B+b -> d p, slot 2B+b -> d n.
__device__ __forceinline__ void bpr_rows(int gid, int B, int64_t U, const float* __restrict__ Emb,
                                         const int* __restrict__ users, const int* __restrict__ pos,
                                         const int* __restrict__ neg, float* __restrict__ loss,
                                         float* __restrict__ contrib, float inv_norm) {
  const int b = gid >> 4;
  const bool ok = b < B;
  const int c = (gid & 15) * 4;
  float4 a = f4(0, 0, 0, 0), p = a, q = a;
  if (ok) {
    a = ld4(Emb + (int64_t)users[b] * 64 + c);
    p = ld4(Emb + (U + pos[b]) * 64 + c);
    q = ld4(Emb + (U + neg[b]) * 64 + c);
  }
  float x = row16_sum(dot4(a, p) - dot4(a, q));
  if (!ok) return;
  float s = 1.f / (1.f + expf(-x));
  float gx = -(s * (1.f - s)) / (1e-10f + s) * inv_norm;  // inv_norm = 1 / rows of the (global) batch
  if ((gid & 15) == 0) loss[b] = -logf(1e-10f + s);
  st4(contrib + (int64_t)b * 64 + c, gmr::f4_scale(gx, sub4(p, q)));
  st4(contrib + ((int64_t)B + b) * 64 + c, gmr::f4_scale(gx, a));
  st4(contrib + (2 * (int64_t)B + b) * 64 + c, gmr::f4_scale(-gx, a));
}

__global__ void bpr_kernel(int B, int64_t U, const float* __restrict__ Emb, const int* __restrict__ users,
                           const int* __restrict__ pos, const int* __restrict__ neg, float* __restrict__ loss,
                           float* __restrict__ contrib, float inv_norm) {
  bpr_rows(blockIdx.x * blockDim.x + threadIdx.x, B, U, Emb, users, pos, neg, loss, contrib, inv_norm);
}

// Row softmax of contrastive logits L (already divided by temp), in place:
//   S_b = sum_j exp(L_bj)   (no max subtraction, as the reference; |L| <= 1/temp)
//   P_bj = coef * exp(L_bj) / S_b ;  lse[b] = log S_b
__global__ void __launch_bounds__(256) row_softmax_kernel(int64_t rows, int64_t cols, float* __restrict__ L, int64_t ld,
                                                          float coef, float* __restrict__ lse) {
  const int64_t r = blockIdx.x;
  if (r >= rows) return;
  float* p = L + r * ld;
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t j = threadIdx.x; j < cols; j += 256) s += expf(p[j]);
  s = gmr::wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float S = (red[0] + red[1]) + (red[2] + red[3]);
  const float k = coef / S;
  for (int64_t j = threadIdx.x; j < cols; j += 256) p[j] = k * expf(p[j]);
  if (threadIdx.x == 0) lse[r] = logf(S);
}

// contrastive per-row terms for a gathered batch.  For row b with node t_b:
//   loss_b = lse_b - <p1_b, p2_b>/temp     (p1 = CLN[t_b, 0:64], p2 = CLN[t_b, 64:128])
//   contrib (128 wide): [ -coef/temp * p2_b | -coef/temp * p1_b ]  (dp1 dense part added by GEMM)
__global__ void contrast_rows_kernel(int B, const float* __restrict__ CLN, const int* __restrict__ nodes, int64_t node_off,
                                     const float* __restrict__ lse, float inv_temp, float coef, float* __restrict__ loss,
                                     float* __restrict__ contrib, int64_t ld_contrib) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = gid >> 4;
  const bool ok = b < B;
  const int c = (gid & 15) * 4;
  float4 p1 = f4(0, 0, 0, 0), p2 = p1;
  if (ok) {
    const int64_t t = node_off + nodes[b];
    p1 = ld4(CLN + t * 128 + c);
    p2 = ld4(CLN + t * 128 + 64 + c);
  }
  float d = row16_sum(dot4(p1, p2));
  if (!ok) return;
  if ((gid & 15) == 0) loss[b] = lse[b] - d * inv_temp;
  const float k = -coef * inv_temp;
  float* o = contrib + (int64_t)b * ld_contrib;
  st4(o + c, gmr::f4_fma(k, p2, ld4(o + c)));  // adds to dp1 produced by P @ table (already in contrib)
  st4(o + 64 + c, gmr::f4_scale(k, p1));
}

// gather rows: out[b] = src[off + idx[b]] (cols % 4 == 0)
__global__ void gather_rows_kernel(int B, int cols, const float* __restrict__ src, int64_t lds, const int* __restrict__ idx,
                                   int64_t off, float* __restrict__ out, int64_t ldo) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c4 = cols / 4;
  const int64_t b = gid / c4;
  if (b >= B) return;
  const int c = (int)(gid % c4) * 4;
  st4(out + b * ldo + c, ld4(src + (off + idx[b]) * lds + c));
}

// Deterministic scatter-add of contribution rows through a sorted (key << 32 | slot) plan:
// each run of equal keys is summed in slot order and added to dst[key] (one 16-lane group per
// run start; runs are disjoint so there is no write race).
__global__ void scatter_sorted_kernel(int n, int cols, const unsigned long long* __restrict__ plan,
                                      const float* __restrict__ contrib, int64_t ldc, float* __restrict__ dst,
                                      int64_t ldd) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lanes = cols / 4;
  const int64_t i = gid / lanes;
  if (i >= n) return;
  const int c = (int)(gid % lanes) * 4;
  const unsigned long long e = plan[i];
  const unsigned key = (unsigned)(e >> 32);
  if (key == 0xFFFFFFFFu) return;
  if (i > 0 && (unsigned)(plan[i - 1] >> 32) == key) return;
  // the run is read 8 plan words at a time (independent loads: a popular item's run of dozens of
  // slots is 1/8 the dependent round trips), then summed in slot order
  float4 s = f4(0, 0, 0, 0);
  for (int64_t j0 = i; j0 < n; j0 += 8) {
    unsigned long long ej[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) ej[q] = j0 + q < n ? plan[j0 + q] : ~0ull;
    float4 x[8];
    int m = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const bool in = (unsigned)(ej[q] >> 32) == key && m == q;
      m += in ? 1 : 0;
      x[q] = in ? ld4(contrib + (int64_t)(unsigned)(ej[q] & 0xFFFFFFFFull) * ldc + c) : f4(0, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < m) s = gmr::f4_add(s, x[q]);
    if (m < 8) break;
  }
  float* o = dst + (int64_t)key * ldd + c;
  st4(o, gmr::f4_add(ld4(o), s));
}

// The contrastive views' sparse gradient rows through the sorted plan (as scatter_sorted_kernel, cols = 128),
// taken through the normalize backward of each 64-column view (y = CLN, nrm = [nrm_img | nrm_txt] per node) and
// added to dK: dK[key] += nbwd([s_img | s_txt]).  The normalize backward is linear in its input, so adding
// nbwd(sparse part) to the table pass's nbwd(dense part) (cl_table_reduce_nbwd_kernel) gives nbwd of the sum.
__global__ void scatter_sorted_nbwd_kernel(int n, const unsigned long long* __restrict__ plan,
                                           const float* __restrict__ contrib, int64_t ldc,
                                           const float* __restrict__ y, const float* __restrict__ nrm, int64_t nn,
                                           float* __restrict__ dK) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = gid >> 5;
  if (i >= n) return;  // (whole 32-lane entries: the 16-lane row sums below see complete groups)
  const int c = (int)(gid & 31) * 4;
  const unsigned long long e = plan[i];
  const unsigned key = (unsigned)(e >> 32);
  if (key == 0xFFFFFFFFu) return;
  if (i > 0 && (unsigned)(plan[i - 1] >> 32) == key) return;
  float4 s = f4(0, 0, 0, 0);
  for (int64_t j0 = i; j0 < n; j0 += 8) {
    unsigned long long ej[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) ej[q] = j0 + q < n ? plan[j0 + q] : ~0ull;
    float4 x[8];
    int m = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const bool in = (unsigned)(ej[q] >> 32) == key && m == q;
      m += in ? 1 : 0;
      x[q] = in ? ld4(contrib + (int64_t)(unsigned)(ej[q] & 0xFFFFFFFFull) * ldc + c) : f4(0, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < m) s = gmr::f4_add(s, x[q]);
    if (m < 8) break;
  }
  const int half = c >> 6;
  const float4 g = nbwd_leaky(s, ld4(y + (int64_t)key * 128 + c), nrm[half * nn + key], 1.f);
  float* o = dK + (int64_t)key * 128 + c;
  st4(o, gmr::f4_add(ld4(o), g));
}

// final backward: dM = dEmb + T1 + ris * nbwd(M, dEmb);  dE = [w0 dM | w1 dM];
// per-block partial sums of <E_img, dM>, <E_txt, dM> for the modal-weight gradient.
// clear: dEmb is zeroed after it is read (this is its last reader in the step), so the next step's sorted
// scatter adds onto zeros without a fill pass.
// Ri / Rt (optional, lam): the left halves of the UI-graph backward sources, lam * dE_img / lam * dE_txt
// (what cl_bwd_kernel would write there).
__global__ void __launch_bounds__(256) final_bwd_kernel(int64_t n, float* __restrict__ dEmb,
                                                        const float* __restrict__ T1, const float* __restrict__ M,
                                                        const float* __restrict__ nrmM, float ris,
                                                        const float* __restrict__ E, const float* __restrict__ mw,
                                                        float* __restrict__ dE, float* __restrict__ part, int clear,
                                                        float lam, float* __restrict__ Ri, float* __restrict__ Rt) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = gid >> 4;
  const bool ok = r < n;
  const int c = (gid & 15) * 4;
  float w0, w1;
  softmax2(mw, w0, w1);
  float4 g = f4(0, 0, 0, 0), m = g, t = g;
  float nv = 1.f;
  if (ok) {
    g = ld4(dEmb + r * 64 + c);
    m = ld4(M + r * 64 + c);
    t = ld4(T1 + r * 64 + c);
    nv = nrmM[r];
    if (clear) st4(dEmb + r * 64 + c, f4(0.f, 0.f, 0.f, 0.f));
  }
  float4 y = gmr::f4_scale(1.f / nv, m);
  float dp = row16_sum(dot4(y, g));
  if (nv <= 1e-12f) dp = 0.f;
  float4 dm = gmr::f4_add(gmr::f4_add(g, t), gmr::f4_scale(ris / nv, sub4(g, gmr::f4_scale(dp, y))));
  float si = 0.f, st = 0.f;
  if (ok) {
    float4 ei = ld4(E + r * 128 + c), et = ld4(E + r * 128 + 64 + c);
    si = dot4(ei, dm);
    st = dot4(et, dm);
    const float4 di = gmr::f4_scale(w0, dm), dt = gmr::f4_scale(w1, dm);
    st4(dE + r * 128 + c, di);
    st4(dE + r * 128 + 64 + c, dt);
    if (Ri) {
      st4(Ri + r * 128 + c, gmr::f4_scale(lam, di));
      st4(Rt + r * 128 + c, gmr::f4_scale(lam, dt));
    }
  }
  __shared__ float red[2][4];
  si = gmr::wave_sum(si);
  st = gmr::wave_sum(st);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = si;
    red[1][threadIdx.x >> 6] = st;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x * 2 + 0] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    part[blockIdx.x * 2 + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

// modal-weight gradient: dw_i = sum of partials; dmw = w .* (dw - <w, dw>)  (softmax backward)
__device__ __forceinline__ void mw_grad_block(int nparts, const float* __restrict__ part, const float* __restrict__ mw,
                                              float* __restrict__ dmw, int accumulate) {
  __shared__ float red[2][4];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  a = gmr::wave_sum(a);
  b = gmr::wave_sum(b);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = a;
    red[1][threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float da = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    float db = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    float w0, w1;
    softmax2(mw, w0, w1);
    float s = w0 * da + w1 * db;
    float g0 = w0 * (da - s), g1 = w1 * (db - s);
    dmw[0] = accumulate ? dmw[0] + g0 : g0;
    dmw[1] = accumulate ? dmw[1] + g1 : g1;
  }
}

__global__ void mw_grad_kernel(int nparts, const float* __restrict__ part, const float* __restrict__ mw,
                               float* __restrict__ dmw, int accumulate) {
  mw_grad_block(nparts, part, mw, dmw, accumulate);
}

// dG = dE + [T2[:U]; 0]   (N x 128)
__global__ void dg_kernel(int64_t n, int64_t U, const float* __restrict__ dE, const float* __restrict__ T2,
                          float* __restrict__ dG) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * 32) return;
  const int64_t r = gid >> 5;
  const int c = (int)(gid & 31) * 4;
  float4 v = ld4(dE + r * 128 + c);
  if (r < U) v = gmr::f4_add(v, ld4(T2 + r * 128 + c));
  st4(dG + r * 128 + c, v);
}

// contrastive backward through "K = C + adj@C":  dC = dK + T  (in place over T); also
// build the iadj/tadj backward sources  Rsrc_img = [lam*dE_img | dC_img], Rsrc_txt likewise.
// clear: dK[:, :64] is zeroed after it is read (its last reader in the step; only the next step's sorted scatter
// writes it, onto zeros); left: also write the lam * dE left halves (0: final_bwd_kernel wrote them)
__global__ void cl_bwd_kernel(int64_t n, float* __restrict__ dK, const float* __restrict__ T,
                              const float* __restrict__ dE, float lam, float* __restrict__ Ri,
                              float* __restrict__ Rt, int clear, int left) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * 16) return;
  const int64_t r = gid >> 4;
  const int c = (int)(gid & 15) * 4;
  float4 dci = gmr::f4_add(ld4(dK + r * 128 + c), ld4(T + r * 128 + c));
  float4 dct = gmr::f4_add(ld4(dK + r * 128 + 64 + c), ld4(T + r * 128 + 64 + c));
  if (clear) st4(dK + r * 128 + c, f4(0.f, 0.f, 0.f, 0.f));
  if (left) {
    st4(Ri + r * 128 + c, gmr::f4_scale(lam, ld4(dE + r * 128 + c)));
    st4(Rt + r * 128 + c, gmr::f4_scale(lam, ld4(dE + r * 128 + 64 + c)));
  }
  st4(Ri + r * 128 + 64 + c, dci);
  st4(Rt + r * 128 + 64 + c, dct);
}

// gradient assembly (dE0 is written, not accumulated: the rec step's slab gradient needs no zeroing pass):
//   dE0[:U]  = T3u_img + T3u_txt + Ri[:U, :64] + Ri[:U, 64:] + Rt[:U, :64] + Rt[:U, 64:] + 2 reg uE
//   dE0[U:]  = T2i_img + T2i_txt + Ri[U:, :64] + Rt[U:, :64] + 2 reg iE
//   dNF[:, :64] = T3[U:, :64] + Ri[U:, 64:] ;  dNF[:, 64:] = T3[U:, 64:] + Rt[U:, 64:]
// T2 = adj@dE (its item rows feed diE), T3 = adj@dG.
// NF / nrmF (optional, slope): dNF leaves through the modality projections' backward, normalize_bwd_kernel with
// the leaky-ReLU slope on each 64-column half (the same expression: bit-identical to the separate launches)
__global__ void assemble_kernel(int64_t n, int64_t U, const float* __restrict__ T2, const float* __restrict__ T3,
                                const float* __restrict__ Ri, const float* __restrict__ Rt,
                                const float* __restrict__ E0, float reg2, float* __restrict__ dE0,
                                float* __restrict__ dNF, const float* __restrict__ NF,
                                const float* __restrict__ nrmF, float slope, float* __restrict__ dK_clear,
                                int t3u_from_t2) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * 16) return;
  const int64_t r = gid >> 4;
  const int c = (int)(gid & 15) * 4;
  const int64_t o = r * 128 + c;
  if (dK_clear) st4(dK_clear + o, f4(0.f, 0.f, 0.f, 0.f));  // dK[:, :64]: zero for the next step's scatter
  float4 g;
  if (r < U) {
    // T3's user rows gather only item rows of dG = dE there: they ARE T2's user rows (adj is bipartite), so a
    // caller that computed only T3's item rows passes t3u_from_t2
    const float* T3u = t3u_from_t2 ? T2 : T3;
    g = gmr::f4_add(ld4(T3u + o), ld4(T3u + o + 64));
    g = gmr::f4_add(g, gmr::f4_add(ld4(Ri + o), ld4(Ri + o + 64)));
    g = gmr::f4_add(g, gmr::f4_add(ld4(Rt + o), ld4(Rt + o + 64)));
  } else {
    g = gmr::f4_add(ld4(T2 + o), ld4(T2 + o + 64));
    g = gmr::f4_add(g, gmr::f4_add(ld4(Ri + o), ld4(Rt + o)));
    const int64_t ri = r - U;
    float4 gi = gmr::f4_add(ld4(T3 + o), ld4(Ri + o + 64));
    float4 gt = gmr::f4_add(ld4(T3 + o + 64), ld4(Rt + o + 64));
    if (NF) {  // (all 16 lanes of a row take this branch together: the row sums below are lane-complete)
      const int64_t I = n - U;
      gi = nbwd_leaky(gi, ld4(NF + ri * 128 + c), nrmF[ri], slope);
      gt = nbwd_leaky(gt, ld4(NF + ri * 128 + 64 + c), nrmF[I + ri], slope);
    }
    st4(dNF + ri * 128 + c, gi);
    st4(dNF + ri * 128 + 64 + c, gt);
  }
  g = gmr::f4_fma(reg2, ld4(E0 + r * 64 + c), g);
  st4(dE0 + r * 64 + c, g);
}

// sum of a float vector into out[0] (single block, deterministic); optional scale and accumulation
__global__ void sum_kernel(int64_t n, const float* __restrict__ x, float scale, float* __restrict__ out, int accumulate) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += (double)x[i];
  s = gmr::wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = (float)(((red[0] + red[1]) + (red[2] + red[3])) * (double)scale);
    out[0] = accumulate ? out[0] + v : v;
  }
}

// squared Frobenius norm: per-block fp64 partials (grid-stride) then one ordered sum
__device__ __forceinline__ void sqnorm_block(int bid, int nblocks, int64_t n, const float* __restrict__ x,
                                             double* __restrict__ part) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t i = (int64_t)bid * 256 + threadIdx.x; i < n; i += (int64_t)nblocks * 256) {
    const double v = x[i];
    s += v * v;
  }
  s = gmr::wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[bid] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) sqnorm_part_kernel(int64_t n, const float* __restrict__ x,
                                                          double* __restrict__ part) {
  sqnorm_block(blockIdx.x, gridDim.x, n, x, part);
}

// the BPR rows (blocks [0, nb)) and the regulariser's squared-norm partials of E0 (blocks [nb, nb + g), the
// partition of sqnorm_part_kernel with g blocks: the same partials) in one launch (DiffMM rec step)
__global__ void __launch_bounds__(256) bpr_sqnorm_kernel(int B, int64_t U, const float* __restrict__ Emb,
                                                         const int* __restrict__ users, const int* __restrict__ pos,
                                                         const int* __restrict__ neg, float* __restrict__ loss,
                                                         float* __restrict__ contrib, float inv_norm, int nb,
                                                         int64_t n_sq, const float* __restrict__ x, int g,
                                                         double* __restrict__ part) {
  if ((int)blockIdx.x < nb)
    bpr_rows(blockIdx.x * blockDim.x + threadIdx.x, B, U, Emb, users, pos, neg, loss, contrib, inv_norm);
  else
    sqnorm_block((int)blockIdx.x - nb, g, n_sq, x, part);
}

__global__ void sqnorm_fin_kernel(int nparts, const double* __restrict__ part, float scale, float* __restrict__ out,
                                  int accumulate) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  s = gmr::wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = (float)(((red[0] + red[1]) + (red[2] + red[3])) * (double)scale);
    out[0] = accumulate ? out[0] + v : v;
  }
}

// bitonic sort of one keyset per block: pairs (key << 32 | slot), size padded to pow2 <= 8192
__global__ void __launch_bounds__(1024) sort_keys_kernel(const int* __restrict__ keys, const int64_t* __restrict__ offs,
                                                         const int* __restrict__ key_add, int n_keysets_per_batch,
                                                         int64_t key_stride, unsigned long long* __restrict__ out,
                                                         int64_t out_stride, int pow2) {
  __shared__ unsigned long long s[8192];
  // block = (batch, keyset); keyset k covers slots [k*len, (k+1)*len) of the batch's key list
  const int64_t batch = blockIdx.x;
  const int64_t beg = offs[batch], end = offs[batch + 1];
  const int len = (int)(end - beg);
  const int nk = n_keysets_per_batch;
  const int total = len * nk;
  for (int i = threadIdx.x; i < pow2; i += 1024) {
    unsigned long long v = ~0ull;
    if (i < total) {
      const int k = i / len, j = i % len;
      const unsigned key = (unsigned)(keys[k * key_stride + beg + j] + key_add[k]);
      v = ((unsigned long long)key << 32) | (unsigned)i;
    }
    s[i] = v;
  }
  __syncthreads();
  for (int size = 2; size <= pow2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < pow2 / 2; i += 1024) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = ((lo & size) == 0);
        unsigned long long a = s[lo], b = s[hi];
        if ((a > b) == up) {
          s[lo] = b;
          s[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < pow2; i += 1024) out[batch * out_stride + i] = s[i];
}

}  // namespace

#define ROWS16(n) dim3(gmr::grid_for((n) * 16, 256)), dim3(256)

extern "C" int gmr_dmm_combine_fwd(int64_t n, float* G, const float* H, const float* Qi, const float* Qt,
                                   const float* mw, float lam, float* M, void* stream) {
  GMR_ARG(G && H && Qi && Qt && mw && M && n > 0, "bad args");
  hipLaunchKernelGGL(combine_fwd_kernel, ROWS16(n), 0, (hipStream_t)stream, n, G, H, Qi, Qt, mw, lam, M);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_final_fwd(int64_t n, const float* M, const float* L, float ris, float* Emb, float* nrm,
                                 void* stream) {
  GMR_ARG(M && L && Emb && nrm && n > 0, "bad args");
  hipLaunchKernelGGL(final_fwd_kernel, ROWS16(n), 0, (hipStream_t)stream, n, M, L, ris, Emb, nrm);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_cl_fwd(int64_t n, const float* Qi, const float* Qt, const float* K2, float* CLN, float* nrm,
                              void* stream) {
  GMR_ARG(Qi && Qt && K2 && CLN && nrm && n > 0, "bad args");
  hipLaunchKernelGGL(cl_fwd_kernel, dim3(gmr::grid_for(n * 32, 256)), dim3(256), 0, (hipStream_t)stream, n, Qi, Qt, K2,
                     CLN, nrm);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_normalize_rows_f32(int64_t n, int32_t cols, const float* x, int64_t ldx, float* y, int64_t ldy,
                                      float* nrm, void* stream) {
  GMR_ARG(x && y && n > 0 && cols > 0 && cols % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0, "bad args");
  hipLaunchKernelGGL(normalize_rows_kernel, ROWS16(n), 0, (hipStream_t)stream, n, cols, x, ldx, y, ldy, nrm);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_normalize_rows_bwd_f32(int64_t n, int32_t cols, const float* y, int64_t ldy, const float* nrm,
                                          const float* dy, int64_t lddy, float* dx, int64_t lddx, float slope,
                                          int32_t accumulate, void* stream) {
  GMR_ARG(y && nrm && dy && dx && n > 0 && cols % 4 == 0, "bad args");
  hipLaunchKernelGGL(normalize_bwd_kernel, ROWS16(n), 0, (hipStream_t)stream, n, cols, y, ldy, nrm, dy, lddy, dx, lddx,
                     slope, accumulate);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_bpr_fwd_bwd(int32_t B, int64_t U, const float* Emb, const int32_t* users, const int32_t* pos,
                               const int32_t* neg, float* loss, float* contrib, float inv_norm, void* stream) {
  GMR_ARG(Emb && users && pos && neg && loss && contrib && B > 0, "bad args");
  hipLaunchKernelGGL(bpr_kernel, ROWS16((int64_t)B), 0, (hipStream_t)stream, B, U, Emb, users, pos, neg, loss, contrib,
                     inv_norm);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_row_softmax_f32(int64_t rows, int64_t cols, float* L, int64_t ld, float coef, float* lse,
                                   void* stream) {
  GMR_ARG(L && lse && rows > 0 && cols > 0, "bad args");
  hipLaunchKernelGGL(row_softmax_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, rows, cols, L, ld, coef,
                     lse);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_contrast_rows(int32_t B, const float* CLN, const int32_t* nodes, int64_t node_off, const float* lse,
                                 float inv_temp, float coef, float* loss, float* contrib, int64_t ld_contrib,
                                 void* stream) {
  GMR_ARG(CLN && nodes && lse && loss && contrib && B > 0 && ld_contrib >= 128, "bad args");
  hipLaunchKernelGGL(contrast_rows_kernel, ROWS16((int64_t)B), 0, (hipStream_t)stream, B, CLN, nodes, node_off, lse,
                     inv_temp, coef, loss, contrib, ld_contrib);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_gather_rows_f32(int32_t B, int32_t cols, const float* src, int64_t lds, const int32_t* idx,
                                   int64_t off, float* out, int64_t ldo, void* stream) {
  GMR_ARG(src && idx && out && B > 0 && cols % 4 == 0, "bad args");
  hipLaunchKernelGGL(gather_rows_kernel, dim3(gmr::grid_for((int64_t)B * cols / 4, 256)), dim3(256), 0,
                     (hipStream_t)stream, B, cols, src, lds, idx, off, out, ldo);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_scatter_sorted_f32(int32_t n, int32_t cols, const uint64_t* plan, const float* contrib, int64_t ldc,
                                      float* dst, int64_t ldd, void* stream) {
  GMR_ARG(plan && contrib && dst && n > 0 && cols % 4 == 0, "bad args");
  hipLaunchKernelGGL(scatter_sorted_kernel, dim3(gmr::grid_for((int64_t)n * cols / 4, 256)), dim3(256), 0,
                     (hipStream_t)stream, n, cols, (const unsigned long long*)plan, contrib, ldc, dst, ldd);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_final_bwd(int64_t n, const float* dEmb, const float* T1, const float* M, const float* nrmM,
                                 float ris, const float* E, const float* mw, float* dE, float* partials,
                                 void* stream) {
  GMR_ARG(dEmb && T1 && M && nrmM && E && mw && dE && partials && n > 0, "bad args");
  hipLaunchKernelGGL(final_bwd_kernel, ROWS16(n), 0, (hipStream_t)stream, n, const_cast<float*>(dEmb), T1, M, nrmM,
                     ris, E, mw, dE, partials, 0, 0.f, nullptr, nullptr);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_final_bwd2(int64_t n, float* dEmb, const float* T1, const float* M, const float* nrmM, float ris,
                                  const float* E, const float* mw, float* dE, float* partials, int32_t clear, float lam,
                                  float* Ri, float* Rt, void* stream) {
  GMR_ARG(dEmb && T1 && M && nrmM && E && mw && dE && partials && n > 0 && (!Ri) == (!Rt), "bad args");
  hipLaunchKernelGGL(final_bwd_kernel, ROWS16(n), 0, (hipStream_t)stream, n, dEmb, T1, M, nrmM, ris, E, mw, dE,
                     partials, (int)clear, lam, Ri, Rt);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_bpr_sqnorm(int32_t B, int64_t U, const float* Emb, const int32_t* users, const int32_t* pos,
                                  const int32_t* neg, float* loss, float* contrib, float inv_norm, int64_t n_sq,
                                  const float* x, double* sq_parts, void* stream) {
  GMR_ARG(Emb && users && pos && neg && loss && contrib && x && sq_parts && B > 0 && n_sq >= 0, "bad args");
  const int nb = gmr::grid_for((int64_t)B * 16, 256);
  const int g = gmr::grid_for(n_sq, 256 * 8, GMR_SQNORM_PARTS);  // gmr_sqnorm_nparts(n_sq)
  hipLaunchKernelGGL(bpr_sqnorm_kernel, dim3((unsigned)(nb + g)), dim3(256), 0, (hipStream_t)stream, B, U, Emb, users,
                     pos, neg, loss, contrib, inv_norm, nb, n_sq, x, g, sq_parts);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_scatter_sorted_nbwd_f32(int32_t n, const uint64_t* plan, const float* contrib, int64_t ldc,
                                           const float* y, const float* nrm, int64_t n_nodes, float* dK, void* stream) {
  GMR_ARG(plan && contrib && y && nrm && dK && n > 0 && ldc >= 128 && ldc % 4 == 0, "bad args");
  hipLaunchKernelGGL(scatter_sorted_nbwd_kernel, dim3(gmr::grid_for((int64_t)n * 32, 256)), dim3(256), 0,
                     (hipStream_t)stream, n, (const unsigned long long*)plan, contrib, ldc, y, nrm, n_nodes, dK);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int64_t gmr_dmm_final_bwd_partials(int64_t n) { return 2 * (int64_t)gmr::grid_for(n * 16, 256); }

extern "C" int gmr_dmm_mw_grad(int64_t nparts, const float* partials, const float* mw, float* dmw, int32_t accumulate,
                               void* stream) {
  GMR_ARG(partials && mw && dmw, "bad args");
  hipLaunchKernelGGL(mw_grad_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, (int)nparts, partials, mw, dmw,
                     accumulate);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_dg(int64_t n, int64_t U, const float* dE, const float* T2, float* dG, void* stream) {
  GMR_ARG(dE && T2 && dG && n > 0, "bad args");
  hipLaunchKernelGGL(dg_kernel, dim3(gmr::grid_for(n * 32, 256)), dim3(256), 0, (hipStream_t)stream, n, U, dE, T2, dG);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_cl_bwd(int64_t n, const float* dK, const float* T, const float* dE, float lam, float* Ri,
                              float* Rt, void* stream) {
  GMR_ARG(dK && T && dE && Ri && Rt && n > 0, "bad args");
  hipLaunchKernelGGL(cl_bwd_kernel, ROWS16(n), 0, (hipStream_t)stream, n, const_cast<float*>(dK), T, dE, lam, Ri, Rt,
                     0, 1);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_cl_bwd2(int64_t n, float* dK, const float* T, const float* dE, float lam, float* Ri, float* Rt,
                               int32_t clear, int32_t left, void* stream) {
  GMR_ARG(dK && T && Ri && Rt && n > 0 && (!left || dE), "bad args");
  hipLaunchKernelGGL(cl_bwd_kernel, ROWS16(n), 0, (hipStream_t)stream, n, dK, T, dE, lam, Ri, Rt, (int)clear,
                     (int)left);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_assemble(int64_t n, int64_t U, const float* T2, const float* T3, const float* Ri,
                                const float* Rt, const float* E0, float reg2, float* dE0, float* dNF, void* stream) {
  GMR_ARG(T2 && T3 && Ri && Rt && E0 && dE0 && dNF && n > 0, "bad args");
  hipLaunchKernelGGL(assemble_kernel, ROWS16(n), 0, (hipStream_t)stream, n, U, T2, T3, Ri, Rt, E0, reg2, dE0, dNF,
                     nullptr, nullptr, 1.f, nullptr, 0);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_assemble2(int64_t n, int64_t U, const float* T2, const float* T3, const float* Ri,
                                 const float* Rt, const float* E0, float reg2, float* dE0, float* dNF, const float* NF,
                                 const float* nrmF, float slope, float* dK_clear, int32_t t3u_from_t2, void* stream) {
  GMR_ARG(T2 && T3 && Ri && Rt && E0 && dE0 && dNF && NF && nrmF && n > 0 && U >= 0 && U <= n, "bad args");
  hipLaunchKernelGGL(assemble_kernel, ROWS16(n), 0, (hipStream_t)stream, n, U, T2, T3, Ri, Rt, E0, reg2, dE0, dNF, NF,
                     nrmF, slope, dK_clear, (int)t3u_from_t2);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_sum_f32(int64_t n, const float* x, float scale, float* out, int32_t accumulate, void* stream) {
  GMR_ARG(x && out && n >= 0, "bad args");
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, n, x, scale, out, accumulate);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_sqnorm_f32(int64_t n, const float* x, float scale, float* out, int32_t accumulate,
                              double* workspace, void* stream) {
  GMR_ARG(x && out && workspace && n >= 0, "bad args");
  const int g = gmr::grid_for(n, 256 * 8, GMR_SQNORM_PARTS);
  hipLaunchKernelGGL(sqnorm_part_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, n, x, workspace);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(sqnorm_fin_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, g, workspace, scale, out,
                     accumulate);
  GMR_LAUNCHED();
  return GMR_OK;
}

// parts-only squared norm (the ordered final sum is done by gmr_dmm_loss_total)
extern "C" int64_t gmr_sqnorm_nparts(int64_t n) { return gmr::grid_for(n, 256 * 8, GMR_SQNORM_PARTS); }

extern "C" int gmr_sqnorm_part_f32(int64_t n, const float* x, double* workspace, void* stream) {
  GMR_ARG(x && workspace && n >= 0, "bad args");
  const int g = gmr::grid_for(n, 256 * 8, GMR_SQNORM_PARTS);
  hipLaunchKernelGGL(sqnorm_part_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, n, x, workspace);
  GMR_LAUNCHED();
  return GMR_OK;
}

namespace {
// the block-wide fp64 sum of sum_kernel / sqnorm_fin_kernel, as a device function (same order)
template <typename T>
__device__ double block_sum_d(int64_t n, const T* __restrict__ x, double* red) {
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += (double)x[i];
  s = gmr::wave_sum_d(s);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// loss = sum(bpr)/nr + reg * |E0|^2 + ssl/nr * (sum(cu) + sum(ci)), in the order of the four
// separate reductions it replaces (sum, sqnorm fin, sum, sum): the same float value
__global__ void __launch_bounds__(256) loss_total_kernel(int64_t B, const float* __restrict__ bpr, float inv_nr,
                                                         const double* __restrict__ parts, int nparts, float reg,
                                                         const float* __restrict__ cu, const float* __restrict__ ci,
                                                         float ssl, float* __restrict__ out) {
  __shared__ double red[4];
  const double a = block_sum_d(B, bpr, red);
  const double b = block_sum_d((int64_t)nparts, parts, red);
  const double c = block_sum_d(B, cu, red);
  const double d = block_sum_d(B, ci, red);
  if (threadIdx.x == 0) {
    float v = (float)(a * (double)inv_nr);
    v = v + (float)(b * (double)reg);
    v = v + (float)(c * (double)ssl);
    v = v + (float)(d * (double)ssl);
    out[0] = v;
  }
}

// block 0: loss_total_kernel's sum (and acc[0] += loss when acc is given: the trainer's epoch loss, the bits of
// its gmr_sum_f32 call); block 1: mw_grad_kernel (the modal-weight gradient from final_bwd's partials)
__global__ void __launch_bounds__(256) loss_mw_kernel(int64_t B, const float* __restrict__ bpr, float inv_nr,
                                                      const double* __restrict__ parts, int nparts, float reg,
                                                      const float* __restrict__ cu, const float* __restrict__ ci,
                                                      float ssl, float* __restrict__ out, float* __restrict__ acc,
                                                      int nmw, const float* __restrict__ mwpart,
                                                      const float* __restrict__ mw, float* __restrict__ dmw) {
  if (blockIdx.x == 1) {
    mw_grad_block(nmw, mwpart, mw, dmw, 0);
    return;
  }
  __shared__ double red[4];
  const double a = block_sum_d(B, bpr, red);
  const double b = block_sum_d((int64_t)nparts, parts, red);
  const double c = block_sum_d(B, cu, red);
  const double d = block_sum_d(B, ci, red);
  if (threadIdx.x == 0) {
    float v = (float)(a * (double)inv_nr);
    v = v + (float)(b * (double)reg);
    v = v + (float)(c * (double)ssl);
    v = v + (float)(d * (double)ssl);
    out[0] = v;
    if (acc) acc[0] = acc[0] + v;
  }
}
}  // namespace

extern "C" int gmr_dmm_loss_mw(int64_t B, const float* loss_bpr, float inv_nr, const double* parts, int64_t nparts,
                               float reg_scale, const float* loss_cu, const float* loss_ci, float ssl_scale, float* out,
                               float* acc, int64_t n_mw_parts, const float* mw_parts, const float* mw, float* dmw,
                               void* stream) {
  GMR_ARG(loss_bpr && parts && loss_cu && loss_ci && out && mw_parts && mw && dmw && B > 0 && nparts > 0 &&
              nparts < (1 << 30) && n_mw_parts > 0 && n_mw_parts < (1 << 30),
          "bad args");
  hipLaunchKernelGGL(loss_mw_kernel, dim3(2), dim3(256), 0, (hipStream_t)stream, B, loss_bpr, inv_nr, parts,
                     (int)nparts, reg_scale, loss_cu, loss_ci, ssl_scale, out, acc, (int)n_mw_parts, mw_parts, mw, dmw);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dmm_loss_total(int64_t B, const float* loss_bpr, float inv_nr, const double* parts, int64_t nparts,
                                  float reg_scale, const float* loss_cu, const float* loss_ci, float ssl_scale,
                                  float* out, void* stream) {
  GMR_ARG(loss_bpr && parts && loss_cu && loss_ci && out && B > 0 && nparts > 0 && nparts < (1 << 30), "bad args");
  hipLaunchKernelGGL(loss_total_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, B, loss_bpr, inv_nr, parts,
                     (int)nparts, reg_scale, loss_cu, loss_ci, ssl_scale, out);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_sort_batch_keys(int64_t n_batches, const int32_t* keys, const int64_t* offsets,
                                   const int32_t* key_add, int32_t n_keysets, int64_t key_stride, uint64_t* out,
                                   int64_t out_stride, int32_t pow2, void* stream) {
  GMR_ARG(keys && offsets && key_add && out && n_batches > 0, "bad args");
  GMR_ARG(pow2 >= 2 && pow2 <= 8192 && (pow2 & (pow2 - 1)) == 0, "pow2 must be a power of two <= 8192");
  hipLaunchKernelGGL(sort_keys_kernel, dim3((unsigned)n_batches), dim3(1024), 0, (hipStream_t)stream, keys, offsets,
                     key_add, n_keysets, key_stride, (unsigned long long*)out, out_stride, pow2);
  GMR_LAUNCHED();
  return GMR_OK;
}

namespace {
__global__ void sum_f64_kernel(int64_t n, const double* __restrict__ x, double scale, double* __restrict__ out,
                               int accumulate) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += x[i];
  s = gmr::wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double v = ((red[0] + red[1]) + (red[2] + red[3])) * scale;
    out[0] = accumulate ? out[0] + v : v;
  }
}
}  // namespace

extern "C" int gmr_sum_f64(int64_t n, const double* x, double scale, double* out, int32_t accumulate, void* stream) {
  GMR_ARG(x && out && n >= 0, "bad args");
  hipLaunchKernelGGL(sum_f64_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, n, x, scale, out, accumulate);
  GMR_LAUNCHED();
  return GMR_OK;
}

// ============================================================================ K8 fused InfoNCE
// contrastLoss (models/diffmm.py:251-258) forward + backward without the B x n logit matrix.
// P = gathered view-1 rows (B x 64, ldp), T = view-2 table (n x 64, ldt), t = 1/temp, k = coef t:
//   E_ij = exp(t <P_i, T_j>),   z_i = sum_j E_ij,   loss_i = log z_i - t <P_i, T_node(i)>
//   dP_i = k (sum_j E_ij T_j / z_i - T_node(i)),    dT_j = k sum_i (E_ij / z_i) P_i
// (the -k P_i term of table row node(i) goes through the sorted scatter with the sparse terms).
// Rows pass: a wave owns 32 rows i, the workgroup's 4 waves share 32-row blocks of T staged in
// LDS.  S^T = T_blk P^T runs on the f32 matrix cores (v_mfma_f32_32x32x2_f32; k order
// d = 32u + 16h + s so both fragments are float4 reads), E = exp in registers, then
// U^T += T_blk^T E^T takes the exp'd accumulator itself as the B operand: its rows j sit in the
// registers, so MFMA step e pairs with j = (e&3) + 8(e>>2) + 4h and only T[j][d] is read (LDS).
// The grid splits j into chunks; the finalise pass adds the per-chunk (U_i, z_i) in chunk order.
// Table pass: the same with the roles swapped (a wave owns 32 table rows, the workgroup shares
// blocks of P and r_i = k / z_i); per-row-chunk partials of dT are added in chunk order.
// Every sum has a fixed order: deterministic.
namespace {

constexpr int kClLd = 68;  // LDS row stride of a staged 32 x 64 block (floats): conflict-free b128 rows
typedef float clx16 __attribute__((ext_vector_type(16)));

// two float4 per thread stage a 32 x 64 block: rows r0 .. r0 + 31 of src, zero at and past r_end
__device__ __forceinline__ void cl_load(float4 (&st)[2], const float* __restrict__ src, int64_t ld, int r0,
                                        int r_end) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int idx = threadIdx.x + 256 * q, r = idx >> 4, c4 = (idx & 15) * 4;
    st[q] = r0 + r < r_end ? ld4(src + (int64_t)(r0 + r) * ld + c4) : f4(0.f, 0.f, 0.f, 0.f);
  }
}
// the same with row r of the block read from src row idx[r0 + r] + off (a gathered operand, read in place)
__device__ __forceinline__ void cl_load_idx(float4 (&st)[2], const float* __restrict__ src, int64_t ld, int r0,
                                            int r_end, const int* __restrict__ idx, int64_t off) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int id = threadIdx.x + 256 * q, r = id >> 4, c4 = (id & 15) * 4;
    st[q] = r0 + r < r_end ? ld4(src + ((int64_t)idx[r0 + r] + off) * ld + c4) : f4(0.f, 0.f, 0.f, 0.f);
  }
}
__device__ __forceinline__ void cl_store(const float4 (&st)[2], float* dst) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int idx = threadIdx.x + 256 * q;
    st4(dst + (idx >> 4) * kClLd + (idx & 15) * 4, st[q]);
  }
}
// the lane's A operands of cl_acc, read from LDS ahead of the exp phase (issued together, so the
// MFMA chain of cl_acc does not wait on one LDS round trip per step)
__device__ __forceinline__ void cl_acc_load(const float* blk, float (&a0)[16], float (&a1)[16], int l32, int h) {
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int r = (e & 3) + 8 * (e >> 2) + 4 * h;
    a0[e] = blk[r * kClLd + l32];
    a1[e] = blk[r * kClLd + 32 + l32];
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the reads here: hipcc otherwise sinks each next to its MFMA
}
// y^T (64 x 32) += blk^T (64 x 32) X, X (32 x 32) in the accumulator registers (row (e&3)+8(e>>2)+4h)
// NF fragments against one staged block: each A read from LDS feeds NF independent MFMA chains
template <int NF>
__device__ __forceinline__ void cl_dot_n(clx16 (&s)[NF], const float* blk, const float4 (&fr)[NF][2][4], int l32,
                                         int h) {
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int e = 0; e < 16; ++e) s[f][e] = 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 a = ld4(blk + l32 * kClLd + 32 * u + 16 * h + 4 * q);
#pragma unroll
      for (int f = 0; f < NF; ++f) s[f] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, fr[f][u][q].x, s[f], 0, 0, 0);
#pragma unroll
      for (int f = 0; f < NF; ++f) s[f] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, fr[f][u][q].y, s[f], 0, 0, 0);
#pragma unroll
      for (int f = 0; f < NF; ++f) s[f] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, fr[f][u][q].z, s[f], 0, 0, 0);
#pragma unroll
      for (int f = 0; f < NF; ++f) s[f] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, fr[f][u][q].w, s[f], 0, 0, 0);
    }
}
template <int NF>
__device__ __forceinline__ void cl_acc_n(const float (&a0)[16], const float (&a1)[16], const clx16 (&X)[NF],
                                         clx16 (&y0)[NF], clx16 (&y1)[NF]) {
#pragma unroll
  for (int e = 0; e < 16; ++e)
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      y0[f] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], X[f][e], y0[f], 0, 0, 0);
      y1[f] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], X[f][e], y1[f], 0, 0, 0);
    }
}
// the lane's 64-float column of y^T: registers 4g .. 4g+3 hold d = 8g + 4h + 0..3 (+32 in y1)
__device__ __forceinline__ void cl_put(float* dst, const clx16& y0, const clx16& y1, int h) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    st4(dst + 8 * g + 4 * h, f4(y0[4 * g], y0[4 * g + 1], y0[4 * g + 2], y0[4 * g + 3]));
    st4(dst + 32 + 8 * g + 4 * h, f4(y1[4 * g], y1[4 * g + 1], y1[4 * g + 2], y1[4 * g + 3]));
  }
}
__device__ __forceinline__ void cl_frag(float4 (&fr)[2][4], const float* __restrict__ src, int64_t ld, int row,
                                        int n_rows, int h) {
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      fr[u][q] = row < n_rows ? ld4(src + (int64_t)row * ld + 32 * u + 16 * h + 4 * q) : f4(0.f, 0.f, 0.f, 0.f);
}

// exp(t x) on the transcendental unit: v_exp_f32 of x * (t log2 e) (relative error ~ |t x| 2^-24
// from rounding the product, 6e-7 at |t x| <= 10) instead of the range-reduced expf (~14 VALU ops)
template <bool FAST>
__device__ __forceinline__ float cl_exp(float inv_t, float x) {
  if (FAST) return __builtin_amdgcn_exp2f(x * (inv_t * 1.4426950408889634f));
  return expf(inv_t * x);
}

template <bool FAST, int NF>
__global__ void __launch_bounds__(256, 2) cl_rows_kernel(int B, int n, const float* __restrict__ P, int64_t ldp,
                                                      const float* __restrict__ T, int64_t ldt, float inv_t, int chunk,
                                                      float* __restrict__ part_u, float* __restrict__ part_z) {
  __shared__ __attribute__((aligned(16))) float s_blk[2][32 * kClLd];
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  // the lane's rows (columns of S^T): NF fragments of 32 rows per wave
  const int i0r = blockIdx.x * 128 * NF + (threadIdx.x >> 6) * 32 * NF + l32;
  const int c = blockIdx.y, j0 = c * chunk, j1 = min(n, j0 + chunk);
  float4 fr[NF][2][4];
#pragma unroll
  for (int f = 0; f < NF; ++f) cl_frag(fr[f], P, ldp, i0r + 32 * f, B, h);
  clx16 y0[NF], y1[NF];
  float z[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    z[f] = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) y0[f][e] = y1[f][e] = 0.f;
  }
  float4 st[2];
  cl_load(st, T, ldt, j0, j1);
  cl_store(st, s_blk[0]);
  __syncthreads();
  int cur = 0;
  for (int j = j0; j < j1; j += 32) {
    const bool more = j + 32 < j1;
    if (more) cl_load(st, T, ldt, j + 32, j1);
    const float* blk = s_blk[cur];
    clx16 s[NF];
    cl_dot_n<NF>(s, blk, fr, l32, h);
    float a0[16], a1[16];
    cl_acc_load(blk, a0, a1, l32, h);
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int r = (e & 3) + 8 * (e >> 2) + 4 * h;
        s[f][e] = j + r < j1 ? cl_exp<FAST>(inv_t, s[f][e]) : 0.f;
        z[f] += s[f][e];
      }
    cl_acc_n<NF>(a0, a1, s, y0, y1);
    if (more) cl_store(st, s_blk[cur ^ 1]);
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int i = i0r + 32 * f;
    const float zf = z[f] + __shfl_xor(z[f], 32);
    if (i < B) {
      cl_put(part_u + ((int64_t)c * B + i) * 64, y0[f], y1[f], h);
      if (h == 0) part_z[(int64_t)c * B + i] = zf;
    }
  }
}

// one wave per row i, lane = d: chunk partials in order, loss, dense dP row, r_i = k / z_i
__global__ void __launch_bounds__(256) cl_finalize_kernel(int B, int nc, const float* __restrict__ part_u,
                                                          const float* __restrict__ part_z, const float* __restrict__ CLN,
                                                          const int* __restrict__ nodes, int64_t node_off, float inv_t,
                                                          float coef, float* __restrict__ loss,
                                                          float* __restrict__ contrib, int64_t ld_contrib,
                                                          float* __restrict__ r_out) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), d = threadIdx.x & 63;
  if (i >= B) return;
  float u = 0.f, z = 0.f;
  int c = 0;
  for (; c + 8 <= nc; c += 8) {  // eight chunk partials in flight, summed in chunk order
    float uu[8], zz[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      uu[q] = part_u[((int64_t)(c + q) * B + i) * 64 + d];
      zz[q] = part_z[(int64_t)(c + q) * B + i];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      u += uu[q];
      z += zz[q];
    }
  }
  for (; c < nc; ++c) {
    u += part_u[((int64_t)c * B + i) * 64 + d];
    z += part_z[(int64_t)c * B + i];
  }
  const int64_t t = node_off + nodes[i];
  const float p1 = CLN[t * 128 + d], p2 = CLN[t * 128 + 64 + d];
  const float dot = gmr::wave_sum(p1 * p2);
  const float k = coef * inv_t;
  float* o = contrib + (int64_t)i * ld_contrib;
  o[d] = k * (u / z - p2);
  o[64 + d] = -k * p1;
  if (d == 0) {
    loss[i] = logf(z) - dot * inv_t;
    r_out[i] = k / z;
  }
}

template <bool FAST, int NF>
__global__ void __launch_bounds__(256, 2) cl_table_kernel(int B, int n, const float* __restrict__ P, int64_t ldp,
                                                       const float* __restrict__ r, const float* __restrict__ T,
                                                       int64_t ldt, float inv_t, int chunk, float* __restrict__ part_t) {
  __shared__ __attribute__((aligned(16))) float s_blk[2][32 * kClLd];
  __shared__ float s_r[2][32];
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int j0r = blockIdx.x * 128 * NF + (threadIdx.x >> 6) * 32 * NF + l32;  // the lane's table rows
  const int c = blockIdx.y, i0 = c * chunk, i1 = min(B, i0 + chunk);
  float4 fr[NF][2][4];
#pragma unroll
  for (int f = 0; f < NF; ++f) cl_frag(fr[f], T, ldt, j0r + 32 * f, n, h);
  clx16 y0[NF], y1[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int e = 0; e < 16; ++e) y0[f][e] = y1[f][e] = 0.f;
  float4 st[2];
  float sr = 0.f;
  cl_load(st, P, ldp, i0, i1);
  if (threadIdx.x < 32) sr = i0 + (int)threadIdx.x < i1 ? r[i0 + threadIdx.x] : 0.f;
  cl_store(st, s_blk[0]);
  if (threadIdx.x < 32) s_r[0][threadIdx.x] = sr;
  __syncthreads();
  int cur = 0;
  for (int i = i0; i < i1; i += 32) {
    const bool more = i + 32 < i1;
    if (more) {
      cl_load(st, P, ldp, i + 32, i1);
      if (threadIdx.x < 32) sr = i + 32 + (int)threadIdx.x < i1 ? r[i + 32 + threadIdx.x] : 0.f;
    }
    const float* blk = s_blk[cur];
    clx16 s[NF];
    cl_dot_n<NF>(s, blk, fr, l32, h);  // S' (rows i of the block x the wave's table rows)
    float a0[16], a1[16];
    cl_acc_load(blk, a0, a1, l32, h);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float re = s_r[cur][(e & 3) + 8 * (e >> 2) + 4 * h];
#pragma unroll
      for (int f = 0; f < NF; ++f) s[f][e] = re * cl_exp<FAST>(inv_t, s[f][e]);
    }
    cl_acc_n<NF>(a0, a1, s, y0, y1);  // dT^T += P_blk^T (r E)
    if (more) {
      cl_store(st, s_blk[cur ^ 1]);
      if (threadIdx.x < 32) s_r[cur ^ 1][threadIdx.x] = sr;
    }
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int j = j0r + 32 * f;
    if (j < n) cl_put(part_t + ((int64_t)c * n + j) * 64, y0[f], y1[f], h);
  }
}

__global__ void cl_table_reduce_kernel(int n, int nc, const float* __restrict__ part_t, float* __restrict__ dT,
                                       int64_t ld) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)n * 16) return;
  const int64_t j = g >> 4;
  const int c4 = (int)(g & 15) * 4;
  float4 s = ld4(part_t + j * 64 + c4);
  int c = 1;
  for (; c + 4 <= nc; c += 4) {  // four chunk partials in flight, summed in chunk order
    float4 t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = ld4(part_t + ((int64_t)(c + q) * n + j) * 64 + c4);
#pragma unroll
    for (int q = 0; q < 4; ++q) s = gmr::f4_add(s, t[q]);
  }
  for (; c < nc; ++c) s = gmr::f4_add(s, ld4(part_t + ((int64_t)c * n + j) * 64 + c4));
  st4(dT + j * ld + c4, s);
}

// the same sums, stored through the normalize backward of the table's view (y = normalised rows, ldy; nrm):
// dT = nbwd(sum of the chunk partials) (DiffMM: the dense part of the text view's gradient, dK[:, 64:])
__global__ void cl_table_reduce_nbwd_kernel(int n, int nc, const float* __restrict__ part_t, float* __restrict__ dT,
                                            int64_t ld, const float* __restrict__ y, int64_t ldy,
                                            const float* __restrict__ nrm) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)n * 16) return;  // (whole 16-lane rows)
  const int64_t j = g >> 4;
  const int c4 = (int)(g & 15) * 4;
  float4 s = ld4(part_t + j * 64 + c4);
  int c = 1;
  for (; c + 4 <= nc; c += 4) {
    float4 t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = ld4(part_t + ((int64_t)(c + q) * n + j) * 64 + c4);
#pragma unroll
    for (int q = 0; q < 4; ++q) s = gmr::f4_add(s, t[q]);
  }
  for (; c < nc; ++c) s = gmr::f4_add(s, ld4(part_t + ((int64_t)c * n + j) * 64 + c4));
  st4(dT + j * ld + c4, nbwd_leaky(s, ld4(y + j * ldy + c4), nrm[j], 1.f));
}

// ---------------------------------------------------------------------------------------------
// The same two passes on the bf16 matrix cores (GMR_CL_X6, default): every fp32 operand is split
// exactly into three bf16 terms (hi + mid + lo, as gemm_x6.hip) and each 32 x 32 x 16 logits product is
// accumulated in fp32 from six v_mfma_f32_32x32x16_bf16 (hi.hi + hi.mid + mid.hi + hi.lo + lo.hi +
// mid.mid; the dropped terms are below 2^-23 |ab|), so S and E keep fp32 accuracy at 6 x 32 cycles
// per 32 x 32 x 16 block instead of 8 x 64 on v_mfma_f32_32x32x2_f32; the gradient-only products U = E T take
// three (c6_mfma3, round 6).
// Per staged 32-row block the workgroup converts the fp32 rows once into LDS as three row-major bf16
// planes [32 rows][64 d] (A operand of S^T = Stg F^T) and three transposed planes [64 d][32 slots]
// (A operand of Y^T += Stg^T E^T), slots permuted so that the 8 staged rows a lane half feeds to one
// K-step of the second product are contiguous: a K position pairs the exp'd accumulator register
// e = 8 t + q (staged row (q & 3) + 8 (q >> 2) + 16 t + 4 h) with the same staged row of Stg^T.
// The fragment rows (queries, or table rows in the table pass) are split once into registers.
typedef __bf16 c6bf8 __attribute__((ext_vector_type(8)));
constexpr int kC6A = 72;                              // bf16 row stride, row-major planes (conflict-free b128)
constexpr int kC6B = 40;                              // bf16 row stride, transposed planes
constexpr int kC6PA = 32 * kC6A, kC6PB = 64 * kC6B;   // bf16 elements per plane
constexpr int kC6Stage = 3 * (kC6PA + kC6PB);         // bf16 elements per staged block

__device__ __forceinline__ void c6_split8(const float (&v)[8], c6bf8 (&o)[3]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 hh = (__bf16)__builtin_amdgcn_fmed3f(v[e], -0x1.fep127f, 0x1.fep127f);
    const float r1 = v[e] - (float)hh;  // exact
    const __bf16 mm = (__bf16)r1;
    o[0][e] = hh;
    o[1][e] = mm;
    o[2][e] = (__bf16)(r1 - (float)mm);  // exact
  }
}

// Y products (E T over the staged block) keep three of the six: hi*hi + hi*mid + mid*hi.  The dropped terms are
// each <= 2^-18 |e t| (round-to-nearest splits: |mid| <= 2^-9 |x|, |lo| <= 2^-18 |x|), so a Y row is fp32-grade
// (<= 1.2e-5 of sum |e t| worst case) for the gradients it feeds (dP, dT: the parity tests' 1e-4 bars); the
// logits S, which feed exp and the loss rows (1e-5), keep all six (round 6: 48 -> 36 MFMAs per staged block)
__device__ __forceinline__ void c6_split8_2(const float (&v)[8], c6bf8 (&o)[2]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 hh = (__bf16)__builtin_amdgcn_fmed3f(v[e], -0x1.fep127f, 0x1.fep127f);
    o[0][e] = hh;
    o[1][e] = (__bf16)(v[e] - (float)hh);
  }
}
// fp32 block (32 x 64, stride kClLd) -> the three row-major and the three transposed bf16 planes
__device__ __forceinline__ void c6_convert(const float* sf, __bf16* stg) {
  const int t = threadIdx.x;
  {  // row-major: thread -> row t / 8, columns 8 c' .. + 8 with c' = t % 8 rotated by -1 in rows 4 i + 2, 4 i + 3
     // (conflict-free 16-byte reads of s_f and writes of the planes; plain t % 8 cost 2-way on the reads)
    const int r = t >> 3, c = (((t & 7) + ((r & 2) ? 7 : 0)) & 7) * 8;
    const float4 a = ld4(sf + r * kClLd + c), b = ld4(sf + r * kClLd + c + 4);
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    c6bf8 o[3];
    c6_split8(v, o);
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<c6bf8*>(stg + p * kC6PA + r * kC6A + c) = o[p];
  }
  {  // transposed: thread -> column d = t % 64, slot group g = t / 64 (slots 8 g .. 8 g + 7): a wave reads 64
     // consecutive floats of one staged row per load and its 16-byte stores land on distinct banks (the
     // (t / 4, t % 4) mapping cost 2-way conflicts on both, ~17 % of the pass's LDS cycles: profiles/r05zy_*)
    const int d = t & 63, g = t >> 6;
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = sf[(16 * (g >> 1) + 4 * (g & 1) + (q & 3) + 8 * (q >> 2)) * kClLd + d];
    c6bf8 o[2];  // the Y products read the hi and mid planes only (c6_mfma3)
    c6_split8_2(v, o);
#pragma unroll
    for (int p = 0; p < 2; ++p) *reinterpret_cast<c6bf8*>(stg + 3 * kC6PA + p * kC6PB + d * kC6B + 8 * g) = o[p];
  }
}

__device__ __forceinline__ clx16 c6_mfma3(const c6bf8 (&a)[2], const c6bf8 (&b)[2], clx16 c) {  // small terms first
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
}

__device__ __forceinline__ clx16 c6_mfma6(const c6bf8 (&a)[3], const c6bf8 (&b)[3], clx16 c) {  // small terms first
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
}

// In-launch reduction of the table pass (replaces cl_table_reduce_kernel): each i-chunk block of a
// 128-row table tile stores its partial, publishes it (agent-scope release) and counts itself in the
// tile's counter; the block that arrives last (acquire) sums the tile's partials in chunk order c = 0,
// 1, ... (cl_table_reduce_kernel's order: same bits) into dT and resets the counter for the next call.
constexpr int kClCounters = 8192;  // counter words leading the contrast workspace (tables <= 1M rows)
__device__ __forceinline__ void cl_table_fixup(int* cnt, const float* __restrict__ part, int n, float* __restrict__ dT,
                                               int64_t ld) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (int)gridDim.y - 1;
    if (last) {
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  const int nc = (int)gridDim.y;
  const int64_t j0 = (int64_t)blockIdx.x * 128;
  for (int g = threadIdx.x; g < 128 * 16; g += blockDim.x) {
    const int64_t j = j0 + (g >> 4);
    if (j >= n) continue;
    const int c4 = (g & 15) * 4;
    float4 a = ld4(part + j * 64 + c4);
    int c = 1;
    for (; c + 8 <= nc; c += 8) {  // eight chunk partials in flight (they come from other XCDs' L2s), summed in order
      float4 t[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) t[q] = ld4(part + ((int64_t)(c + q) * n + j) * 64 + c4);
#pragma unroll
      for (int q = 0; q < 8; ++q) a = gmr::f4_add(a, t[q]);
    }
    for (; c < nc; ++c) a = gmr::f4_add(a, ld4(part + ((int64_t)c * n + j) * 64 + c4));
    st4(dT + j * ld + c4, a);
  }
}

// TABLE = false (rows pass): F = P (queries), Stg = T (keys), part_y / part_z per query chunk;
// TABLE = true (table pass): F = T rows, Stg = P rows weighted by w = r_i, part_y = dT partials
template <bool FAST, bool TABLE>
__global__ void __launch_bounds__(256, 2) cl6_kernel(int nf, int ns, const float* __restrict__ F, int64_t ldf,
                                                     const float* __restrict__ Stg, int64_t lds,
                                                     const float* __restrict__ w, float inv_t, int chunk,
                                                     float* __restrict__ part_y, float* __restrict__ part_z,
                                                     int* __restrict__ cnt, float* __restrict__ dT, int64_t ld_dt) {
  __shared__ __attribute__((aligned(16))) __bf16 s_stg[2 * kC6Stage];
  __shared__ __attribute__((aligned(16))) float s_f[32 * kClLd];
  __shared__ float s_w[2][32];
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int f = blockIdx.x * 128 + (threadIdx.x >> 6) * 32 + l32;  // the lane's fragment row
  const int c = blockIdx.y, s0 = c * chunk, s1 = min(ns, s0 + chunk);
  c6bf8 fr[4][3];  // K-step k: d = 16 k + 8 h + 0..7
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float4 a = f4(0.f, 0.f, 0.f, 0.f), b = a;
    if (f < nf) {
      a = ld4(F + (int64_t)f * ldf + 16 * k + 8 * h);
      b = ld4(F + (int64_t)f * ldf + 16 * k + 8 * h + 4);
    }
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    c6_split8(v, fr[k]);
  }
  clx16 y0, y1;
#pragma unroll
  for (int e = 0; e < 16; ++e) y0[e] = y1[e] = 0.f;
  float z = 0.f, sw = 0.f;
  float4 st[2];
  cl_load(st, Stg, lds, s0, s1);
  if (TABLE && threadIdx.x < 32) sw = s0 + (int)threadIdx.x < s1 ? w[s0 + threadIdx.x] : 0.f;
  cl_store(st, s_f);
  __syncthreads();
  c6_convert(s_f, s_stg);
  if (TABLE && threadIdx.x < 32) s_w[0][threadIdx.x] = sw;
  __syncthreads();
  int cur = 0;
  for (int j = s0; j < s1; j += 32) {
    const bool more = j + 32 < s1;
    if (more) {
      cl_load(st, Stg, lds, j + 32, s1);
      if (TABLE && threadIdx.x < 32) sw = j + 32 + (int)threadIdx.x < s1 ? w[j + 32 + threadIdx.x] : 0.f;
    }
    const __bf16* A = s_stg + cur * kC6Stage;
    clx16 sacc;  // S^T: row = staged row (e & 3) + 8 (e >> 2) + 4 h, column = fragment row l32
#pragma unroll
    for (int e = 0; e < 16; ++e) sacc[e] = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c6bf8 a[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const c6bf8*>(A + p * kC6PA + l32 * kC6A + 16 * k + 8 * h);
      sacc = c6_mfma6(a, fr[k], sacc);
    }
    float ev[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int r = (e & 3) + 8 * (e >> 2) + 4 * h;
      const float x = j + r < s1 ? cl_exp<FAST>(inv_t, sacc[e]) : 0.f;
      if (TABLE) {
        ev[e] = s_w[cur][r] * x;
      } else {
        ev[e] = x;
        z += x;
      }
    }
    const __bf16* Bt = A + 3 * kC6PA;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {  // Y^T (64 d x 32) += Stg^T E^T, K = 32 staged rows in two steps
      const float evs[8] = {ev[8 * t2], ev[8 * t2 + 1], ev[8 * t2 + 2], ev[8 * t2 + 3],
                            ev[8 * t2 + 4], ev[8 * t2 + 5], ev[8 * t2 + 6], ev[8 * t2 + 7]};
      c6bf8 eb[2], a0[2], a1[2];
      c6_split8_2(evs, eb);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        a0[p] = *reinterpret_cast<const c6bf8*>(Bt + p * kC6PB + l32 * kC6B + 8 * (2 * t2 + h));
        a1[p] = *reinterpret_cast<const c6bf8*>(Bt + p * kC6PB + (32 + l32) * kC6B + 8 * (2 * t2 + h));
      }
      y0 = c6_mfma3(a0, eb, y0);
      y1 = c6_mfma3(a1, eb, y1);
    }
    if (more) {  // s_f's last reader (the convert) finished before the previous barrier
      cl_store(st, s_f);
      __syncthreads();
      c6_convert(s_f, s_stg + (cur ^ 1) * kC6Stage);
      if (TABLE && threadIdx.x < 32) s_w[cur ^ 1][threadIdx.x] = sw;
    }
    __syncthreads();
    cur ^= 1;
  }
  if (f < nf) cl_put(part_y + ((int64_t)c * nf + f) * 64, y0, y1, h);
  if (!TABLE) {
    const float zf = z + __shfl_xor(z, 32);
    if (f < nf && h == 0) part_z[(int64_t)c * nf + f] = zf;
  }
  if (TABLE && cnt) cl_table_fixup(cnt + blockIdx.x, part_y, nf, dT, ld_dt);
}

// The same pass with the S product of block j + 1 issued before the exp / split phase of block j (PIPE,
// GMR_CL_PIPE, default): the matrix pipe runs the next S while the vector pipe exponentiates and splits
// this block's logits, instead of each wave alternating MFMA-only and VALU-only phases.  Both staged
// blocks are in LDS by then (block j + 2 is staged into block j's buffer after its Y product), so the
// staging, the chunking and every sum are those of cl6_kernel: bit-identical results.
// gidx (optional): the batch operand is read in place through the node index - the fragment rows F[gidx[f] +
// goff] in the rows pass (!TABLE), the staged rows Stg[gidx[j] + goff] in the table pass - instead of from a
// gathered copy (round 6: the two gather launches of the rec step; the same values, bit-identical sums)
template <bool FAST, bool TABLE>
__global__ void __launch_bounds__(256, 2) cl6p_kernel(int nf, int ns, const float* __restrict__ F, int64_t ldf,
                                                      const float* __restrict__ Stg, int64_t lds,
                                                      const float* __restrict__ w, float inv_t, int chunk,
                                                      float* __restrict__ part_y, float* __restrict__ part_z,
                                                      int* __restrict__ cnt, float* __restrict__ dT, int64_t ld_dt,
                                                      const int* __restrict__ gidx, int64_t goff) {
  __shared__ __attribute__((aligned(16))) __bf16 s_stg[2 * kC6Stage];
  __shared__ __attribute__((aligned(16))) float s_f[32 * kClLd];
  __shared__ float s_w[2][32];
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int f = blockIdx.x * 128 + (threadIdx.x >> 6) * 32 + l32;  // the lane's fragment row
  const int c = blockIdx.y, s0 = c * chunk, s1 = min(ns, s0 + chunk);
  c6bf8 fr[4][3];  // K-step k: d = 16 k + 8 h + 0..7
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float4 a = f4(0.f, 0.f, 0.f, 0.f), b = a;
    if (f < nf) {
      const int64_t fr_row = !TABLE && gidx ? (int64_t)gidx[f] + goff : (int64_t)f;
      a = ld4(F + fr_row * ldf + 16 * k + 8 * h);
      b = ld4(F + fr_row * ldf + 16 * k + 8 * h + 4);
    }
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    c6_split8(v, fr[k]);
  }
  auto sprod = [&](const __bf16* A) {  // S^T of a staged block
    clx16 sacc;
#pragma unroll
    for (int e = 0; e < 16; ++e) sacc[e] = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c6bf8 a[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const c6bf8*>(A + p * kC6PA + l32 * kC6A + 16 * k + 8 * h);
      sacc = c6_mfma6(a, fr[k], sacc);
    }
    return sacc;
  };
  auto stage = [&](int j, int buf) {  // block starting at row j -> s_stg[buf] (and its weights), two barriers
    float4 st[2];
    float sw = 0.f;
    if (TABLE && gidx)
      cl_load_idx(st, Stg, lds, j, s1, gidx, goff);
    else
      cl_load(st, Stg, lds, j, s1);
    if (TABLE && threadIdx.x < 32) sw = j + (int)threadIdx.x < s1 ? w[j + threadIdx.x] : 0.f;
    cl_store(st, s_f);
    __syncthreads();
    c6_convert(s_f, s_stg + buf * kC6Stage);
    if (TABLE && threadIdx.x < 32) s_w[buf][threadIdx.x] = sw;
    __syncthreads();
  };
  clx16 y0, y1;
#pragma unroll
  for (int e = 0; e < 16; ++e) y0[e] = y1[e] = 0.f;
  float z = 0.f;
  stage(s0, 0);
  if (s0 + 32 < s1) stage(s0 + 32, 1);
  clx16 scur = sprod(s_stg);
  int cur = 0;
  float4 st[2];
  float sw = 0.f;
  for (int j = s0; j < s1; j += 32) {
    const bool more = j + 32 < s1, refill = j + 64 < s1;
    if (refill) {  // block j + 2's rows travel while this block is computed
      if (TABLE && gidx)
        cl_load_idx(st, Stg, lds, j + 64, s1, gidx, goff);
      else
        cl_load(st, Stg, lds, j + 64, s1);
      if (TABLE && threadIdx.x < 32) sw = j + 64 + (int)threadIdx.x < s1 ? w[j + 64 + threadIdx.x] : 0.f;
    }
    const __bf16* A = s_stg + cur * kC6Stage;
    clx16 snext;
    if (more) snext = sprod(s_stg + (cur ^ 1) * kC6Stage);  // the matrix pipe's next S ...
    float ev[16];  // ... while this block's logits are exponentiated
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int r = (e & 3) + 8 * (e >> 2) + 4 * h;
      const float x = j + r < s1 ? cl_exp<FAST>(inv_t, scur[e]) : 0.f;
      if (TABLE) {
        ev[e] = s_w[cur][r] * x;
      } else {
        ev[e] = x;
        z += x;
      }
    }
    const __bf16* Bt = A + 3 * kC6PA;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {  // Y^T (64 d x 32) += Stg^T E^T, K = 32 staged rows in two steps
      const float evs[8] = {ev[8 * t2], ev[8 * t2 + 1], ev[8 * t2 + 2], ev[8 * t2 + 3],
                            ev[8 * t2 + 4], ev[8 * t2 + 5], ev[8 * t2 + 6], ev[8 * t2 + 7]};
      c6bf8 eb[2], a0[2], a1[2];
      c6_split8_2(evs, eb);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        a0[p] = *reinterpret_cast<const c6bf8*>(Bt + p * kC6PB + l32 * kC6B + 8 * (2 * t2 + h));
        a1[p] = *reinterpret_cast<const c6bf8*>(Bt + p * kC6PB + (32 + l32) * kC6B + 8 * (2 * t2 + h));
      }
      y0 = c6_mfma3(a0, eb, y0);
      y1 = c6_mfma3(a1, eb, y1);
    }
    if (refill) {  // block j + 2 takes this block's buffer (s_f's last reader, a convert, finished before a barrier)
      cl_store(st, s_f);
      __syncthreads();  // ... and every wave is done with this block's buffer
      c6_convert(s_f, s_stg + cur * kC6Stage);
      if (TABLE && threadIdx.x < 32) s_w[cur][threadIdx.x] = sw;
      __syncthreads();
    }
    if (more) scur = snext;
    cur ^= 1;
  }
  if (f < nf) cl_put(part_y + ((int64_t)c * nf + f) * 64, y0, y1, h);
  if (!TABLE) {
    const float zf = z + __shfl_xor(z, 32);
    if (f < nf && h == 0) part_z[(int64_t)c * nf + f] = zf;
  }
  if (TABLE && cnt) cl_table_fixup(cnt + blockIdx.x, part_y, nf, dT, ld_dt);
}

// GMR_CL_FIXUP=1 (opt-in; read per call): the table pass reduces its own partials (last block per tile).
// Default 0, cl_table_reduce_kernel: the last block's serial sum is a tail of the launch, 180 / 101 us vs
// 165 / 80 us per call at the DiffMM baby shapes, epoch 99.0 vs 97.0 ms (profiles/r04u_ab.txt)
int cl_fixup() {
  const char* e = getenv("GMR_CL_FIXUP");
  return e && atoi(e) == 1;
}

int cl_pipe() {  // read per call (a getenv), so a test can compare both forms in one process
  const char* e = getenv("GMR_CL_PIPE");
  return !(e && atoi(e) == 0);
}

int cl_x6() {  // read per call (a getenv), so a test can compare both pipes in one process
  const char* e = getenv("GMR_CL_X6");
  return !(e && atoi(e) == 0);
}

struct ClPlan {
  int nca, chunk_a, ncb, chunk_b;
};
// fragments of 32 rows per wave (GMR_CL_NF = 2: each staged block feeds two independent MFMA
// chains per wave and half the workgroups; the chunking, and so every sum, is the same for 1 and 2)
int cl_nf() {  // read per call (a getenv), so a test can compare both in one process
  const char* e = getenv("GMR_CL_NF");
  return (e && atoi(e) == 2) ? 2 : 1;
}
// workgroups per pass (GMR_CL_WG_ROWS / GMR_CL_WG_TABLE override, for tuning)
int cl_wg_target(const char* env, int dflt) {
  const char* s = getenv(env);
  const int v = s ? atoi(s) : 0;
  return v >= 64 && v <= 16384 ? v : dflt;
}
// chunk the j (rows pass) and i (table pass) ranges for ~cl_wg_target workgroups each, in 32-row blocks
ClPlan cl_plan(int64_t B, int64_t n) {
  static const int wa = cl_wg_target("GMR_CL_WG_ROWS", 512), wb = cl_wg_target("GMR_CL_WG_TABLE", 768);
  ClPlan p;
  const int64_t rb = (B + 127) / 128, tb = (n + 127) / 128;
  int64_t want = std::max<int64_t>(1, std::min<int64_t>((wa + rb - 1) / rb, (n + 31) / 32));
  p.chunk_a = (int)(((n + want - 1) / want + 31) / 32 * 32);
  p.nca = (int)((n + p.chunk_a - 1) / p.chunk_a);
  want = std::max<int64_t>(1, std::min<int64_t>((wb + tb - 1) / tb, (B + 31) / 32));
  p.chunk_b = (int)(((B + want - 1) / want + 31) / 32 * 32);
  p.ncb = (int)((B + p.chunk_b - 1) / p.chunk_b);
  return p;
}

}  // namespace

// workspace: [kClCounters table-tile counters (zero between calls) | part_u | part_z | r | part_t]
extern "C" int64_t gmr_contrast_workspace_floats(int32_t B, int64_t n) {
  if (B <= 0 || n <= 0) return -1;
  const ClPlan p = cl_plan(B, n);
  return kClCounters + (int64_t)p.nca * B * 65 + B + (int64_t)p.ncb * n * 64;
}

namespace {
// y2 / ldy2 / nrm2 (optional): dT leaves through the normalize backward of the table's view (the reduce pass)
int contrast_fused(const char* fn, int32_t B, int64_t n, const float* P, int64_t ldp, const float* T, int64_t ldt,
                   const float* CLN, const int32_t* nodes, int64_t node_off, float inv_temp, float coef, float* loss,
                   float* contrib, int64_t ld_contrib, float* dT, int64_t ld_dt, float* workspace,
                   int64_t workspace_floats, const float* y2, int64_t ldy2, const float* nrm2, void* stream) {
  (void)fn;
  // P == nullptr: the batch rows are read in place, P_i = CLN[node_off + nodes[i], 0:64] with ldp = CLN's leading
  // dimension (the pipelined split-bf16 passes only)
  const bool pin = P == nullptr;
  if (pin) P = CLN;
  GMR_ARG(P && T && CLN && nodes && loss && contrib && dT && workspace, "null pointer");
  GMR_ARG(!pin || (cl_x6() && cl_pipe()), "P = null (rows read through nodes) needs the pipelined split-bf16 passes");
  GMR_ARG(B > 0 && n > 0 && n < (1ll << 31), "bad size");
  GMR_ARG(ldp >= 64 && ldt >= 64 && ld_contrib >= 128 && ld_dt >= 64 && ldp % 4 == 0 && ldt % 4 == 0 &&
              ld_dt % 4 == 0,
          "bad leading dimension");
  GMR_ARG((((uintptr_t)P | (uintptr_t)T | (uintptr_t)dT) & 15) == 0, "P, T and dT must be 16-byte aligned");
  GMR_ARG(workspace_floats >= gmr_contrast_workspace_floats(B, n), "workspace too small");
  const ClPlan p = cl_plan(B, n);
  int* counters = reinterpret_cast<int*>(workspace);
  float* part_u = workspace + kClCounters;
  float* part_z = part_u + (int64_t)p.nca * B * 64;
  float* r = part_z + (int64_t)p.nca * B;
  float* part_t = r + B;
  hipStream_t st = (hipStream_t)stream;
  static const bool fast = [] {  // v_exp_f32 (default; 8 % faster, scripts/contrast_bench.py); =0: expf
    const char* e = getenv("GMR_CL_FASTEXP");
    return !(e && atoi(e) == 0);
  }();
  if (cl_x6()) {  // split-bf16 passes (128 fragment rows per workgroup)
    const dim3 ga((unsigned)((B + 127) / 128), (unsigned)p.nca), gb((unsigned)((n + 127) / 128), (unsigned)p.ncb);
    const bool pipe = cl_pipe();
    auto rows6 = fast ? cl6p_kernel<true, false> : cl6p_kernel<false, false>;
    auto table6 = fast ? cl6p_kernel<true, true> : cl6p_kernel<false, true>;
    auto rows6u = fast ? cl6_kernel<true, false> : cl6_kernel<false, false>;
    auto table6u = fast ? cl6_kernel<true, true> : cl6_kernel<false, true>;

    const int* gi = pin ? nodes : nullptr;
    if (pipe)
      hipLaunchKernelGGL(rows6, ga, dim3(256), 0, st, B, (int)n, P, ldp, T, ldt, nullptr, inv_temp, p.chunk_a, part_u,
                         part_z, nullptr, nullptr, 0, gi, node_off);
    else
      hipLaunchKernelGGL(rows6u, ga, dim3(256), 0, st, B, (int)n, P, ldp, T, ldt, nullptr, inv_temp, p.chunk_a, part_u,
                         part_z, nullptr, nullptr, 0);
    GMR_LAUNCHED();
    hipLaunchKernelGGL(cl_finalize_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, p.nca, part_u, part_z,
                       CLN, nodes, node_off, inv_temp, coef, loss, contrib, ld_contrib, r);
    GMR_LAUNCHED();
    // the table pass reduces its own partials (last block per tile) when its tiles fit the counters
    const bool fix = cl_fixup() && gb.x <= (unsigned)kClCounters && !y2;
    if (pipe)
      hipLaunchKernelGGL(table6, gb, dim3(256), 0, st, (int)n, B, T, ldt, P, ldp, r, inv_temp, p.chunk_b, part_t,
                         nullptr, fix ? counters : nullptr, dT, ld_dt, gi, node_off);
    else
      hipLaunchKernelGGL(table6u, gb, dim3(256), 0, st, (int)n, B, T, ldt, P, ldp, r, inv_temp, p.chunk_b, part_t,
                         nullptr, fix ? counters : nullptr, dT, ld_dt);
    GMR_LAUNCHED();
    if (!fix && y2) {
      hipLaunchKernelGGL(cl_table_reduce_nbwd_kernel, dim3(gmr::grid_for(n * 16, 256)), dim3(256), 0, st, (int)n,
                         p.ncb, part_t, dT, ld_dt, y2, ldy2, nrm2);
      GMR_LAUNCHED();
    } else if (!fix) {
      hipLaunchKernelGGL(cl_table_reduce_kernel, dim3(gmr::grid_for(n * 16, 256)), dim3(256), 0, st, (int)n, p.ncb,
                         part_t, dT, ld_dt);
      GMR_LAUNCHED();
    }
    return GMR_OK;
  }
  const int nf = cl_nf();
  const dim3 ga((unsigned)((B + 128 * nf - 1) / (128 * nf)), (unsigned)p.nca);
  const dim3 gb((unsigned)((n + 128 * nf - 1) / (128 * nf)), (unsigned)p.ncb);
  auto rows = fast ? (nf == 2 ? cl_rows_kernel<true, 2> : cl_rows_kernel<true, 1>)
                   : (nf == 2 ? cl_rows_kernel<false, 2> : cl_rows_kernel<false, 1>);
  hipLaunchKernelGGL(rows, ga, dim3(256), 0, st, B, (int)n, P, ldp, T, ldt, inv_temp, p.chunk_a, part_u, part_z);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(cl_finalize_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, B, p.nca, part_u, part_z, CLN,
                     nodes, node_off, inv_temp, coef, loss, contrib, ld_contrib, r);
  GMR_LAUNCHED();
  auto table = fast ? (nf == 2 ? cl_table_kernel<true, 2> : cl_table_kernel<true, 1>)
                    : (nf == 2 ? cl_table_kernel<false, 2> : cl_table_kernel<false, 1>);
  hipLaunchKernelGGL(table, gb, dim3(256), 0, st, B, (int)n, P, ldp, r, T, ldt, inv_temp, p.chunk_b, part_t);
  GMR_LAUNCHED();
  if (y2)
    hipLaunchKernelGGL(cl_table_reduce_nbwd_kernel, dim3(gmr::grid_for(n * 16, 256)), dim3(256), 0, st, (int)n, p.ncb,
                       part_t, dT, ld_dt, y2, ldy2, nrm2);
  else
    hipLaunchKernelGGL(cl_table_reduce_kernel, dim3(gmr::grid_for(n * 16, 256)), dim3(256), 0, st, (int)n, p.ncb,
                       part_t, dT, ld_dt);
  GMR_LAUNCHED();
  return GMR_OK;
}
}  // namespace

extern "C" int gmr_contrast_fused_f32(int32_t B, int64_t n, const float* P, int64_t ldp, const float* T, int64_t ldt,
                                      const float* CLN, const int32_t* nodes, int64_t node_off, float inv_temp,
                                      float coef, float* loss, float* contrib, int64_t ld_contrib, float* dT,
                                      int64_t ld_dt, float* workspace, int64_t workspace_floats, void* stream) {
  return contrast_fused(__func__, B, n, P, ldp, T, ldt, CLN, nodes, node_off, inv_temp, coef, loss, contrib, ld_contrib,
                        dT, ld_dt, workspace, workspace_floats, nullptr, 0, nullptr, stream);
}

extern "C" int gmr_contrast_fused_nbwd_f32(int32_t B, int64_t n, const float* P, int64_t ldp, const float* T,
                                           int64_t ldt, const float* CLN, const int32_t* nodes, int64_t node_off,
                                           float inv_temp, float coef, float* loss, float* contrib, int64_t ld_contrib,
                                           float* dT, int64_t ld_dt, const float* y, int64_t ldy, const float* nrm,
                                           float* workspace, int64_t workspace_floats, void* stream) {
  GMR_ARG(y && nrm && ldy >= 64 && ldy % 4 == 0 && (((uintptr_t)y) & 15) == 0, "bad normalised view");
  return contrast_fused(__func__, B, n, P, ldp, T, ldt, CLN, nodes, node_off, inv_temp, coef, loss, contrib, ld_contrib,
                        dT, ld_dt, workspace, workspace_floats, y, ldy, nrm, stream);
}
