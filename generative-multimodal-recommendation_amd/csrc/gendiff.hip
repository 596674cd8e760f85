// GenRecV1 generative side:
//   FlipInterestDiffusion (models/genrecv1.py:460-648) — schedule from the batch sparsity, flip
//   q_sample, the Bayesian p_sample step, BCE(pos_weight) + curriculum KL rows;
//   ModalDenoiseTransformer (models/genrecv1.py:650-710) row kernels — LayerNorm (+ residual,
//   + dropout, + GELU) forward/backward, adaLN modulation, dropout masks, time embedding, SiLU.
// The dense products of the transformer run on the MFMA GEMM (gemm.hip).
#include <algorithm>

#include "gmr_common.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ float unit01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }  // [0, 1)

// Draw mapping of the per-element Bernoulli kernels (round 6): the 32-bit word of draw unit g (a global index,
// keyed by the GLOBAL row so any row split draws the same values) is word g % 4 of Philox(seed, step, g / 4) -
// one Philox call per four units instead of one per unit (the draws were 14 % and 11 % of the GenRecV1 leg's
// wave cycles, profiles/r05zz4_legs_lds_stalls.txt: dropout_kernel, flip_step_kernel).  Kernels that take one
// unit per thread compute the same word with ph_word; the hot ones give a thread the four units of one call.
__device__ __forceinline__ uint32_t ph_pick(const uint4& r, int k) {
  return k == 0 ? r.x : k == 1 ? r.y : k == 2 ? r.z : r.w;
}
__device__ __forceinline__ uint32_t ph_word(uint64_t seed, uint64_t step, uint64_t g) {
  return ph_pick(gmr::Philox::gen(seed, step, g >> 2), (int)(g & 3));
}
// quads of global units covering the local units [0, n) whose global index is base + u
__host__ __device__ __forceinline__ int64_t ph_quads(int64_t base, int64_t n) { return ((base + n + 3) >> 2) - (base >> 2); }

// ----------------------------------------------------------------- schedule (get_cum, :480-498)
// tables: [gamma_cum (T) | eps_cum (T) | pos_weight | sparsity]; fp32 op order of the reference
// (no contraction), linspace as ATen's CPU kernel (start + step*i below the midpoint, end - step*(T-1-i) above).
__global__ void flip_schedule_kernel(int B, const int* __restrict__ users, const int* __restrict__ user_ptr, int I,
                                     int T, float* __restrict__ tab) {
  __shared__ long long s_ones[256];
  long long ones = 0;
  for (int b = threadIdx.x; b < B; b += 256) {
    const int u = users[b];
    ones += user_ptr[u + 1] - user_ptr[u];
  }
  s_ones[threadIdx.x] = ones;
  __syncthreads();
  if (threadIdx.x != 0) return;
  long long tot = 0;
  for (int j = 0; j < 256; ++j) tot += s_ones[j];
  const long long n = (long long)B * I;
  const float zeros = (float)(n - tot);
  const float s = __fdiv_rn(zeros, (float)n);
  const float gs = __fadd_rn(__fmul_rn(0.1f, __fsub_rn(1.f, s)), 0.001f);
  const float ge = __fmul_rn(gs, 0.1f);
  const float es = __fadd_rn(__fmul_rn(0.005f, s), 0.0001f);
  const float ee = __fmul_rn(es, 0.1f);
  const float gstep = __fdiv_rn(__fsub_rn(ge, gs), (float)(T - 1));
  const float estep = __fdiv_rn(__fsub_rn(ee, es), (float)(T - 1));
  const int half = T / 2;
  double gc = 1.0, ec = 1.0;  // ATen's CPU cumprod accumulates float in double (acc_type)
  for (int i = 0; i < T; ++i) {
    float g, e;
    if (i < half) {
      g = __fadd_rn(gs, __fmul_rn(gstep, (float)i));
      e = __fadd_rn(es, __fmul_rn(estep, (float)i));
    } else {
      g = __fsub_rn(ge, __fmul_rn(gstep, (float)(T - i - 1)));
      e = __fsub_rn(ee, __fmul_rn(estep, (float)(T - i - 1)));
    }
    e = fminf(e, 0.01f);
    gc = __dmul_rn(gc, (double)__fsub_rn(1.f, g));
    ec = __dmul_rn(ec, (double)__fsub_rn(1.f, e));
    tab[i] = __fsub_rn(1.f, (float)gc);
    tab[T + i] = __fsub_rn(1.f, (float)ec);
  }
  tab[2 * T] = __fdiv_rn(zeros, __fadd_rn((float)tot, 1e-8f));
  tab[2 * T + 1] = s;
}

// x_t = x0 xor Bernoulli(sigmoid((a_t - u) * temp)), a_t = gamma_cum[t] (x0 == 0) or eps_cum[t] (x0 == 1)
// Draws: unit g = (row0 + b) I + i takes words 2 (g % 2), 2 (g % 2) + 1 of Philox(seed, step, g / 2) (two units
// per call; each needs two words).  A thread takes the two units of one call.
__global__ void flip_qsample_kernel(int B, int I, const float* __restrict__ x0, int64_t ld0, const int* __restrict__ t,
                                    int t_const, const float* __restrict__ tab, int T, float temp,
                                    const uint8_t* __restrict__ flip, int64_t ldf, uint64_t seed, uint64_t step,
                                    int64_t row0, float* __restrict__ xt, int64_t ldt) {
  const int64_t n = (int64_t)B * I, base = row0 * I;
  const int64_t q = (base >> 1) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t u0 = (q << 1) - base;
  if (u0 >= n) return;
  uint4 r = make_uint4(0u, 0u, 0u, 0u);
  if (!flip) r = gmr::Philox::gen(seed, step, (uint64_t)q);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int64_t u = u0 + k;
    if (u < 0 || u >= n) continue;
    const int b = (int)((uint32_t)u / (uint32_t)I), i = (int)(u - (int64_t)b * I);
    const float x = x0[(int64_t)b * ld0 + i];
    bool f;
    if (flip) {
      f = flip[(int64_t)b * ldf + i] != 0;
    } else {
      const int tt = t ? t[b] : t_const;
      const float a = x == 0.f ? tab[tt] : tab[T + tt];
      const float p = sigm((a - unit01(k ? r.z : r.x)) * temp);
      f = unit01(k ? r.w : r.y) < p;
    }
    xt[(int64_t)b * ldt + i] = f ? 1.f - x : x;
  }
}

// p_sample step on the model logits: probs = sigmoid(z); x = Bernoulli(p1 / (p0 + p1)) with
// a0 = gamma_cum[qi], a1 = eps_cum[qi] (the q_sample(t = qi) tables re-indexed by row, :541-545), or
// Bernoulli(probs) on the last step; draws (0/1 bytes) replace the Bernoulli when given
__global__ void flip_step_kernel(int B, int I, const float* __restrict__ z, int64_t ldz, const float* __restrict__ tab,
                                 int T, int qi, int last, const uint8_t* __restrict__ draws, int64_t ldd, uint64_t seed,
                                 uint64_t step, int64_t row0, float* __restrict__ x, int64_t ldx,
                                 float* __restrict__ probs, int64_t ldp) {
  // unit g = (row0 + b) I + i: word g % 4 of Philox(seed, step, g / 4); a thread takes the four units of one call
  const int64_t n = (int64_t)B * I, base = row0 * I;
  const int64_t qd = (base >> 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t u0 = (qd << 2) - base;
  if (u0 >= n) return;
  uint4 r = make_uint4(0u, 0u, 0u, 0u);
  if (!draws) r = gmr::Philox::gen(seed, step, (uint64_t)qd);
  const float a0 = tab[qi], a1 = tab[T + qi];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t u = u0 + k;
    if (u < 0 || u >= n) continue;
    const int b = (int)((uint32_t)u / (uint32_t)I), i = (int)(u - (int64_t)b * I);
    const float p = sigm(z[(int64_t)b * ldz + i]);
    if (probs) probs[(int64_t)b * ldp + i] = p;
    float q = p;
    if (!last) {
      const float p0 = p * (1.f - a0) + (1.f - p) * a1;
      const float p1 = p * a0 + (1.f - p) * (1.f - a1);
      q = p1 / (p0 + p1);
    }
    const float v = draws ? (draws[(int64_t)b * ldd + i] ? 1.f : 0.f) : (unit01(ph_pick(r, k)) < q ? 1.f : 0.f);
    x[(int64_t)b * ldx + i] = v;
  }
}

// per row: bce_row = sum_i (1-y) z - lw logsigmoid(z), lw = 1 + (pw-1) y (ATen's
// binary_cross_entropy_with_logits); kl_row = cw[t] * mean_i KL(post || clamp(p)); the BCE
// gradient (1-y) - lw sigmoid(-z) times grad_scale overwrites dz (may alias z)
__global__ void __launch_bounds__(256) flip_loss_kernel(int B, int I, const float* __restrict__ x0, int64_t ld0,
                                                        const float* z, int64_t ldz, const int* __restrict__ t,
                                                        const float* __restrict__ tab, int T, float grad_scale,
                                                        float* dz, int64_t lddz, double* __restrict__ bce_row,
                                                        double* __restrict__ kl_row) {
  const int b = blockIdx.x;
  const float pw = tab[2 * T];
  const float a0 = tab[T - 1], a1 = tab[2 * T - 1];
  const float eps = 1e-8f;
  double sb = 0.0, sk = 0.0;
  for (int i = threadIdx.x; i < I; i += 256) {
    const float y = x0[(int64_t)b * ld0 + i];
    const float zz = z[(int64_t)b * ldz + i];
    const float lw = (pw - 1.f) * y + 1.f;
    const float ls = fminf(zz, 0.f) - log1pf(expf(-fabsf(zz)));  // log sigmoid
    sb += (double)((1.f - y) * zz - lw * ls);
    // KL against the true posterior (genrecv1.py:608-627)
    const float num = (y == 0.f ? 1.f : 0.f) * (1.f - a0) + (y == 1.f ? 1.f : 0.f) * a1;
    const float den = (y == 0.f ? 1.f : 0.f) * (1.f - a0 + a1) + (y == 1.f ? 1.f : 0.f) * (a0 + 1.f - a1);
    const float post = fminf(fmaxf(num / (den + eps), eps), 1.f - eps);
    const float pr = fminf(fmaxf(sigm(zz), eps), 1.f - eps);
    const float kl = post * (logf(post + 1e-10f) - logf(pr + 1e-10f)) +
                     (1.f - post) * (logf(1.f - post + 1e-10f) - logf(1.f - pr + 1e-10f));
    sk += (double)kl;
    if (dz) dz[(int64_t)b * lddz + i] = grad_scale * ((1.f - y) - lw * sigm(-zz));
  }
  __shared__ double rb[4], rk[4];
  sb = gmr::wave_sum_d(sb);
  sk = gmr::wave_sum_d(sk);
  if ((threadIdx.x & 63) == 0) {
    rb[threadIdx.x >> 6] = sb;
    rk[threadIdx.x >> 6] = sk;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    bce_row[b] = (rb[0] + rb[1]) + (rb[2] + rb[3]);
    float cw = (float)t[b] / (float)T;
    cw = fminf(fmaxf(cw, 0.f), 0.5f);
    kl_row[b] = (double)cw * ((rk[0] + rk[1]) + (rk[2] + rk[3])) / (double)I;
  }
}

// ----------------------------------------------------------------- LayerNorm (one wave per row, D <= 1024)
// s = a + keep * scale * b (b: matrix, or a broadcast vector when ldb == 0); y = LN(s) w + bias [-> GELU].
// LnDraw.on: the keep bytes are drawn here (gmr_keep_mask_u8's Philox key, counter ctr0 + r D + c) and stored
// to keep, instead of read from it: the residual-branch dropout without its separate mask launch.
struct LnDraw {
  float p_keep;
  uint64_t seed, step, ctr0;
  int on;
};
template <int PER>  // floats per lane (D = 64 * PER; PER 1 with Dsmall = 32 or 64)
__global__ void __launch_bounds__(256) ln_fwd_kernel(int Dsmall, int64_t rows, const float* __restrict__ a, int64_t lda,
                                                     const float* __restrict__ bsrc, int64_t ldb,
                                                     uint8_t* __restrict__ keep, int64_t ldk, float kscale, LnDraw dr,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     float eps, int gelu, float* __restrict__ y, int64_t ldy,
                                                     float* __restrict__ s_out, int64_t lds,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  const int D = PER == 1 ? Dsmall : 64 * PER;  // PER == 1 also serves D = 32 (upper lanes idle)
  const bool act = lane < D;
  float v[PER];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = j * 64 + lane;
    float x = 0.f;
    if (act) {
      x = a[r * lda + c];
      if (bsrc) {
        float bb = bsrc[(ldb ? r * ldb : 0) + c];
        if (dr.on) {
          const uint4 q = gmr::Philox::gen(dr.seed, dr.step, dr.ctr0 + (uint64_t)(r * D + c));
          const uint8_t k = (float)(q.x >> 8) * (1.0f / 16777216.0f) < dr.p_keep ? 1 : 0;
          keep[r * ldk + c] = k;
          bb = k ? bb * kscale : 0.f;
        } else if (keep) {
          bb = keep[r * ldk + c] ? bb * kscale : 0.f;
        }
        x += bb;
      }
    }
    v[j] = x;
    sum += x;
  }
  const float mean = gmr::wave_sum(sum) / (float)D;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const float d = act ? v[j] - mean : 0.f;
    sq += d * d;
  }
  const float rstd = 1.f / sqrtf(gmr::wave_sum(sq) / (float)D + eps);
  if (!act) return;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = j * 64 + lane;
    if (s_out) s_out[r * lds + c] = v[j];
    float o = (v[j] - mean) * rstd * w[c] + bias[c];
    if (gelu) o = 0.5f * o * (1.f + erff(o * 0.70710678118654752f));
    y[r * ldy + c] = o;
  }
  if (lane == 0) {
    mean_out[r] = mean;
    rstd_out[r] = rstd;
  }
}

// dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dy w (dy through GELU first);
// dw/db column partials per block (rows blockIdx.x*RB .. ) -> part[blk][2*D]
constexpr int kLnRowsPerBlock = 8;
template <int PER>
__global__ void __launch_bounds__(256) ln_bwd_kernel(int Dsmall, int64_t rows, const float* __restrict__ s, int64_t lds,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     int gelu, const float* __restrict__ dy, int64_t lddy,
                                                     float* __restrict__ dx, int64_t lddx, int accumulate,
                                                     float* __restrict__ part) {
  constexpr int DM = 64 * PER;
  const int D = PER == 1 ? Dsmall : DM;
  __shared__ float red[4][2 * DM];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool act = lane < D;
  float pw[PER], pb[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) pw[j] = pb[j] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * kLnRowsPerBlock;
  for (int64_t r = r0 + wv; r < rows && r < r0 + kLnRowsPerBlock; r += 4) {
    const float mu = mean[r], rs = rstd[r];
    float xh[PER], g[PER];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = j * 64 + lane;
      if (!act) {
        xh[j] = g[j] = 0.f;
        continue;
      }
      xh[j] = (s[r * lds + c] - mu) * rs;
      float d = dy[r * lddy + c];
      if (gelu) {
        const float u = xh[j] * w[c] + bias[c];
        const float cdf = 0.5f * (1.f + erff(u * 0.70710678118654752f));
        const float pdf = 0.3989422804014327f * expf(-0.5f * u * u);
        d *= cdf + u * pdf;
      }
      pw[j] += d * xh[j];
      pb[j] += d;
      g[j] = d * w[c];
      s1 += g[j];
      s2 += g[j] * xh[j];
    }
    s1 = gmr::wave_sum(s1) / (float)D;
    s2 = gmr::wave_sum(s2) / (float)D;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = j * 64 + lane;
      if (!act) continue;
      float o = rs * (g[j] - s1 - xh[j] * s2);
      if (accumulate) o += dx[r * lddx + c];
      dx[r * lddx + c] = o;
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    red[wv][j * 64 + lane] = act ? pw[j] : 0.f;
    red[wv][DM + j * 64 + lane] = act ? pb[j] : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += 256) {
    const int cc = c < D ? c : DM + (c - D);
    part[(int64_t)blockIdx.x * 2 * D + c] = (red[0][cc] + red[1][cc]) + (red[2][cc] + red[3][cc]);
  }
}

// column c of the P x 2D partials: 16 part groups per column (fixed order), 64 columns per block
__global__ void __launch_bounds__(1024) ln_param_reduce_kernel(int P, int D, const float* __restrict__ part,
                                                               float* __restrict__ dw, float* __restrict__ db,
                                                               int accumulate) {
  __shared__ double red[16][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s = 0.0;
  if (c < 2 * D)
    for (int p = g; p < P; p += 16) s += part[(int64_t)p * 2 * D + c];
  red[g][cl] = s;
  __syncthreads();
  if (g != 0 || c >= 2 * D) return;
  s = 0.0;
  for (int j = 0; j < 16; ++j) s += red[j][cl];
  float* o = c < D ? dw + c : db + (c - D);
  *o = (float)s + (accumulate ? *o : 0.f);
}

// ----------------------------------------------------------------- adaLN, dropout, time embedding, SiLU
// h1 = h0 (1 + scale[t]) + shift[t]; S = T x 2D table [shift | scale] (chunk(2) order, :702)
__global__ void adaln_fwd_kernel(int64_t rows, int D, const float* __restrict__ h0, int64_t ld0,
                                 const int* __restrict__ t, int t_const, const float* __restrict__ S, int64_t lds,
                                 float* __restrict__ h1, int64_t ld1) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= rows * D) return;
  const int64_t r = gid / D;
  const int c = (int)(gid % D);
  const int tt = t ? t[r] : t_const;
  const float* srow = S + (int64_t)tt * lds;
  h1[r * ld1 + c] = h0[r * ld0 + c] * (1.f + srow[D + c]) + srow[c];
}

// dh0 = dh1 (1 + scale[t]); prod = dh1 * h0 (for the grouped column sums of dscale)
__global__ void adaln_bwd_kernel(int64_t rows, int D, const float* __restrict__ h0, int64_t ld0,
                                 const float* __restrict__ dh1, int64_t ldd, const int* __restrict__ t,
                                 const float* __restrict__ S, int64_t lds, float* __restrict__ dh0, int64_t ldo,
                                 float* __restrict__ prod, int64_t ldp) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= rows * D) return;
  const int64_t r = gid / D;
  const int c = (int)(gid % D);
  const float g = dh1[r * ldd + c];
  prod[r * ldp + c] = g * h0[r * ld0 + c];
  dh0[r * ldo + c] = g * (1.f + S[(int64_t)t[r] * lds + D + c]);
}

// y = x * keep / p_keep; keep drawn per (row, column / group) when mask_in is null (written to
// mask_out), else read from mask_in
__global__ void dropout_kernel(int64_t rows, int D, int group, const float* __restrict__ x, int64_t ldx,
                               float p_keep, const uint8_t* __restrict__ mask_in, uint8_t* __restrict__ mask_out,
                               int64_t ldm, uint64_t seed, uint64_t step, int64_t row0, float* __restrict__ y,
                               int64_t ldy) {
  // draw unit g = (row0 + r) (D / group) + c / group (ph_word); group 1: a thread takes the four units of one call
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (group == 1) {
    const int64_t n = rows * D, base = row0 * D;
    const int64_t qd = (base >> 2) + gid;
    const int64_t u0 = (qd << 2) - base;
    if (u0 >= n) return;
    uint4 rr = make_uint4(0u, 0u, 0u, 0u);
    if (!mask_in) rr = gmr::Philox::gen(seed, step, (uint64_t)qd);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t u = u0 + q;
      if (u < 0 || u >= n) continue;
      const int64_t r = (uint32_t)u / (uint32_t)D;  // rows * D < 2^31 (checked at launch)
      const int c = (int)(u - r * D);
      bool k;
      if (mask_in) {
        k = mask_in[r * ldm + c] != 0;
      } else {
        k = unit01(ph_pick(rr, q)) < p_keep;
        if (mask_out) mask_out[r * ldm + c] = k ? 1 : 0;
      }
      y[r * ldy + c] = k ? x[r * ldx + c] / p_keep : 0.f;
    }
    return;
  }
  if (gid >= rows * D) return;
  const int64_t r = gid / D;
  const int c = (int)(gid % D);
  const int mc = c / group;
  bool k;
  if (mask_in) {
    k = mask_in[r * ldm + mc] != 0;
  } else {
    k = unit01(ph_word(seed, step, (uint64_t)((row0 + r) * (D / group) + mc))) < p_keep;
    if (mask_out && c % group == 0) mask_out[r * ldm + mc] = k ? 1 : 0;
  }
  y[r * ldy + c] = k ? x[r * ldx + c] / p_keep : 0.f;
}

// ---------------------------------------------------------------- cross-attention on the zero memory
// nn.TransformerDecoderLayer's multihead_attn over the all-zero memory (models/genrecv1.py:650-710):
// every key / value is the in-projection bias, so head h's attention output is bv'_h for every row and
// the block is out_proj(dropout_head(bv')) + b_o.  With head dropout that is, per row, a mixture of
// nhead fixed vectors: CA[r] = b_o + sum_h keep[r][h] P[h], P[h][j] = sum_{c in head h} Wo[j][c] bv'[c] /
// p_keep, so the B x D x D product of the unfused path becomes a table of nhead x D (once per weight
// version) and a per-row sum; its backward, the per-head column sums Gs[h][j] = sum_r keep[r][h] dCA[r][j].
// P[l][h][j] for the L layers at once (layer l's tensors at woc0 / bvc0 + l * lstride; Wo row-major, ld D)
__global__ void xattn_table_kernel(int L, int D, int nhead, const float* __restrict__ woc0,
                                   const float* __restrict__ bvc0, int64_t lstride, float p_keep, float* __restrict__ P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)L * nhead * D) return;
  const int j = (int)(i % D), h = (int)((i / D) % nhead);
  const int64_t l = i / ((int64_t)D * nhead);
  const float* w = woc0 + l * lstride + (int64_t)j * D;
  const float* b = bvc0 + l * lstride;
  const int g = D / nhead;
  float s = 0.f;
  for (int c = h * g; c < (h + 1) * g; ++c) s = fmaf(w[c], b[c] / p_keep, s);
  P[i] = s;
}

// one row per block: the row's nhead keep flags (the head-dropout draw of dropout_kernel, group D / nhead:
// draw unit (row0 + r) * nhead + h, ph_word) or the given mask, then CA[r][j] = sum_h keep P[h][j] + b_o[j]
__global__ void __launch_bounds__(256) xattn_fwd_kernel(int D, int nhead, const float* __restrict__ P,
                                                        const float* __restrict__ bo, float p_keep,
                                                        const uint8_t* __restrict__ mask_in, uint8_t* __restrict__ mask_out,
                                                        int64_t ldm, uint64_t seed, uint64_t step, int64_t row0,
                                                        float* __restrict__ CA, int64_t ldc) {
  __shared__ float kf[64];
  const int64_t r = blockIdx.x;
  if ((int)threadIdx.x < nhead) {
    const int h = threadIdx.x;
    bool k;
    if (mask_in) {
      k = mask_in[r * ldm + h] != 0;
    } else {
      k = unit01(ph_word(seed, step, (uint64_t)((row0 + r) * nhead + h))) < p_keep;
      if (mask_out) mask_out[r * ldm + h] = k ? 1 : 0;
    }
    kf[h] = k ? 1.f : 0.f;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < D; j += blockDim.x) {
    float s = 0.f;
    for (int h = 0; h < nhead; ++h)
      if (kf[h] != 0.f) s += P[(int64_t)h * D + j];
    CA[r * ldc + j] = s + bo[j];
  }
}

// per-head column sums of dCA over a chunk of rows -> part[chunk][h][j] (64 columns x 4 row lanes per block)
constexpr int kXattnMaxHeads = 16;
__global__ void __launch_bounds__(256) xattn_bwd_part_kernel(int64_t rows, int D, int nhead,
                                                             const float* __restrict__ dCA, int64_t ld,
                                                             const uint8_t* __restrict__ mask, int64_t ldm,
                                                             int64_t chunk, float* __restrict__ part) {
  __shared__ float red[4][kXattnMaxHeads][64];
  const int tx = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + tx;
  const int64_t r0 = (int64_t)blockIdx.y * chunk, r1 = min(rows, r0 + chunk);
  float acc[kXattnMaxHeads];
#pragma unroll
  for (int h = 0; h < kXattnMaxHeads; ++h) acc[h] = 0.f;
  if (j < D)
    for (int64_t r = r0 + rl; r < r1; r += 4) {
      const float d = dCA[r * ld + j];
#pragma unroll
      for (int h = 0; h < kXattnMaxHeads; ++h)
        if (h < nhead && mask[r * ldm + h]) acc[h] += d;
    }
#pragma unroll
  for (int h = 0; h < kXattnMaxHeads; ++h) red[rl][h][tx] = acc[h];
  __syncthreads();
  if (rl == 0 && j < D)
    for (int h = 0; h < nhead; ++h)
      part[((int64_t)blockIdx.y * nhead + h) * D + j] = (red[0][h][tx] + red[1][h][tx]) + (red[2][h][tx] + red[3][h][tx]);
}

// Gs[h][j] = sum over the chunks (fixed order)
__global__ void xattn_bwd_reduce_kernel(int D, int nhead, int chunks, const float* __restrict__ part,
                                        float* __restrict__ G) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nhead * D) return;
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += part[(int64_t)c * nhead * D + i];
  G[i] = s;
}

// dWo[j][c] += Gs[h(c)][j] bv'[c] / p_keep (Bc = keep bv' / p_keep); dbv'[c] += sum_j Wo[j][c] Gs[h(c)][j] / p_keep.
// The first D / 16 blocks reduce dbv' (16 columns x 16 row lanes, summed across the lanes in a fixed order: one
// thread per column walking all D rows was a serial tail of the launch); the rest update dWo elementwise.
constexpr int kXattnBvCols = 16;
__global__ void __launch_bounds__(256) xattn_bwd_apply_kernel(int D, int nhead, const float* __restrict__ G,
                                                              const float* __restrict__ wo, const float* __restrict__ bv,
                                                              float p_keep, float* __restrict__ g_wo,
                                                              float* __restrict__ g_bv) {
  const int g = D / nhead;
  const int nbv = (D + kXattnBvCols - 1) / kXattnBvCols;
  if ((int)blockIdx.x < nbv) {
    __shared__ float red[256 / kXattnBvCols][kXattnBvCols];
    const int cc = threadIdx.x % kXattnBvCols, rl = threadIdx.x / kXattnBvCols;
    const int c = blockIdx.x * kXattnBvCols + cc;
    float s = 0.f;
    if (c < D) {
      const float* gh = G + (int64_t)(c / g) * D;
      for (int j = rl; j < D; j += 256 / kXattnBvCols) s = fmaf(wo[(int64_t)j * D + c], gh[j], s);
    }
    red[rl][cc] = s;
    __syncthreads();
    if (rl == 0 && c < D) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 256 / kXattnBvCols; ++q) t += red[q][cc];
      g_bv[c] += t / p_keep;
    }
    return;
  }
  const int64_t i = (int64_t)(blockIdx.x - nbv) * blockDim.x + threadIdx.x;
  if (i < (int64_t)D * D) {
    const int j = (int)(i / D), c = (int)(i % D);
    g_wo[i] += G[(int64_t)(c / g) * D + j] * (bv[c] / p_keep);
  }
}

// temb[t] = [cos(t f_k) | sin(t f_k)], f_k = exp(-ln(1e4) k / half) (:692-696); odd sizes zero-pad
__global__ void time_embedding_kernel(int T, int E, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T * E) return;
  const int t = i / E, k = i % E, half = E / 2;
  float v = 0.f;
  if (k < 2 * half) {
    const int kk = k < half ? k : k - half;
    const float f = expf(__fdiv_rn(__fmul_rn(-9.210340371976184f, (float)kk), (float)half));
    const float a = __fmul_rn((float)t, f);
    v = k < half ? cosf(a) : sinf(a);
  }
  out[i] = v;
}

__global__ void flip_total_kernel(const double* __restrict__ bk, const float* __restrict__ cl, float w_cl,
                                  float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const float b = (float)bk[0], k = (float)bk[1], c = cl[0];
  out[0] = b;
  out[1] = k;
  out[2] = c;
  out[3] = b + k + w_cl * c;
}

__global__ void silu_kernel(int64_t n, const float* __restrict__ x, const float* __restrict__ dy,
                            float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i], s = sigm(v);
  y[i] = dy ? dy[i] * s * (1.f + v * (1.f - s)) : v * s;
}

}  // namespace

extern "C" int gmr_flip_schedule(int32_t B, const int32_t* users, const int32_t* user_ptr, int32_t I, int32_t T,
                                 float* tables, void* stream) {
  GMR_ARG(users && user_ptr && tables && B > 0 && I > 0 && T >= 2, "bad args");
  hipLaunchKernelGGL(flip_schedule_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, B, users, user_ptr, I, T,
                     tables);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_flip_qsample(int32_t B, int32_t I, const float* x0, int64_t ld0, const int32_t* t, int32_t t_const,
                                const float* tables, int32_t T, float temp, const uint8_t* flip, int64_t ld_flip,
                                uint64_t seed, uint64_t step, int64_t row0, float* xt, int64_t ldt, void* stream) {
  GMR_ARG(x0 && tables && xt && B > 0 && I > 0 && row0 >= 0, "bad args");
  GMR_ARG(t || (t_const >= 0 && t_const < T), "bad t");
  GMR_ARG((int64_t)B * I < (1ll << 31), "B * I too large");
  const int64_t npairs = ((row0 * I + (int64_t)B * I + 1) >> 1) - ((row0 * I) >> 1);
  hipLaunchKernelGGL(flip_qsample_kernel, dim3(gmr::grid_for(npairs, 256)), dim3(256), 0, (hipStream_t)stream,
                     B, I, x0, ld0, t, t_const, tables, T, temp, flip, ld_flip, seed, step, row0, xt, ldt);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_flip_step(int32_t B, int32_t I, const float* z, int64_t ldz, const float* tables, int32_t T,
                             int32_t qi, int32_t last, const uint8_t* draws, int64_t ldd, uint64_t seed, uint64_t step,
                             int64_t row0, float* x, int64_t ldx, float* probs, int64_t ldp, void* stream) {
  GMR_ARG(z && tables && x && B > 0 && I > 0 && qi >= 0 && qi < T && row0 >= 0, "bad args");
  GMR_ARG((int64_t)B * I < (1ll << 31), "B * I too large");
  hipLaunchKernelGGL(flip_step_kernel, dim3(gmr::grid_for(ph_quads(row0 * I, (int64_t)B * I), 256)), dim3(256), 0,
                     (hipStream_t)stream, B,
                     I, z, ldz, tables, T, qi, last, draws, ldd, seed, step, row0, x, ldx, probs, ldp);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_flip_loss_rows(int32_t B, int32_t I, const float* x0, int64_t ld0, const float* z, int64_t ldz,
                                  const int32_t* t, const float* tables, int32_t T, float grad_scale, float* dz,
                                  int64_t lddz, double* bce_row, double* kl_row, void* stream) {
  GMR_ARG(x0 && z && t && tables && bce_row && kl_row && B > 0 && I > 0, "bad args");
  hipLaunchKernelGGL(flip_loss_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, B, I, x0, ld0, z, ldz, t, tables, T,
                     grad_scale, dz, lddz, bce_row, kl_row);
  GMR_LAUNCHED();
  return GMR_OK;
}

namespace {
int layernorm_launch(int64_t rows, int32_t D, const float* a, int64_t lda, const float* b, int64_t ldb, uint8_t* keep,
                     int64_t ld_keep, float keep_scale, LnDraw dr, const float* w, const float* bias, float eps,
                     int32_t gelu, float* y, int64_t ldy, float* s_out, int64_t lds, float* mean, float* rstd,
                     void* stream) {
  GMR_ARG(a && w && bias && y && mean && rstd && rows > 0, "bad args");
  GMR_ARG(D == 32 || D == 64 || D == 128 || D == 256 || D == 512 || D == 1024, "D must be 32..1024 (power of two)");
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
#define GMR_LNF(P)                                                                                                \
  hipLaunchKernelGGL(ln_fwd_kernel<P>, grid, dim3(256), 0, st, (int)D, rows, a, lda, b, ldb, keep, ld_keep,        \
                     keep_scale, dr, w, bias, eps, (int)gelu, y, ldy, s_out, lds, mean, rstd)
  switch (D) {
    case 32:
    case 64: GMR_LNF(1); break;
    case 128: GMR_LNF(2); break;
    case 256: GMR_LNF(4); break;
    case 512: GMR_LNF(8); break;
    default: GMR_LNF(16); break;
  }
#undef GMR_LNF
  GMR_LAUNCHED();
  return GMR_OK;
}
}  // namespace

extern "C" int gmr_layernorm_fwd(int64_t rows, int32_t D, const float* a, int64_t lda, const float* b, int64_t ldb,
                                 const uint8_t* keep, int64_t ld_keep, float keep_scale, const float* w,
                                 const float* bias, float eps, int32_t gelu, float* y, int64_t ldy, float* s_out,
                                 int64_t lds, float* mean, float* rstd, void* stream) {
  return layernorm_launch(rows, D, a, lda, b, ldb, const_cast<uint8_t*>(keep), ld_keep, keep_scale, LnDraw{1.f, 0, 0, 0, 0},
                          w, bias, eps, gelu, y, ldy, s_out, lds, mean, rstd, stream);
}

extern "C" int gmr_layernorm_drop_fwd(int64_t rows, int32_t D, const float* a, int64_t lda, const float* b, int64_t ldb,
                                      float p_keep, uint64_t seed, uint64_t step, uint64_t ctr0, uint8_t* keep_out,
                                      int64_t ld_keep, float keep_scale, const float* w, const float* bias, float eps,
                                      int32_t gelu, float* y, int64_t ldy, float* s_out, int64_t lds, float* mean,
                                      float* rstd, void* stream) {
  GMR_ARG(b && ldb > 0 && keep_out && ld_keep >= D, "the dropped branch b and the keep buffer are required");
  GMR_ARG(p_keep > 0.f && p_keep <= 1.f, "p_keep in (0, 1]");
  return layernorm_launch(rows, D, a, lda, b, ldb, keep_out, ld_keep, keep_scale, LnDraw{p_keep, seed, step, ctr0, 1}, w,
                          bias, eps, gelu, y, ldy, s_out, lds, mean, rstd, stream);
}

extern "C" int64_t gmr_layernorm_parts_floats(int64_t rows, int32_t D) {
  return ((rows + kLnRowsPerBlock - 1) / kLnRowsPerBlock) * 2 * (int64_t)D;
}

extern "C" int gmr_layernorm_bwd(int64_t rows, int32_t D, const float* s, int64_t lds, const float* mean,
                                 const float* rstd, const float* w, const float* bias, int32_t gelu, const float* dy,
                                 int64_t lddy, float* dx, int64_t lddx, int32_t accumulate_dx, float* parts, float* dw,
                                 float* db, int32_t accumulate_params, void* stream) {
  GMR_ARG(s && mean && rstd && w && bias && dy && dx && parts && dw && db && rows > 0, "bad args");
  GMR_ARG(D == 32 || D == 64 || D == 128 || D == 256 || D == 512 || D == 1024, "D must be 32..1024 (power of two)");
  hipStream_t st = (hipStream_t)stream;
  const int P = (int)((rows + kLnRowsPerBlock - 1) / kLnRowsPerBlock);
#define GMR_LNB(PP)                                                                                                  \
  hipLaunchKernelGGL(ln_bwd_kernel<PP>, dim3(P), dim3(256), 0, st, (int)D, rows, s, lds, mean, rstd, w, bias,         \
                     (int)gelu, dy, lddy, dx, lddx, (int)accumulate_dx, parts)
  switch (D) {
    case 32:
    case 64: GMR_LNB(1); break;
    case 128: GMR_LNB(2); break;
    case 256: GMR_LNB(4); break;
    case 512: GMR_LNB(8); break;
    default: GMR_LNB(16); break;
  }
#undef GMR_LNB
  GMR_LAUNCHED();
  hipLaunchKernelGGL(ln_param_reduce_kernel, dim3(gmr::grid_for(2 * D, 64)), dim3(1024), 0, st, P, D, parts, dw, db,
                     (int)accumulate_params);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_adaln_fwd(int64_t rows, int32_t D, const float* h0, int64_t ld0, const int32_t* t, int32_t t_const,
                             const float* S, int64_t lds, float* h1, int64_t ld1, void* stream) {
  GMR_ARG(h0 && S && h1 && rows > 0 && D > 0, "bad args");
  hipLaunchKernelGGL(adaln_fwd_kernel, dim3(gmr::grid_for(rows * D, 256)), dim3(256), 0, (hipStream_t)stream, rows, D,
                     h0, ld0, t, t_const, S, lds, h1, ld1);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_adaln_bwd(int64_t rows, int32_t D, const float* h0, int64_t ld0, const float* dh1, int64_t ldd,
                             const int32_t* t, const float* S, int64_t lds, float* dh0, int64_t ldo, float* prod,
                             int64_t ldp, void* stream) {
  GMR_ARG(h0 && dh1 && t && S && dh0 && prod && rows > 0, "bad args");
  hipLaunchKernelGGL(adaln_bwd_kernel, dim3(gmr::grid_for(rows * D, 256)), dim3(256), 0, (hipStream_t)stream, rows, D,
                     h0, ld0, dh1, ldd, t, S, lds, dh0, ldo, prod, ldp);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_dropout_f32(int64_t rows, int32_t D, int32_t group, const float* x, int64_t ldx, float p_keep,
                               const uint8_t* mask_in, uint8_t* mask_out, int64_t ldm, uint64_t seed, uint64_t step,
                               int64_t row0, float* y, int64_t ldy, void* stream) {
  GMR_ARG(x && y && rows > 0 && D > 0 && group >= 1 && D % group == 0 && row0 >= 0, "bad args");
  GMR_ARG(p_keep > 0.f && p_keep <= 1.f, "p_keep in (0, 1]");
  GMR_ARG(rows * D < (1ll << 31), "rows * D too large");
  const int64_t nthreads = group == 1 ? ph_quads(row0 * D, rows * D) : rows * D;
  hipLaunchKernelGGL(dropout_kernel, dim3(gmr::grid_for(nthreads, 256)), dim3(256), 0, (hipStream_t)stream, rows, D,
                     group, x, ldx, p_keep, mask_in, mask_out, ldm, seed, step, row0, y, ldy);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_xattn_table_f32(int32_t L, int32_t D, int32_t nhead, const float* woc0, const float* bvc0,
                                   int64_t layer_stride, float p_keep, float* P, void* stream) {
  GMR_ARG(woc0 && bvc0 && P && L > 0 && D > 0 && nhead > 0 && nhead <= 64 && D % nhead == 0, "bad args");
  GMR_ARG(p_keep > 0.f && p_keep <= 1.f, "p_keep in (0, 1]");
  const int64_t n = (int64_t)L * nhead * D;
  hipLaunchKernelGGL(xattn_table_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, L, D, nhead,
                     woc0, bvc0, layer_stride, p_keep, P);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_xattn_fwd_f32(int64_t rows, int32_t D, int32_t nhead, const float* P, const float* bo, float p_keep,
                                 const uint8_t* mask_in, uint8_t* mask_out, int64_t ldm, uint64_t seed, uint64_t step,
                                 int64_t row0, float* CA, int64_t ldc, void* stream) {
  GMR_ARG(P && bo && CA && rows > 0 && rows < (1ll << 31) && D > 0 && nhead > 0 && nhead <= 64 && D % nhead == 0 &&
              ldm >= nhead && ldc >= D && row0 >= 0,
          "bad args");
  GMR_ARG(p_keep > 0.f && p_keep <= 1.f, "p_keep in (0, 1]");
  hipLaunchKernelGGL(xattn_fwd_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, D, nhead, P, bo, p_keep,
                     mask_in, mask_out, ldm, seed, step, row0, CA, ldc);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int64_t gmr_xattn_bwd_workspace_floats(int64_t rows, int32_t D, int32_t nhead) {
  const int64_t chunks = std::min<int64_t>(32, std::max<int64_t>(1, (rows + 127) / 128));
  return chunks * nhead * D + (int64_t)nhead * D;
}

extern "C" int gmr_xattn_bwd_f32(int64_t rows, int32_t D, int32_t nhead, const float* dCA, int64_t ld,
                                 const uint8_t* mask, int64_t ldm, const float* wo, const float* bv, float p_keep,
                                 float* g_wo, float* g_bv, float* ws, int64_t ws_floats, void* stream) {
  GMR_ARG(dCA && mask && wo && bv && g_wo && g_bv && ws && rows > 0 && D > 0 && nhead > 0 &&
              nhead <= kXattnMaxHeads && D % nhead == 0 && ld >= D && ldm >= nhead,
          "bad args");
  GMR_ARG(p_keep > 0.f && p_keep <= 1.f, "p_keep in (0, 1]");
  GMR_ARG(ws_floats >= gmr_xattn_bwd_workspace_floats(rows, D, nhead), "workspace too small");
  const int64_t chunks = std::min<int64_t>(32, std::max<int64_t>(1, (rows + 127) / 128));
  const int64_t chunk = (rows + chunks - 1) / chunks;
  float* part = ws;
  float* G = ws + chunks * nhead * D;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(xattn_bwd_part_kernel, dim3((unsigned)((D + 63) / 64), (unsigned)chunks), dim3(256), 0, st, rows, D,
                     nhead, dCA, ld, mask, ldm, chunk, part);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(xattn_bwd_reduce_kernel, dim3(gmr::grid_for((int64_t)nhead * D, 256)), dim3(256), 0, st, D, nhead,
                     (int)chunks, part, G);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(xattn_bwd_apply_kernel,
                     dim3((unsigned)((D + kXattnBvCols - 1) / kXattnBvCols + gmr::grid_for((int64_t)D * D, 256))),
                     dim3(256), 0, st, D, nhead,
                     G, wo, bv, p_keep, g_wo, g_bv);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_time_embedding(int32_t T, int32_t E, float* out, void* stream) {
  GMR_ARG(out && T > 0 && E > 0, "bad args");
  hipLaunchKernelGGL(time_embedding_kernel, dim3(gmr::grid_for((int64_t)T * E, 256)), dim3(256), 0,
                     (hipStream_t)stream, T, E, out);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_silu_f32(int64_t n, const float* x, const float* dy, float* y, void* stream) {
  GMR_ARG(x && y && n > 0, "bad args");
  hipLaunchKernelGGL(silu_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, x, dy, y);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_flip_total(const double* bce_kl, const float* cl, float w_cl, float* out4, void* stream) {
  GMR_ARG(bce_kl && cl && out4, "bad args");
  hipLaunchKernelGGL(flip_total_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, bce_kl, cl, w_cl, out4);
  GMR_LAUNCHED();
  return GMR_OK;
}
