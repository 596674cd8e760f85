// K5 / K6 — Gaussian diffusion over per-user interaction vectors (gfx950).
//
// Reference: GaussianDiffusion.q_sample / training_losses / p_sample and Denoise.forward
// (models/diffmm.py:340-484; models/diffrec.py:75-310).  The denoiser GEMMs themselves
// run in gemm.hip; this file holds the row-wise pieces around them:
//   * q_sample fused with the x0 densification (from the train CSR), N(0,1) noise and the
//     p = 0.5 input dropout of Denoise (train mode), written straight into the GEMM input.
//     Noise / keep mask / timesteps come from Philox (or caller buffers for parity tests).
//   * per-timestep input bias EB[t] = emb_layer(temb(t)) @ W1[:, I:]^T + b1: the time
//     embedding only takes T distinct values, so the concat([x, emb]) columns of the first
//     Linear collapse into a T x H bias table indexed by t in the GEMM epilogue.
//   * the loss rows (mse with SNR weight, gc loss) and the first dout term.
#include "gmr_common.h"

namespace {

__device__ __forceinline__ bool in_row(const int* __restrict__ items, int beg, int end, int v) {
  int lo = beg, hi = end;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (items[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo < end && items[lo] == v;
}

struct Draw4 {
  float eps[4];
  float keep[4];
};

// noise and keep-mask of the 4 columns [c4*4, c4*4+4) of row b, step `step`
__device__ __forceinline__ Draw4 draw4(uint64_t seed, uint64_t step, int64_t b, int64_t c4, float keep_prob) {
  Draw4 d;
  const uint64_t off = ((uint64_t)b << 24) ^ (uint64_t)c4;
  uint4 r = gmr::Philox::gen(seed, step * 2 + 0, off);
  float2 n0 = gmr::box_muller(r.x, r.y), n1 = gmr::box_muller(r.z, r.w);
  d.eps[0] = n0.x;
  d.eps[1] = n0.y;
  d.eps[2] = n1.x;
  d.eps[3] = n1.y;
  uint4 q = gmr::Philox::gen(seed, step * 2 + 1, off);
  d.keep[0] = gmr::u32_to_unit(q.x) <= keep_prob ? 1.f : 0.f;
  d.keep[1] = gmr::u32_to_unit(q.y) <= keep_prob ? 1.f : 0.f;
  d.keep[2] = gmr::u32_to_unit(q.z) <= keep_prob ? 1.f : 0.f;
  d.keep[3] = gmr::u32_to_unit(q.w) <= keep_prob ? 1.f : 0.f;
  return d;
}

__global__ void sample_t_kernel(int B, int T, uint64_t seed, uint64_t step, int64_t row0, int* __restrict__ t) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  uint4 r = gmr::Philox::gen(seed ^ 0xA5A5A5A5ull, step, (uint64_t)(row0 + b));
  t[b] = (int)(((uint64_t)r.x * (uint64_t)T) >> 32);
}

// dense part: x0 = 0 everywhere -> x_in = (s1[t] * eps) * keep/kp ; sparse part fixes the ones
__global__ void qsample_dense_kernel(int B, int I, const int* __restrict__ t, const float* __restrict__ sa,
                                     const float* __restrict__ s1, const float* __restrict__ noise, int64_t ld_noise,
                                     const float* __restrict__ keep, int64_t ld_keep, float keep_prob, int dropout,
                                     uint64_t seed, uint64_t step, int64_t row0, float* __restrict__ x, int64_t ldx) {
  const int64_t c4n = (I + 3) / 4;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)B * c4n) return;
  const int64_t b = gid / c4n, c4 = gid % c4n;
  const int tb = t[b];
  const float s1v = s1[tb];
  Draw4 d;
  if (!noise || (dropout && !keep)) d = draw4(seed, step, row0 + b, c4, keep_prob);
  const float kscale = 1.f / keep_prob;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t c = c4 * 4 + j;
    if (c >= I) break;
    const float e = noise ? noise[b * ld_noise + c] : d.eps[j];
    float v = s1v * e;
    if (dropout) v = v * ((keep ? keep[b * ld_keep + c] : d.keep[j]) * kscale);
    x[b * ldx + c] = v;
  }
}

__global__ void qsample_sparse_kernel(int B, const int* __restrict__ users, const int* __restrict__ uptr,
                                      const int* __restrict__ uitems, const int* __restrict__ t,
                                      const float* __restrict__ sa, const float* __restrict__ s1,
                                      const float* __restrict__ noise, int64_t ld_noise, const float* __restrict__ keep,
                                      int64_t ld_keep, float keep_prob, int dropout, uint64_t seed, uint64_t step,
                                      int64_t row0, float* __restrict__ x, int64_t ldx) {
  const int b = blockIdx.x;
  if (b >= B) return;
  const int u = users[b];
  const int tb = t[b];
  const float sav = sa[tb], s1v = s1[tb];
  const float kscale = 1.f / keep_prob;
  for (int e = uptr[u] + threadIdx.x; e < uptr[u + 1]; e += blockDim.x) {
    const int64_t c = uitems[e];
    const int64_t c4 = c >> 2;
    Draw4 d;
    if (!noise || (dropout && !keep)) d = draw4(seed, step, row0 + b, c4, keep_prob);
    const float eps = noise ? noise[b * ld_noise + c] : d.eps[c & 3];
    float v = sav * 1.0f + s1v * eps;
    if (dropout) v = v * ((keep ? keep[b * ld_keep + c] : d.keep[c & 3]) * kscale);
    x[b * ldx + c] = v;
  }
}

// x0 rows: zero then ones at the user's train items
__global__ void densify_zero_kernel(int B, int I, float* __restrict__ x, int64_t ldx) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)B * I) return;
  x[(gid / I) * ldx + gid % I] = 0.f;
}

__global__ void densify_ones_kernel(int B, const int* __restrict__ users, const int* __restrict__ uptr,
                                    const int* __restrict__ uitems, float* __restrict__ x, int64_t ldx) {
  const int b = blockIdx.x;
  const int u = users ? users[b] : b;
  for (int e = uptr[u] + threadIdx.x; e < uptr[u + 1]; e += blockDim.x) x[(int64_t)b * ldx + uitems[e]] = 1.f;
}

// EB[t][h] = sum_j emb[t][j] * W1[h][off + j] + b1[h],  emb[t] = emb_W @ temb(t) + emb_b
// One block per timestep t: the E-dim sinusoidal embedding and emb_layer(temb) go to LDS once
// (thread j / i), then EB[t][h] = W1[h, off:off+E] . emb[t] + b1[h] over the block's threads.
// (one thread per (t, h) recomputing the E x E emb_layer product was 0.43 ms at DiffRec's
// T = 100, E = 64, H = 300.)
__global__ void __launch_bounds__(256) time_bias_kernel(int T, int E, const float* __restrict__ embW,
                                                        const float* __restrict__ embB, const float* __restrict__ W1,
                                                        int64_t ldw, int64_t off, const float* __restrict__ b1, int H,
                                                        float* __restrict__ EB, float* __restrict__ temb_out,
                                                        float* __restrict__ emb_out) {
  __shared__ float te[64], em[64];
  const int t = blockIdx.x, tid = threadIdx.x;
  const int half = E / 2;
  if (tid < E) {
    float v = 0.f;
    if (tid < 2 * half) {
      const int j = tid < half ? tid : tid - half;
      const float a = (float)t * expf(-9.210340371976184f * (float)j / (float)half);  // ln(10000)
      v = tid < half ? cosf(a) : sinf(a);
    }
    te[tid] = v;
    if (temb_out) temb_out[t * E + tid] = v;
  }
  __syncthreads();
  if (tid < E) {
    float s = 0.f;
    for (int j = 0; j < E; ++j) s = fmaf(embW[tid * E + j], te[j], s);
    em[tid] = s + embB[tid];
    if (emb_out) emb_out[t * E + tid] = s + embB[tid];
  }
  __syncthreads();
  for (int h = tid; h < H; h += blockDim.x) {
    const float* w = W1 + (int64_t)h * ldw + off;
    float acc = 0.f;
    for (int j = 0; j < E; ++j) acc = fmaf(em[j], w[j], acc);
    EB[(int64_t)t * H + h] = acc + b1[h];
  }
}

// One block per row: d = out - x0 ; mse_b = mean(d^2);  out <- ca_b * d  (first dout term)
// diff_b = w[t_b] * mse_b (double).  ca_b = w[t_b] * 2 / (I * B) * scale.
__global__ void __launch_bounds__(256) loss_rows_kernel(int B, int I, const int* __restrict__ users,
                                                        const int* __restrict__ uptr, const int* __restrict__ uitems,
                                                        const int* __restrict__ t, const double* __restrict__ wtab,
                                                        const float* __restrict__ pt, float* __restrict__ out,
                                                        int64_t ld, float grad_scale, double* __restrict__ mse_out,
                                                        double* __restrict__ diff_out, double* __restrict__ loss_out,
                                                        int write_grad) {
  extern __shared__ __attribute__((aligned(16))) uint32_t bits[];
  const int b = blockIdx.x;
  const int u = users[b];
  const int nw = (I + 31) / 32;
  for (int i = threadIdx.x; i < nw; i += 256) bits[i] = 0u;
  __syncthreads();
  for (int e = uptr[u] + threadIdx.x; e < uptr[u + 1]; e += 256) {
    const int c = uitems[e];
    atomicOr(&bits[c >> 5], 1u << (c & 31));
  }
  __syncthreads();
  const double w = wtab[t[b]];
  const double div = pt ? (double)pt[b] : 1.0;
  const float ca = (float)(w / div * 2.0 / (double)I) * grad_scale;
  float* row = out + (int64_t)b * ld;
  float s = 0.f;
  for (int i = threadIdx.x; i < I; i += 256) {
    const float x0 = (bits[i >> 5] >> (i & 31)) & 1u ? 1.f : 0.f;
    const float d = row[i] - x0;
    s = fmaf(d, d, s);
    if (write_grad) row[i] = ca * d;
  }
  __shared__ float red[4];
  s = gmr::wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double mse = (double)((red[0] + red[1]) + (red[2] + red[3])) / (double)I;
    mse_out[b] = mse;
    diff_out[b] = w * mse;
    if (loss_out) loss_out[b] = w * mse / div;
  }
}

// gc term: Y = x0 @ iE (sum of the user's item rows), D = Z - Y;  gc_b = mean(D^2) ;
// G = gscale * D  (B x 64, feeds dout += G @ feats^T).  One 64-lane wave per row.
__global__ void gc_rows_kernel(int B, const int* __restrict__ users, const int* __restrict__ uptr,
                               const int* __restrict__ uitems, const float* __restrict__ iE, int64_t ld_ie,
                               const float* __restrict__ Z, int64_t ldz, float gscale, float* __restrict__ G,
                               int64_t ldg, double* __restrict__ gc_out) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63;
  const int u = users[b];
  float y = 0.f;
  for (int e = uptr[u]; e < uptr[u + 1]; ++e) y += iE[(int64_t)uitems[e] * ld_ie + lane];
  const float d = Z[(int64_t)b * ldz + lane] - y;
  const float s = gmr::wave_sum(d * d);
  if (G) G[(int64_t)b * ldg + lane] = gscale * d;
  if (lane == 0) gc_out[b] = (double)s / 64.0;
}

// deterministic column sums: out[g][c] (+)= sum_{r: group[r] == g} x[r][c].
// One block = 64 columns x 16 waves; wave w takes rows w, w+16, ...; each lane keeps the sums of
// up to GMAX groups in registers; waves are combined in a fixed order through LDS.
template <int GMAX>
__global__ void __launch_bounds__(1024) colsum_kernel(int64_t rows, int64_t cols, const float* __restrict__ x,
                                                      int64_t ld, const int* __restrict__ group, int n_groups,
                                                      float* __restrict__ out, int accumulate) {
  __shared__ float red[16][GMAX][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  float s[GMAX];
#pragma unroll
  for (int q = 0; q < GMAX; ++q) s[q] = 0.f;
  if (c < cols) {
#pragma unroll 4
    for (int64_t r = w; r < rows; r += 16) {
      const float v = x[r * ld + c];
      const int gr = group ? group[r] : 0;
#pragma unroll
      for (int q = 0; q < GMAX; ++q) s[q] += (gr == q) ? v : 0.f;
    }
  }
#pragma unroll
  for (int q = 0; q < GMAX; ++q) red[w][q][lane] = s[q];
  __syncthreads();
  if (w < n_groups && w < GMAX && c < cols) {
    float v = 0.f;
    for (int k = 0; k < 16; ++k) v += red[k][w][lane];
    float* o = out + (int64_t)w * cols + c;
    *o = accumulate ? *o + v : v;
  }
}

// few column blocks (cols <= 64 * 32): rows split over blockIdx.y into fixed-order partials, then
// a second pass adds the partials in split order (deterministic)
constexpr int kColSplits = 32;
__global__ void __launch_bounds__(256) colsum_split_kernel(int64_t rows, int64_t cols, const float* __restrict__ x,
                                                           int64_t ld, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  const int64_t rc = (rows + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = (int64_t)blockIdx.y * rc, r1 = r0 + rc < rows ? r0 + rc : rows;
  float s = 0.f;
  if (c < cols)
    for (int64_t r = r0 + w; r < r1; r += 4) s += x[r * ld + c];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < cols) part[(int64_t)blockIdx.y * cols + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// rows <= 4096, cols % 4 == 0, 16-byte rows: one 1024-thread workgroup per 64 columns; a lane group of 16
// lanes reads one row's 64 columns as float4, so a wave covers 4 rows and the workgroup 64 rows per pass,
// eight passes unrolled (their loads in flight together); the 64 partial rows meet in a fixed LDS order.
// One launch (the split + finish pair cost 15 + 10 us at 2048 x 512).
__global__ void __launch_bounds__(1024) colsum_wide_kernel(int64_t rows, int64_t cols, const float* __restrict__ x,
                                                           int64_t ld, float* __restrict__ out, int accumulate) {
  __shared__ float4 red[64][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane & 15, rr = 4 * w + (lane >> 4);  // column quad, row slot (0..63)
  const int64_t c = (int64_t)blockIdx.x * 64 + 4 * q;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < cols) {
    int64_t r = rr;
    for (; r + 7 * 64 < rows; r += 8 * 64) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(x + (r + 64 * u) * ld + c);
#pragma unroll
      for (int u = 0; u < 8; ++u) s = gmr::f4_add(s, v[u]);
    }
    for (; r < rows; r += 64) s = gmr::f4_add(s, *reinterpret_cast<const float4*>(x + r * ld + c));
  }
  red[rr][q] = s;
  __syncthreads();
  if (threadIdx.x < 64) {  // column blockIdx.x * 64 + threadIdx.x: its 64 row-slot partials in order
    const int cq = threadIdx.x >> 2, ce = threadIdx.x & 3;
    const int64_t cc = (int64_t)blockIdx.x * 64 + threadIdx.x;
    float t = 0.f;
    for (int j = 0; j < 64; ++j) {
      const float4 p = red[j][cq];
      t += ce == 0 ? p.x : ce == 1 ? p.y : ce == 2 ? p.z : p.w;
    }
    if (cc < cols) out[cc] = accumulate ? out[cc] + t : t;
  }
}

__global__ void colsum_split_fin_kernel(int64_t cols, int S, const float* __restrict__ part, float* __restrict__ out,
                                        int accumulate) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int j = 0; j < S; ++j) s += part[(int64_t)j * cols + c];
  out[c] = accumulate ? out[c] + s : s;
}

// generic fallback (many groups): one group per blockIdx.y
__global__ void __launch_bounds__(256) colsum_grouped_kernel(int64_t rows, int64_t cols, const float* __restrict__ x,
                                                             int64_t ld, const int* __restrict__ group,
                                                             float* __restrict__ out, int accumulate) {
  __shared__ float red[4][64];
  const int64_t c = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  const int g = blockIdx.y;
  float s = 0.f;
  if (c < cols)
    for (int64_t r = w; r < rows; r += 4)
      if (group[r] == g) s += x[r * ld + c];
  red[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && c < cols) {
    float v = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    float* o = out + (int64_t)g * cols + c;
    *o = accumulate ? *o + v : v;
  }
}

// time-embedding backward from S[t][h] = sum_{b: t_b = t} dpre[b][h]:
//   dW1[h][off + j] (+)= sum_t S[t][h] emb[t][j] ; db1[h] (+)= sum_t S[t][h]
//   demb[t][j] = sum_h S[t][h] W1[h][off + j] ; d emb_W[i][j] = sum_t demb[t][i] temb[t][j] ; d emb_b[i] = sum_t demb[t][i]
// One thread per (h, j) output of dW1 (the j = 0 thread also sums db1[h]); every sum runs over t
// in order, as before.
__global__ void __launch_bounds__(256) time_bwd_h_kernel(int T, int E, int H, const float* __restrict__ S,
                                                         const float* __restrict__ emb, float* __restrict__ dW1,
                                                         int64_t ldw, int64_t off, float* __restrict__ db1,
                                                         int accumulate) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= (int64_t)H * E) return;
  const int h = (int)(o / E), j = (int)(o % E);
  float a = 0.f;
  for (int t = 0; t < T; ++t) a = fmaf(S[(int64_t)t * H + h], emb[t * E + j], a);
  float* d = dW1 + (int64_t)h * ldw + off + j;
  *d = accumulate ? *d + a : a;
  if (j == 0) {
    float sb = 0.f;
    for (int t = 0; t < T; ++t) sb += S[(int64_t)t * H + h];
    db1[h] = accumulate ? db1[h] + sb : sb;
  }
}

// demb[t][i] = sum_h S[t][h] W1[h][off+i]: a wave per output (t, i), its lanes splitting h (lane l sums
// h = l, l + 64, ... in four chains, then a fixed xor butterfly: deterministic); one thread per (t, i)
// with a serial h loop took 115 us at T x E = 50, H = 1000.  Then
// d emb_W[i][j] = sum_t demb[t][i] temb[t][j], d emb_b[i] = sum_t demb[t][i]
// FEW (T x E <= 64): a wave per output; else a thread per output
template <bool FEW>
__global__ void __launch_bounds__(1024) time_bwd_e_kernel(int T, int E, int H, const float* __restrict__ S,
                                                          const float* __restrict__ W1, int64_t ldw, int64_t off,
                                                          const float* __restrict__ temb, float* __restrict__ dembW,
                                                          float* __restrict__ dembB, int accumulate) {
  extern __shared__ __attribute__((aligned(16))) float demb[];  // T * E
  constexpr int kTbeThreads = 1024;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if constexpr (!FEW) {  // many outputs (DiffRec: T = 100): one thread per output, a serial h loop in 4 chains
    for (int o = threadIdx.x; o < T * E; o += kTbeThreads) {
      const int t = o / E, i = o % E;
      const float* srow = S + (int64_t)t * H;
      const float* wcol = W1 + off + i;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
      int h = 0;
      for (; h + 4 <= H; h += 4) {
        a0 = fmaf(srow[h], wcol[(int64_t)h * ldw], a0);
        a1 = fmaf(srow[h + 1], wcol[(int64_t)(h + 1) * ldw], a1);
        a2 = fmaf(srow[h + 2], wcol[(int64_t)(h + 2) * ldw], a2);
        a3 = fmaf(srow[h + 3], wcol[(int64_t)(h + 3) * ldw], a3);
      }
      for (; h < H; ++h) a0 = fmaf(srow[h], wcol[(int64_t)h * ldw], a0);
      demb[o] = (a0 + a1) + (a2 + a3);
    }
  } else {  // few outputs (DiffMM: T x E = 50, H = 1000): a wave per output, its lanes splitting h
    // (lane l sums h = l, l + 64, ... in four chains, then a fixed xor butterfly: deterministic).  A lane
    // per h holding all T x E sums in registers measured slower (52.8 vs 32.5 us: 100 loads per h)
    for (int o = wv; o < T * E; o += kTbeThreads / 64) {
      const int t = o / E, i = o % E;
      const float* srow = S + (int64_t)t * H;
      const float* wcol = W1 + off + i;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
      int h = lane;
      for (; h + 192 < H; h += 256) {
        a0 = fmaf(srow[h], wcol[(int64_t)h * ldw], a0);
        a1 = fmaf(srow[h + 64], wcol[(int64_t)(h + 64) * ldw], a1);
        a2 = fmaf(srow[h + 128], wcol[(int64_t)(h + 128) * ldw], a2);
        a3 = fmaf(srow[h + 192], wcol[(int64_t)(h + 192) * ldw], a3);
      }
      for (; h < H; h += 64) a0 = fmaf(srow[h], wcol[(int64_t)h * ldw], a0);
      const float v = gmr::wave_sum((a0 + a1) + (a2 + a3));
      if (lane == 0) demb[o] = v;
    }
  }
  __syncthreads();
  for (int o = threadIdx.x; o < E * E; o += kTbeThreads) {
    const int i = o / E, j = o % E;
    float a = 0.f;
    for (int t = 0; t < T; ++t) a = fmaf(demb[t * E + i], temb[t * E + j], a);
    dembW[o] = accumulate ? dembW[o] + a : a;
  }
  for (int i = threadIdx.x; i < E; i += kTbeThreads) {
    float a = 0.f;
    for (int t = 0; t < T; ++t) a += demb[t * E + i];
    dembB[i] = accumulate ? dembB[i] + a : a;
  }
}

// DiffRec GaussianDiffusion.sample_timesteps (models/diffrec.py:234-250).  Until every t has a
// full loss history: uniform t (same Philox stream as sample_t_kernel) and pt = 1.  Then
// pt_all = (1 - up) * sqrt(mean(hist^2)) / sum + up / T, t ~ pt_all (inverse CDF), pt = pt_all[t] * T.
// One 1024-thread block; T <= 1024.
__global__ void __launch_bounds__(1024) sample_t_importance_kernel(int B, int T, int Hn, const double* __restrict__ hist,
                                                                  const int* __restrict__ count, double uniform_prob,
                                                                  uint64_t seed, uint64_t step, int64_t row0,
                                                                  int* __restrict__ t, float* __restrict__ pt) {
  __shared__ double cdf[1024];
  __shared__ double pall[1024];
  const int i = threadIdx.x;
  const int full = __syncthreads_and(i >= T || count[i] == Hn);
  if (!full) {
    for (int b = i; b < B; b += 1024) {
      uint4 r = gmr::Philox::gen(seed ^ 0xA5A5A5A5ull, step, (uint64_t)(row0 + b));
      t[b] = (int)(((uint64_t)r.x * (uint64_t)T) >> 32);
      pt[b] = 1.f;
    }
    return;
  }
  if (i < T) {
    double m = 0.0;
    for (int j = 0; j < Hn; ++j) m += hist[(int64_t)i * Hn + j] * hist[(int64_t)i * Hn + j];
    pall[i] = sqrt(m / (double)Hn);
  }
  __syncthreads();
  if (i == 0) {
    double tot = 0.0;
    for (int j = 0; j < T; ++j) tot += pall[j];
    double run = 0.0;
    for (int j = 0; j < T; ++j) {
      pall[j] = pall[j] / tot * (1.0 - uniform_prob) + uniform_prob / (double)T;
      run += pall[j];
      cdf[j] = run;
    }
  }
  __syncthreads();
  for (int b = i; b < B; b += 1024) {
    uint4 r = gmr::Philox::gen(seed ^ 0x5EED5EEDull, step, (uint64_t)(row0 + b));
    const double u = (((uint64_t)r.x << 21) ^ (uint64_t)(r.y >> 11)) * (1.0 / 9007199254740992.0) * cdf[T - 1];
    int lo = 0, hi = T - 1;  // first j with cdf[j] > u
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid] > u) hi = mid; else lo = mid + 1;
    }
    t[b] = lo;
    pt[b] = (float)(pall[lo] * (double)T);
  }
}

// Lt_history / Lt_count update of training_losses (models/diffrec.py:279-286), with the
// reference's per-sample sequential semantics: the rows of the batch are applied in order
// (rows with t < 0 are padding and skipped), so timestep i ends up with the latest Hn losses of
// its rows.  The batch's t go to LDS; wave w handles timesteps w, w + 16, ...: it scans the batch
// from the end 64 rows at a time with a ballot and takes the latest matches (at most Hn) from the
// mask, latest first, into its LDS list; then its lanes write the history.
__global__ void __launch_bounds__(1024) lt_update_kernel(int B, int T, int Hn, const int* __restrict__ t,
                                                         const double* __restrict__ loss, double* __restrict__ hist,
                                                         int* __restrict__ count) {
  extern __shared__ int st[];  // B timesteps
  __shared__ int keep[16][16];
  for (int b = threadIdx.x; b < B; b += 1024) st[b] = t[b];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < T; i += 16) {
    int seen = 0;  // uniform over the wave
    for (int end = B; end > 0 && seen < Hn; end -= 64) {
      const int b = end - 64 + lane;
      const unsigned long long m = __ballot(b >= 0 && st[b] == i);
      unsigned long long rest = m;
      while (rest && seen < Hn) {  // latest match first: highest set bit
        const int bit = 63 - __clzll(rest);
        if (lane == 0) keep[w][seen] = end - 64 + bit;
        rest &= ~(1ull << bit);
        ++seen;
      }
    }
    if (seen == 0) continue;
    double* h = hist + (int64_t)i * Hn;
    const int c = count[i];
    if (c + seen <= Hn && seen < Hn) {  // (seen == Hn may mean more matches: always the shift branch)
      if (lane < seen) h[c + lane] = loss[keep[w][seen - 1 - lane]];
      if (lane == 0) count[i] = c + seen;
    } else {
      const int kn = min(seen, Hn), ko = Hn - kn;
      const double old = lane < ko ? h[c - ko + lane] : 0.0;  // all reads before any write
      if (lane < ko) h[lane] = old;
      if (lane < kn) h[ko + lane] = loss[keep[w][kn - 1 - lane]];
      if (lane == 0) count[i] = Hn;
    }
  }
}

// 32x32 LDS-tiled transpose: out[c][r] = in[r][c] (rows x cols, leading dims ldi / ldo).
__global__ void __launch_bounds__(256) transpose_kernel(int64_t rows, int64_t cols, const float* __restrict__ in,
                                                        int64_t ldi, float* __restrict__ out, int64_t ldo) {
  __shared__ float t[32][33];
  const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int64_t r = r0 + ty + k, c = c0 + tx;
    t[ty + k][tx] = (r < rows && c < cols) ? in[r * ldi + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int64_t c = c0 + ty + k, r = r0 + tx;
    if (c < cols && r < rows) out[c * ldo + r] = t[tx][ty + k];
  }
}

// First p_sample step on a binary x0: h[b] = tanh(sum_{i in items(b)} W1T[i] + EB), the sparse
// form of tanh(x0 @ W1[:, :I]^T + EB[t]) (x0 rows hold ~6 ones out of I).  One block per row,
// float4 columns; the items are summed in ascending order.
__global__ void __launch_bounds__(256) sparse_hidden_kernel(int B, int H, const int* __restrict__ users,
                                                            const int* __restrict__ uptr,
                                                            const int* __restrict__ uitems,
                                                            const float* __restrict__ W1T, int64_t ldw,
                                                            const float* __restrict__ eb, float* __restrict__ h,
                                                            int64_t ldh) {
  const int b = blockIdx.x;
  const int u = users[b];
  const int beg = uptr[u], end = uptr[u + 1];
  for (int c = threadIdx.x * 4; c < H; c += 1024) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e = beg; e < end; ++e) acc = gmr::f4_add(acc, *reinterpret_cast<const float4*>(W1T + (int64_t)uitems[e] * ldw + c));
    const float4 bb = *reinterpret_cast<const float4*>(eb + c);
    float4 o = make_float4(tanhf(acc.x + bb.x), tanhf(acc.y + bb.y), tanhf(acc.z + bb.z), tanhf(acc.w + bb.w));
    *reinterpret_cast<float4*>(h + (int64_t)b * ldh + c) = o;
  }
}

// the same gather, keeping the pre-activation a = x0 W1[:, :I]^T (no bias) beside h = tanh(a + eb): the
// first step of the folded p_sample chain (Denoiser.p_sample_fold).  The sum runs in the same order as
// sparse_hidden_kernel, so h is bit-identical to it.
__global__ void __launch_bounds__(256) sparse_pre_kernel(int B, int H, const int* __restrict__ users,
                                                         const int* __restrict__ uptr, const int* __restrict__ uitems,
                                                         const float* __restrict__ W1T, int64_t ldw,
                                                         const float* __restrict__ eb, float* __restrict__ a,
                                                         int64_t lda, float* __restrict__ h, int64_t ldh) {
  const int b = blockIdx.x;
  const int u = users[b];
  const int beg = uptr[u], end = uptr[u + 1];
  for (int c = threadIdx.x * 4; c < H; c += 1024) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e = beg; e < end; ++e) acc = gmr::f4_add(acc, *reinterpret_cast<const float4*>(W1T + (int64_t)uitems[e] * ldw + c));
    const float4 bb = *reinterpret_cast<const float4*>(eb + c);
    *reinterpret_cast<float4*>(a + (int64_t)b * lda + c) = acc;
    float4 o = make_float4(tanhf(acc.x + bb.x), tanhf(acc.y + bb.y), tanhf(acc.z + bb.z), tanhf(acc.w + bb.w));
    *reinterpret_cast<float4*>(h + (int64_t)b * ldh + c) = o;
  }
}

// h = tanh(a + bias) (rows x cols, cols % 4 == 0), float4 per thread
__global__ void __launch_bounds__(256) tanh_bias_kernel(int64_t rows, int cols, const float* __restrict__ a,
                                                        int64_t lda, const float* __restrict__ bias,
                                                        float* __restrict__ h, int64_t ldh) {
  const int c4 = cols / 4;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < rows * c4; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = g / c4;
    const int c = (int)(g % c4) * 4;
    const float4 x = *reinterpret_cast<const float4*>(a + r * lda + c);
    const float4 bb = *reinterpret_cast<const float4*>(bias + c);
    *reinterpret_cast<float4*>(h + r * ldh + c) =
        make_float4(tanhf(x.x + bb.x), tanhf(x.y + bb.y), tanhf(x.z + bb.z), tanhf(x.w + bb.w));
  }
}

}  // namespace

extern "C" int gmr_diff_sparse_pre(int32_t B, int32_t H, const int32_t* users, const int32_t* user_ptr,
                                   const int32_t* user_items, const float* W1T, int64_t ldw, const float* eb, float* a,
                                   int64_t lda, float* h, int64_t ldh, void* stream) {
  GMR_ARG(users && user_ptr && user_items && W1T && eb && a && h && B > 0 && H > 0, "bad args");
  GMR_ARG(H % 4 == 0 && ldw % 4 == 0 && lda % 4 == 0 && ldh % 4 == 0, "H and the leading dims must be multiples of 4");
  GMR_ARG((((uintptr_t)W1T | (uintptr_t)eb | (uintptr_t)a | (uintptr_t)h) & 15) == 0, "16-byte alignment");
  hipLaunchKernelGGL(sparse_pre_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, B, H, users, user_ptr, user_items,
                     W1T, ldw, eb, a, lda, h, ldh);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_tanh_bias_f32(int64_t rows, int32_t cols, const float* a, int64_t lda, const float* bias, float* h,
                                 int64_t ldh, void* stream) {
  GMR_ARG(a && bias && h && rows >= 0 && cols > 0, "bad args");
  GMR_ARG(cols % 4 == 0 && lda % 4 == 0 && ldh % 4 == 0, "cols and the leading dims must be multiples of 4");
  GMR_ARG((((uintptr_t)a | (uintptr_t)bias | (uintptr_t)h) & 15) == 0, "16-byte alignment");
  if (rows == 0) return GMR_OK;
  hipLaunchKernelGGL(tanh_bias_kernel, dim3(gmr::grid_for(rows * (cols / 4), 256, 16384)), dim3(256), 0,
                     (hipStream_t)stream, rows, cols, a, lda, bias, h, ldh);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_diff_sample_t(int32_t B, int32_t T, uint64_t seed, uint64_t step, int64_t row0, int32_t* t,
                                 void* stream) {
  GMR_ARG(t && B > 0 && T > 0 && row0 >= 0, "bad args");
  hipLaunchKernelGGL(sample_t_kernel, dim3(gmr::grid_for(B, 256)), dim3(256), 0, (hipStream_t)stream, B, T, seed, step,
                     row0, t);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_diff_sample_t_importance(int32_t B, int32_t T, int32_t hist_len, const double* hist,
                                            const int32_t* count, double uniform_prob, uint64_t seed, uint64_t step,
                                            int64_t row0, int32_t* t, float* pt, void* stream) {
  GMR_ARG(hist && count && t && pt && B > 0 && T > 0 && T <= 1024 && row0 >= 0, "bad args (T <= 1024)");
  GMR_ARG(hist_len >= 1 && hist_len <= 16, "history length must be 1..16");
  hipLaunchKernelGGL(sample_t_importance_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, B, T, hist_len, hist,
                     count, uniform_prob, seed, step, row0, t, pt);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_diff_history_update(int32_t B, int32_t T, int32_t hist_len, const int32_t* t, const double* loss,
                                       double* hist, int32_t* count, void* stream) {
  GMR_ARG(t && loss && hist && count && B > 0 && T > 0 && T <= 1024, "bad args (T <= 1024)");
  GMR_ARG(hist_len >= 1 && hist_len <= 16, "history length must be 1..16");
  GMR_ARG((size_t)B * sizeof(int) <= 65536, "batch too large for the LDS copy of t (B <= 16384)");
  hipLaunchKernelGGL(lt_update_kernel, dim3(1), dim3(1024), sizeof(int) * (size_t)B, (hipStream_t)stream, B, T,
                     hist_len, t, loss, hist, count);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_diff_qsample(int32_t B, int32_t I, const int32_t* users, const int32_t* user_ptr,
                                const int32_t* user_items, const int32_t* t, const float* sqrt_ac,
                                const float* sqrt_1mac, const float* noise, int64_t ld_noise, const float* keep,
                                int64_t ld_keep, float keep_prob, int32_t dropout, uint64_t seed, uint64_t step,
                                int64_t row0, float* x, int64_t ldx, void* stream) {
  GMR_ARG(users && user_ptr && user_items && t && sqrt_ac && sqrt_1mac && x && B > 0 && I > 0 && row0 >= 0,
          "bad args");
  GMR_ARG(keep_prob > 0.f && keep_prob <= 1.f, "keep_prob must be in (0, 1]");
  hipStream_t st = (hipStream_t)stream;
  const int64_t c4n = (I + 3) / 4;
  hipLaunchKernelGGL(qsample_dense_kernel, dim3(gmr::grid_for((int64_t)B * c4n, 256)), dim3(256), 0, st, B, I, t,
                     sqrt_ac, sqrt_1mac, noise, ld_noise, keep, ld_keep, keep_prob, dropout, seed, step, row0, x, ldx);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(qsample_sparse_kernel, dim3(B), dim3(64), 0, st, B, users, user_ptr, user_items, t, sqrt_ac,
                     sqrt_1mac, noise, ld_noise, keep, ld_keep, keep_prob, dropout, seed, step, row0, x, ldx);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_diff_densify(int32_t B, int32_t I, const int32_t* users, const int32_t* user_ptr,
                                const int32_t* user_items, float* x, int64_t ldx, void* stream) {
  GMR_ARG(user_ptr && user_items && x && B > 0 && I > 0, "bad args");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(densify_zero_kernel, dim3(gmr::grid_for((int64_t)B * I, 256)), dim3(256), 0, st, B, I, x, ldx);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(densify_ones_kernel, dim3(B), dim3(64), 0, st, B, users, user_ptr, user_items, x, ldx);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_transpose_f32(int64_t rows, int64_t cols, const float* in, int64_t ldi, float* out, int64_t ldo,
                                 void* stream) {
  GMR_ARG(in && out && rows > 0 && cols > 0 && ldi >= cols && ldo >= rows, "bad args");
  dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32));
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, in, ldi, out, ldo);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_diff_sparse_hidden(int32_t B, int32_t H, const int32_t* users, const int32_t* user_ptr,
                                      const int32_t* user_items, const float* W1T, int64_t ldw, const float* eb,
                                      float* h, int64_t ldh, void* stream) {
  GMR_ARG(users && user_ptr && user_items && W1T && eb && h && B > 0 && H > 0, "bad args");
  GMR_ARG(H % 4 == 0 && ldw % 4 == 0 && ldh % 4 == 0, "H and the leading dims must be multiples of 4");
  GMR_ARG(((uintptr_t)W1T & 15) == 0 && ((uintptr_t)eb & 15) == 0 && ((uintptr_t)h & 15) == 0, "16-byte alignment");
  hipLaunchKernelGGL(sparse_hidden_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, B, H, users, user_ptr,
                     user_items, W1T, ldw, eb, h, ldh);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_diff_time_bias(int32_t T, int32_t E, const float* emb_W, const float* emb_b, const float* W1,
                                  int64_t ld_w1, int64_t col_off, const float* b1, int32_t H, float* EB,
                                  float* temb_out, float* emb_out, void* stream) {
  GMR_ARG(emb_W && emb_b && W1 && b1 && EB && T > 0 && H > 0, "bad args");
  GMR_ARG(E >= 1 && E <= 64, "time embedding size must be 1..64");
  hipLaunchKernelGGL(time_bias_kernel, dim3((unsigned)T), dim3(256), 0, (hipStream_t)stream, T, E,
                     emb_W, emb_b, W1, ld_w1, col_off, b1, H, EB, temb_out, emb_out);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_diff_loss_rows(int32_t B, int32_t I, const int32_t* users, const int32_t* user_ptr,
                                  const int32_t* user_items, const int32_t* t, const double* wtab, const float* pt,
                                  float* out, int64_t ld, float grad_scale, double* mse_out, double* diff_out,
                                  double* loss_out, int32_t write_grad, void* stream) {
  GMR_ARG(users && user_ptr && user_items && t && wtab && out && mse_out && diff_out && B > 0 && I > 0, "bad args");
  const size_t dyn = sizeof(uint32_t) * (size_t)((I + 31) / 32);
  GMR_ARG(dyn <= 60000, "item count too large for the LDS bitmap");
  hipLaunchKernelGGL(loss_rows_kernel, dim3(B), dim3(256), dyn, (hipStream_t)stream, B, I, users, user_ptr, user_items,
                     t, wtab, pt, out, ld, grad_scale, mse_out, diff_out, loss_out, write_grad);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_diff_gc_rows(int32_t B, const int32_t* users, const int32_t* user_ptr, const int32_t* user_items,
                                const float* item_embeds, int64_t ld_ie, const float* Z, int64_t ldz, float gscale,
                                float* G, int64_t ldg, double* gc_out, void* stream) {
  GMR_ARG(users && user_ptr && user_items && item_embeds && Z && gc_out && B > 0, "bad args");
  hipLaunchKernelGGL(gc_rows_kernel, dim3(gmr::grid_for(B, 4)), dim3(256), 0, (hipStream_t)stream, B, users, user_ptr,
                     user_items, item_embeds, ld_ie, Z, ldz, gscale, G, ldg, gc_out);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_colsum_f32(int64_t rows, int64_t cols, const float* x, int64_t ld, const int32_t* group,
                              int32_t n_groups, float* out, int32_t accumulate, void* stream) {
  GMR_ARG(x && out && rows > 0 && cols > 0 && n_groups >= 1, "bad args");
  GMR_ARG(n_groups == 1 || group, "groups need a group array");
  hipStream_t st = (hipStream_t)stream;
  const unsigned gx = (unsigned)((cols + 63) / 64);
  if (n_groups == 1)
    hipLaunchKernelGGL(colsum_kernel<1>, dim3(gx), dim3(1024), 0, st, rows, cols, x, ld, group, 1, out, accumulate);
  else if (n_groups <= 8)
    hipLaunchKernelGGL(colsum_kernel<8>, dim3(gx), dim3(1024), 0, st, rows, cols, x, ld, group, n_groups, out,
                       accumulate);
  else
    hipLaunchKernelGGL(colsum_grouped_kernel, dim3(gx, (unsigned)n_groups), dim3(256), 0, st, rows, cols, x, ld, group,
                       out, accumulate);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_diff_time_bwd(int32_t T, int32_t E, int32_t H, const float* S, const float* temb, const float* emb,
                                 const float* W1, int64_t ld_w1, int64_t col_off, float* dW1, float* db1,
                                 float* d_emb_W, float* d_emb_b, int32_t accumulate, void* stream) {
  GMR_ARG(S && temb && emb && W1 && dW1 && db1 && d_emb_W && d_emb_b && T > 0 && H > 0, "bad args");
  GMR_ARG(E >= 1 && E <= 64, "time embedding size must be 1..64");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(time_bwd_h_kernel, dim3(gmr::grid_for((int64_t)H * E, 256)), dim3(256), 0, st, T, E, H, S, emb, dW1,
                     ld_w1,
                     col_off, db1, accumulate);
  GMR_LAUNCHED();
  GMR_ARG((size_t)T * E * sizeof(float) <= 60000, "T * E too large for the LDS staging");
  if (T * E <= 64)
    hipLaunchKernelGGL(time_bwd_e_kernel<true>, dim3(1), dim3(1024), sizeof(float) * (size_t)T * E, st, T, E, H, S, W1,
                       ld_w1, col_off, temb, d_emb_W, d_emb_b, accumulate);
  else
    hipLaunchKernelGGL(time_bwd_e_kernel<false>, dim3(1), dim3(1024), sizeof(float) * (size_t)T * E, st, T, E, H, S, W1,
                       ld_w1, col_off, temb, d_emb_W, d_emb_b, accumulate);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int64_t gmr_colsum_split_floats(int64_t cols) { return (int64_t)kColSplits * cols; }

extern "C" int gmr_colsum_split_f32(int64_t rows, int64_t cols, const float* x, int64_t ld, float* out,
                                   int32_t accumulate, float* workspace, int64_t workspace_floats, void* stream) {
  GMR_ARG(x && out && workspace && rows > 0 && cols > 0, "bad args");
  GMR_ARG(workspace_floats >= (int64_t)kColSplits * cols, "workspace too small (gmr_colsum_split_floats)");
  hipStream_t st = (hipStream_t)stream;
  const unsigned gx = (unsigned)((cols + 63) / 64);
  if (rows <= 4096 && cols % 4 == 0 && ld % 4 == 0 && ((uintptr_t)x & 15) == 0) {
    hipLaunchKernelGGL(colsum_wide_kernel, dim3(gx), dim3(1024), 0, st, rows, cols, x, ld, out, (int)accumulate);
    GMR_LAUNCHED();
    return GMR_OK;
  }
  hipLaunchKernelGGL(colsum_split_kernel, dim3(gx, kColSplits), dim3(256), 0, st, rows, cols, x, ld, workspace);
  GMR_LAUNCHED();
  hipLaunchKernelGGL(colsum_split_fin_kernel, dim3(gmr::grid_for(cols, 256)), dim3(256), 0, st, cols, kColSplits,
                     workspace, out, (int)accumulate);
  GMR_LAUNCHED();
  return GMR_OK;
}
