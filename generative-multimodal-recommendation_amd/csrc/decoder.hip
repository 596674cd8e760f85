// G5 — GenRecV1's ModalDenoiseTransformer decoder stack in one launch (models/genrecv1.py:650-710).
//
// nn.TransformerDecoder (post-norm, ReLU feed-forward, d_model = dim_feedforward = 512, 8 heads) on a
// length-1 target with an all-zero memory.  Per layer (gmr/transformer.py restates the algebra):
//   SAin = dropout_head(h Wv^T + bv)                 self-attention value (the softmax over one key is 1)
//   h1   = LN1(h + drop1(SAin Wo^T + bo))
//   h2   = LN2(h1 + drop2(CA)),  CA = bo' + sum_h keep_c[h] P[h]   (cross-attention on the zero memory;
//                                                                   eval: every head kept, P without 1/p)
//   F1   = drop_f(relu(h2 W1^T + b1))
//   h'   = LN3(h2 + drop3(F1 W2^T + b2))
// The unfused path runs this as 4 GEMM launches + 6 row kernels per layer.  Here a workgroup owns 32 rows
// (16 with GMR_DEC_ROWS=16)
// and carries them through all L layers in LDS: the four products per layer run on the bf16 matrix
// cores from exact three-way splits (the six products of gemm_x6.hip, fp32-accurate sums; the weights
// arrive pre-split as bf16 planes, gmr_decoder_split_f32, the activations are split in registers at
// fragment load), and the LayerNorms, residual adds, dropouts and the cross-attention mixture are the
// products' epilogues and LDS row passes.  Eight waves, each 64 output columns (= one attention head)
// of every product; the weights stream from L2 with the next 32-deep k step's fragments in flight.
// Dropout masks are read from the mask buffers gmr_decoder_masks_u8 fills with the unfused path's
// Philox keys, so both paths drop the same units.  A training forward (acts != NULL) also stores what the
// layer-by-layer backward reads: every layer's input, SAin, s1 / s2 / s3 with the LayerNorm statistics,
// h2 and F1; the p_sample forwards store only the last layer's rows.
#include <hip/hip_runtime.h>

#include "gmr_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kDD = 512;        // d_model
constexpr int kNH = 8;          // heads (64 columns each)
constexpr int kDW = 8;          // waves per workgroup: wave w owns columns [64 w, 64 w + 64)
constexpr int kDLd = kDD + 4;   // LDS row stride (floats): the 16 rows of a fragment read hit distinct banks
constexpr int64_t kPlane = (int64_t)kDD * kDD;

enum { O_BV, O_BO, O_N1W, O_N1B, O_BOC, O_N2W, O_N2B, O_B1, O_B2, O_N3W, O_N3B, O_COUNT };

struct DecArgs {
  const float* slab;      // the denoiser's parameter slab
  int64_t off[O_COUNT];   // layer 0's offsets (floats) of the vectors above
  int64_t lstride;        // floats between one layer's tensors and the next's
  const __bf16* W;        // weight planes [L][4: Wv, Wo, W1, W2][3][D][D]
  const float* xP;        // [L][NH][D] head vectors of the cross-attention (train: 1 / p_keep folded in)
  const uint8_t *ma, *mc; // [L][Bmax][NH] head masks (self-attention value, cross-attention)
  const uint8_t *m1, *m2, *m3, *mf;  // [L][Bmax][D] residual masks of LN1..3 and the feed-forward mask
  int64_t msh, msd;       // per-layer strides of the head / unit masks
  // STORE (a training forward: the backward reads them): [L+1][Bmax][D] layer inputs / outputs, [L][Bmax][D]
  // SAin (V without dropout), s1, s2, h2, F1, s3, and [L][3][Bmax] LayerNorm means (row 0) / rstds (row 1)
  float *hs, *sa, *s1, *s2, *h2, *f1, *s3, *st1, *st2, *st3;
  int64_t asd, ast, ab;   // strides: activation layer, statistics layer; Bmax (rstd row offset)
};

__device__ __forceinline__ void dec_split8(const float (&v)[8], bf16x8 (&o)[3]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 h = (__bf16)__builtin_amdgcn_fmed3f(v[e], -0x1.fep127f, 0x1.fep127f);
    const float r1 = v[e] - (float)h;  // exact
    const __bf16 m = (__bf16)r1;
    o[0][e] = h;
    o[1][e] = m;
    o[2][e] = (__bf16)(r1 - (float)m);  // exact
  }
}

__device__ __forceinline__ f32x4 dec_mfma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 c) {  // small terms first
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
}

// acc[rt][t] = A (32 x 512, LDS) . W^T for the wave's four 16-column tiles (columns 64 w + 16 t + (lane & 15))
// and both 16-row tiles rt.  Fragments of v_mfma_f32_16x16x32_bf16: lane l holds A[16 rt + (l & 15)][k0 + 8 (l >> 4)
// + j] and W[n][same k]; result element e of lane l is row 16 rt + 4 (l >> 4) + e, column l & 15 of the tile.
template <int kDR>
__device__ __forceinline__ void dec_gemm(const float* A, const __bf16* __restrict__ Wm, f32x4 (&acc)[kDR / 16][4], int w,
                                         int lane) {
  constexpr int kRT = kDR / 16;
  const int row = lane & 15, g = lane >> 4;
  const __bf16* wb = Wm + (int64_t)(64 * w + row) * kDD + 8 * g;
  auto load = [&](bf16x8 (&b)[4][3], int k0) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int p = 0; p < 3; ++p) b[t][p] = *reinterpret_cast<const bf16x8*>(wb + p * kPlane + t * 16 * kDD + k0);
  };
  auto step = [&](const bf16x8 (&b)[4][3], int k0) {
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) {
      const float* ap = A + (16 * rt + row) * kDLd + k0 + 8 * g;
      const float4 x0 = *reinterpret_cast<const float4*>(ap), x1 = *reinterpret_cast<const float4*>(ap + 4);
      const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      bf16x8 a[3];
      dec_split8(v, a);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[rt][t] = dec_mfma6(a, b[t], acc[rt][t]);
    }
  };
#pragma unroll
  for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 b0[4][3], b1[4][3];
  load(b0, 0);
#pragma unroll 1
  for (int k0 = 0; k0 < kDD; k0 += 64) {  // two 32-deep steps per trip: the next step's fragments in flight
    load(b1, k0 + 32);
    step(b0, k0);
    if (k0 + 64 < kDD) load(b0, k0 + 64);
    step(b1, k0 + 32);
  }
}

// LayerNorm of the 32 rows of S into X (four rows per wave; lane holds columns j * 64 + lane, summed in j
// order: ln_fwd_kernel's arithmetic), eps 1e-5
template <int kDR, bool STORE>
__device__ __forceinline__ void dec_ln(const float* S, float* X, const float* __restrict__ wt, const float* __restrict__ bs,
                                       int w, int lane, int64_t r0, int64_t B, float* __restrict__ gx,
                                       float* __restrict__ st, int64_t ab) {
#pragma unroll
  for (int q = 0; q < kDR / kDW; ++q) {
    const int r = (kDR / kDW) * w + q;
    float v[8];
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = S[r * kDLd + j * 64 + lane];
      sum += v[j];
    }
    const float mean = gmr::wave_sum(sum) / (float)kDD;
    float sq = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[j] - mean;
      sq += d * d;
    }
    const float rstd = 1.f / sqrtf(gmr::wave_sum(sq) / (float)kDD + 1e-5f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = j * 64 + lane;
      const float y = (v[j] - mean) * rstd * wt[c] + bs[c];
      X[r * kDLd + c] = y;
      if (STORE && gx && r0 + r < B) gx[(r0 + r) * kDD + c] = y;
    }
    if (STORE && lane == 0 && r0 + r < B) {
      st[r0 + r] = mean;
      st[ab + r0 + r] = rstd;
    }
  }
}

// the 32 rows of an LDS matrix -> rows r0.. of a [Bmax][D] activation buffer (rows < B)
template <int kDR>
__device__ __forceinline__ void dec_store(const float* S, float* __restrict__ g, int64_t r0, int64_t B) {
  for (int i = threadIdx.x; i < kDR * kDD / 4; i += 64 * kDW) {
    const int r = i / (kDD / 4), c4 = (i % (kDD / 4)) * 4;
    if (r0 + r < B) *reinterpret_cast<float4*>(g + (r0 + r) * kDD + c4) = *reinterpret_cast<const float4*>(S + r * kDLd + c4);
  }
}

template <int kDR, bool STORE>
__global__ void __launch_bounds__(64 * kDW, 1) decoder_fwd_kernel(int64_t B, int L, const float* __restrict__ h0,
                                                                  int64_t ld0, float* __restrict__ out, int64_t ldo,
                                                                  DecArgs p, float keep, int train) {
  // X: the residual stream h, h1, h2; Y: the second products' A operand (SAin, F1) and, after a product has
  // read it, the pre-LayerNorm sums s1, s2, s3
  __shared__ __attribute__((aligned(16))) float X[kDR * kDLd];
  __shared__ __attribute__((aligned(16))) float Y[kDR * kDLd];
  constexpr int kRT = kDR / 16;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int64_t r0 = (int64_t)blockIdx.x * kDR;
  for (int i = tid; i < kDR * kDD / 4; i += 64 * kDW) {
    const int r = i / (kDD / 4), c4 = (i % (kDD / 4)) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < B) v = *reinterpret_cast<const float4*>(h0 + (r0 + r) * ld0 + c4);
    *reinterpret_cast<float4*>(X + r * kDLd + c4) = v;
  }
  __syncthreads();
  const float inv_keep = 1.f / keep;
  const int g = lane >> 4, cl = lane & 15;
  // the lane's output rows (clamped for the masks of a ragged last block: those rows are never stored)
  int rg[kRT][4];
#pragma unroll
  for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
    for (int e = 0; e < 4; ++e) rg[rt][e] = (int)min(r0 + 16 * rt + 4 * g + e, B - 1);
  f32x4 acc[kRT][4];
  // epilogue over the wave's fragment elements: f(row in block, global row for masks, column, value)
  auto epi = [&](auto&& f) {
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int c = 64 * w + 16 * t + cl;
#pragma unroll
        for (int e = 0; e < 4; ++e) f(16 * rt + 4 * g + e, rg[rt][e], c, acc[rt][t][e]);
      }
  };
  for (int l = 0; l < L; ++l) {
    const float* P = p.slab + (int64_t)l * p.lstride;
    const __bf16* Wl = p.W + (int64_t)l * 12 * kPlane;
    const uint8_t* ma = p.ma + l * p.msh;
    const uint8_t* m1 = p.m1 + l * p.msd;
    const uint8_t* mf = p.mf + l * p.msd;
    const uint8_t* m3 = p.m3 + l * p.msd;
    // 1. SAin = dropout_head(h Wv^T + bv) -> Y   (wave w's 64 columns are head w)
    dec_gemm<kDR>(X, Wl, acc, w, lane);
    {
      const float* bv = P + p.off[O_BV];
      epi([&](int r, int rr, int c, float a) {
        float v = a + bv[c];
        if (train) v = ma[rr * kNH + w] ? v / keep : 0.f;
        Y[r * kDLd + c] = v;
      });
    }
    __syncthreads();
    if (STORE) dec_store<kDR>(Y, p.sa + l * p.asd, r0, B);
    // 2. s1 = h + drop1(SAin Wo^T + bo) -> Y (once every wave has read SAin)
    dec_gemm<kDR>(Y, Wl + 3 * kPlane, acc, w, lane);
    __syncthreads();
    {
      const float* bo = P + p.off[O_BO];
      epi([&](int r, int rr, int c, float a) {
        float v = a + bo[c];
        if (train) v = m1[rr * kDD + c] ? v * inv_keep : 0.f;
        Y[r * kDLd + c] = X[r * kDLd + c] + v;
      });
    }
    __syncthreads();
    if (STORE) dec_store<kDR>(Y, p.s1 + l * p.asd, r0, B);
    dec_ln<kDR, STORE>(Y, X, P + p.off[O_N1W], P + p.off[O_N1B], w, lane, r0, B, nullptr, p.st1 + l * p.ast, p.ab);  // h1
    __syncthreads();
    // 3. s2 = h1 + drop2(CA) -> Y, CA = b_o' + sum_h keep_c[h] P[h] (eval: all heads, no drop)
    {
      const float* boc = P + p.off[O_BOC];
      const uint8_t* mc = p.mc + l * p.msh;
      const uint8_t* m2 = p.m2 + l * p.msd;
      const float* xp = p.xP + (int64_t)l * kNH * kDD;
      for (int i = tid; i < kDR * kDD; i += 64 * kDW) {
        const int r = i / kDD, c = i % kDD;
        const int64_t rr = min(r0 + r, B - 1);
        float s = 0.f;
#pragma unroll
        for (int h = 0; h < kNH; ++h)
          if (!train || mc[rr * kNH + h]) s += xp[h * kDD + c];
        float ca = s + boc[c];
        if (train) ca = m2[rr * kDD + c] ? ca * inv_keep : 0.f;
        Y[r * kDLd + c] = X[r * kDLd + c] + ca;
      }
    }
    __syncthreads();
    if (STORE) dec_store<kDR>(Y, p.s2 + l * p.asd, r0, B);
    dec_ln<kDR, STORE>(Y, X, P + p.off[O_N2W], P + p.off[O_N2B], w, lane, r0, B, STORE ? p.h2 + l * p.asd : nullptr,
                  p.st2 + l * p.ast, p.ab);  // h2
    __syncthreads();
    // 4. F1 = drop_f(relu(h2 W1^T + b1)) -> Y
    dec_gemm<kDR>(X, Wl + 6 * kPlane, acc, w, lane);
    {
      const float* b1 = P + p.off[O_B1];
      epi([&](int r, int rr, int c, float a) {
        float v = fmaxf(a + b1[c], 0.f);
        if (train) v = mf[rr * kDD + c] ? v / keep : 0.f;
        Y[r * kDLd + c] = v;
      });
    }
    __syncthreads();
    if (STORE) dec_store<kDR>(Y, p.f1 + l * p.asd, r0, B);
    // 5. s3 = h2 + drop3(F1 W2^T + b2) -> Y (once every wave has read F1); h' = LN3(s3) -> X
    dec_gemm<kDR>(Y, Wl + 9 * kPlane, acc, w, lane);
    __syncthreads();
    {
      const float* b2 = P + p.off[O_B2];
      epi([&](int r, int rr, int c, float a) {
        float v = a + b2[c];
        if (train) v = m3[rr * kDD + c] ? v * inv_keep : 0.f;
        Y[r * kDLd + c] = X[r * kDLd + c] + v;
      });
    }
    __syncthreads();
    if (STORE) dec_store<kDR>(Y, p.s3 + l * p.asd, r0, B);
    dec_ln<kDR, STORE>(Y, X, P + p.off[O_N3W], P + p.off[O_N3B], w, lane, r0, B,
                  STORE && l + 1 < L ? p.hs + (l + 1) * p.asd : nullptr, p.st3 + l * p.ast, p.ab);  // h' (the last: out)
    __syncthreads();
  }
  for (int i = tid; i < kDR * kDD / 4; i += 64 * kDW) {
    const int r = i / (kDD / 4), c4 = (i % (kDD / 4)) * 4;
    if (r0 + r < B) *reinterpret_cast<float4*>(out + (r0 + r) * ldo + c4) = *reinterpret_cast<const float4*>(X + r * kDLd + c4);
  }
}

// the four D x D weights of the L layers -> bf16 planes [L][4][3][D][D]
__global__ void decoder_split_kernel(int L, const float* __restrict__ slab, int64_t o0, int64_t o1, int64_t o2,
                                     int64_t o3, int64_t lstride, __bf16* __restrict__ W) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (l, m, n, k8): 8 consecutive k
  const int64_t per_l = 4 * kPlane / 8;
  if (i >= L * per_l) return;
  const int64_t l = i / per_l, rem = i % per_l;
  const int m = (int)(rem / (kPlane / 8));
  const int64_t e = (rem % (kPlane / 8)) * 8;
  const int64_t o = m == 0 ? o0 : m == 1 ? o1 : m == 2 ? o2 : o3;
  const float* src = slab + l * lstride + o + e;
  const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  bf16x8 pl[3];
  dec_split8(v, pl);
  __bf16* dst = W + (l * 4 + m) * 3 * kPlane + e;
#pragma unroll
  for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x8*>(dst + q * kPlane) = pl[q];
}

// the dropout masks of the L layers with the unfused path's Philox keys: site s in "ac123f", step
// ((step * 64 + l) * 8 + s) mod 2^48, counter (row0 + r) * width + index (width = NH for the head
// masks a / c, D for the unit masks); keep when (x >> 8) / 2^24 < p_keep
__global__ void decoder_masks_kernel(int64_t B, int L, float keep, uint64_t seed, uint64_t step, int64_t row0,
                                     uint8_t* __restrict__ ma, uint8_t* __restrict__ mc, int64_t msh,
                                     uint8_t* __restrict__ m1, uint8_t* __restrict__ m2, uint8_t* __restrict__ m3,
                                     uint8_t* __restrict__ mf, int64_t msd) {
  const int64_t per_l = 2 * B * kNH + 4 * B * kDD;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)L * per_l) return;
  const int64_t l = i / per_l;
  int64_t j = i % per_l;
  int site, width;
  uint8_t* dst;
  if (j < 2 * B * kNH) {
    site = (int)(j / (B * kNH));  // 0 = a, 1 = c
    j %= B * kNH;
    width = kNH;
    dst = (site == 0 ? ma : mc) + l * msh;
  } else {
    j -= 2 * B * kNH;
    const int u = (int)(j / (B * kDD));  // 0..3 = 1, 2, 3, f
    j %= B * kDD;
    site = 2 + u;
    width = kDD;
    dst = (u == 0 ? m1 : u == 1 ? m2 : u == 2 ? m3 : mf) + l * msd;
  }
  const int64_t r = j / width, idx = j % width;
  const uint64_t sstep = ((step * 64 + (uint64_t)l) * 8 + (uint64_t)site) & 0xFFFFFFFFFFFFull;
  const uint4 x = gmr::Philox::gen(seed, sstep, (uint64_t)((row0 + r) * width + idx));
  dst[r * width + idx] = (float)(x.x >> 8) * (1.0f / 16777216.0f) < keep ? 1 : 0;
}

}  // namespace

extern "C" int gmr_decoder_split_f32(int32_t L, int32_t D, const float* slab, const int64_t* w_offsets,
                                     int64_t layer_stride, uint16_t* planes, void* stream) {
  GMR_ARG(slab && w_offsets && planes && L > 0, "bad args");
  GMR_ARG(D == kDD, "fused decoder: d_model 512");
  for (int m = 0; m < 4; ++m) GMR_ARG(w_offsets[m] % 4 == 0, "weight offsets must be float4-aligned");
  GMR_ARG(layer_stride % 4 == 0 && ((uintptr_t)slab & 15) == 0, "slab / layer stride alignment");
  const int64_t n = (int64_t)L * 4 * kPlane / 8;
  hipLaunchKernelGGL(decoder_split_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, L, slab,
                     w_offsets[0], w_offsets[1], w_offsets[2], w_offsets[3], layer_stride,
                     reinterpret_cast<__bf16*>(planes));
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_decoder_masks_u8(int64_t B, int32_t L, int32_t D, int32_t nhead, float p_keep, uint64_t seed,
                                    uint64_t step, int64_t row0, uint8_t* mask_a, uint8_t* mask_c, int64_t msh,
                                    uint8_t* mask_1, uint8_t* mask_2, uint8_t* mask_3, uint8_t* mask_f, int64_t msd,
                                    void* stream) {
  GMR_ARG(mask_a && mask_c && mask_1 && mask_2 && mask_3 && mask_f && B > 0 && L > 0 && row0 >= 0, "bad args");
  GMR_ARG(D == kDD && nhead == kNH, "fused decoder: d_model 512, 8 heads");
  GMR_ARG(msh >= B * kNH && msd >= B * kDD, "mask layer strides too small");
  GMR_ARG(p_keep > 0.f && p_keep <= 1.f, "p_keep in (0, 1]");
  const int64_t n = (int64_t)L * (2 * B * kNH + 4 * B * kDD);
  hipLaunchKernelGGL(decoder_masks_kernel, dim3(gmr::grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, B, L, p_keep,
                     seed, step, row0, mask_a, mask_c, msh, mask_1, mask_2, mask_3, mask_f, msd);
  GMR_LAUNCHED();
  return GMR_OK;
}

extern "C" int gmr_decoder_fwd_f32(int64_t B, int32_t L, int32_t D, int32_t nhead, const float* h0, int64_t ld0,
                                   float* out, int64_t ldo, const float* slab, const int64_t* offsets,
                                   int64_t layer_stride, const uint16_t* planes, const float* xattn_table,
                                   float p_keep, int32_t train, const uint8_t* mask_a,
                                   const uint8_t* mask_c, int64_t msh, const uint8_t* mask_1, const uint8_t* mask_2,
                                   const uint8_t* mask_3, const uint8_t* mask_f, int64_t msd, float* const* acts,
                                   int64_t act_ld, int64_t act_stride, int64_t stat_rows, void* stream) {
  GMR_ARG(h0 && out && slab && offsets && planes && B > 0 && B < (1ll << 31) && L > 0, "bad args");
  GMR_ARG(D == kDD && nhead == kNH, "fused decoder: d_model 512, 8 heads");
  GMR_ARG(ld0 >= kDD && ldo >= kDD && ld0 % 4 == 0 && ldo % 4 == 0 && (((uintptr_t)h0 | (uintptr_t)out) & 15) == 0,
          "h0 / out: 16-byte aligned rows of >= 512 floats");
  GMR_ARG(((uintptr_t)planes & 15) == 0, "planes must be 16-byte aligned");
  GMR_ARG(xattn_table, "the cross-attention head table is required");
  if (train) {
    GMR_ARG(mask_a && mask_c && mask_1 && mask_2 && mask_3 && mask_f, "train mode needs the dropout masks");
    GMR_ARG(msh >= B * kNH && msd >= B * kDD && p_keep > 0.f && p_keep <= 1.f, "bad mask strides / p_keep");
  }
  DecArgs a{};
  a.slab = slab;
  for (int i = 0; i < O_COUNT; ++i) a.off[i] = offsets[i];
  a.lstride = layer_stride;
  a.W = reinterpret_cast<const __bf16*>(planes);
  a.xP = xattn_table;
  a.ma = mask_a;
  a.mc = mask_c;
  a.m1 = mask_1;
  a.m2 = mask_2;
  a.m3 = mask_3;
  a.mf = mask_f;
  a.msh = msh;
  a.msd = msd;
  // rows per workgroup: 32 (default; two 16-row MFMA tiles share every weight fragment, halving the weight
  // stream from L2 / MALL) or 16 (GMR_DEC_ROWS=16: twice the workgroups for small batches)
  static const int rows = [] {
    const char* e = getenv("GMR_DEC_ROWS");
    return e && atoi(e) == 16 ? 16 : 32;
  }();
  const dim3 grid((unsigned)((B + rows - 1) / rows));
  if (acts) {
    GMR_ARG(acts[0] && acts[1] && acts[2] && acts[3] && acts[4] && acts[5] && acts[6] && acts[7] && acts[8] && acts[9],
            "acts: ten activation buffers");
    GMR_ARG(act_ld == kDD && act_stride >= B * kDD && stat_rows >= B, "activation buffers: rows of 512, per-layer stride");
    a.hs = acts[0];
    a.sa = acts[1];
    a.s1 = acts[2];
    a.s2 = acts[3];
    a.h2 = acts[4];
    a.f1 = acts[5];
    a.s3 = acts[6];
    a.st1 = acts[7];
    a.st2 = acts[8];
    a.st3 = acts[9];
    a.asd = act_stride;
    a.ast = 3 * stat_rows;
    a.ab = stat_rows;
    auto kern = rows == 16 ? decoder_fwd_kernel<16, true> : decoder_fwd_kernel<32, true>;
    hipLaunchKernelGGL(kern, grid, dim3(64 * kDW), 0, (hipStream_t)stream, B, L, h0, ld0, out, ldo,
                       a, p_keep, train);
  } else {
    auto kern = rows == 16 ? decoder_fwd_kernel<16, false> : decoder_fwd_kernel<32, false>;
    hipLaunchKernelGGL(kern, grid, dim3(64 * kDW), 0, (hipStream_t)stream, B, L, h0, ld0, out, ldo,
                       a, p_keep, train);
  }
  GMR_LAUNCHED();
  return GMR_OK;
}
