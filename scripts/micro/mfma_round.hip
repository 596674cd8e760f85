// How do the gfx950 MFMAs round their fp32 accumulation?  (round 6: the split-bf16 GEMM's error has a
// directed component, scripts/x6_bias_probe.py)
// Each wave evaluates one case d = c + sum_k a_k b_k with every row of A equal to a and every column of B
// equal to b (so all 1,024 outputs of the 32 x 32 tile equal d), and the host compares d with the exact value
// (__float128) and with its round-to-nearest-even fp32 image.
// over S k steps of 16 (one accumulator chain per case):
//   mode 0: one v_mfma_f32_32x32x16_bf16 per step, a, b bf16 values
//   mode 1: the split-bf16 k step of gemm_x6_kernel: a, b fp32 split 3 ways, six chained bf16 MFMAs (small
//           terms first)
//   mode 2: the same 16 products on eight chained v_mfma_f32_32x32x2f32 (fp32 inputs)
//   mode 3: x6 with the odd steps' A negated into a second accumulator (result = acc - acc2)
//   mode 4: x6 with hi*hi alone in acc and the five small products in acc2 (result = acc + acc2; the kernel's
//           form since round 6)
//   mode 5: x6 with every operand negated, -(x6(-a, b, -c))
// Errors are reported in ulps of the case's scale |c| + sum |a b|, split by the sign of the exact result.
// hipcc -O3 --offload-arch=gfx950 mfma_round.hip -o mfma_round && ./mfma_round
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

__device__ __forceinline__ floatx16 x6_step(const bf16x8 (&fa)[3], const bf16x8 (&fb)[3], floatx16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc, 0, 0, 0);
}

// S k steps of 16 per case; a, b: [case][16 S]
__global__ void __launch_bounds__(64) round_kernel(int mode, int S, const float* __restrict__ a,
                                                   const float* __restrict__ b, const float* __restrict__ c,
                                                   float* __restrict__ d) {
  const int cs = blockIdx.x, l = threadIdx.x, hk = l >> 5;
  floatx16 acc, acc2;
  for (int e = 0; e < 16; ++e) acc[e] = c[cs], acc2[e] = 0.f;
  for (int s = 0; s < S; ++s) {
    const float* as = a + ((int64_t)cs * S + s) * 16;
    const float* bs = b + ((int64_t)cs * S + s) * 16;
    if (mode == 2) {
      for (int q = 0; q < 8; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(as[2 * q + hk], bs[2 * q + hk], acc, 0, 0, 0);
      continue;
    }
    const float sg = (mode == 3 && (s & 1)) || mode == 5 ? -1.f : 1.f;  // negated A
    bf16x8 fa[3], fb[3];
    for (int i = 0; i < 8; ++i) {
      __bf16 h, m, lo;
      split3(sg * as[8 * hk + i], h, m, lo);
      fa[0][i] = h, fa[1][i] = m, fa[2][i] = lo;
      split3(bs[8 * hk + i], h, m, lo);
      fb[0][i] = h, fb[1][i] = m, fb[2][i] = lo;
    }
    if (mode == 0) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc, 0, 0, 0);
    } else if (mode == 1) {
      acc = x6_step(fa, fb, acc);
    } else if (mode == 3) {
      if (s & 1) acc2 = x6_step(fa, fb, acc2); else acc = x6_step(fa, fb, acc);
    } else if (mode == 4) {  // hi * hi alone into acc, the five small products into acc2
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1], acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2], acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0], acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1], acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0], acc2, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc, 0, 0, 0);
    } else if (mode == 5) {  // everything negated: -(x6(-a, b, -c))
      if (s == 0)
        for (int e = 0; e < 16; ++e) acc[e] = -acc[e];
      acc = x6_step(fa, fb, acc);
    }
  }
  float r = acc[0];
  if (mode == 3) r = acc[0] - acc2[0];
  if (mode == 4) r = acc[0] + acc2[0];
  if (mode == 5) r = -acc[0];
  if (l == 0) d[cs] = r;
}

static float bf16_rne(float x) {  // host image of (__bf16)x for finite x
  unsigned u;
  memcpy(&u, &x, 4);
  u += 0x7fff + ((u >> 16) & 1);
  u &= 0xffff0000u;
  float r;
  memcpy(&r, &u, 4);
  return r;
}

static double ulp_of(float x) {
  const float ax = fabsf(x);
  return (double)nextafterf(ax, INFINITY) - (double)ax;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 100000;
  std::mt19937_64 rng(1);
  std::normal_distribution<float> N01(0.f, 1.f);
  struct Case {
    const char* name;
    int mode, S;
    float cscale;  // c = cscale * N(0,1)
    float amean;   // a ~ amean + N(0,1) (a positive mean: sums of one sign)
  };
  const Case cases[] = {
      {"bf16 MFMA, 1 step", 0, 1, 0.f, 0.f},
      {"bf16 MFMA, 64 steps", 0, 64, 0.f, 0.f},
      {"bf16 MFMA, 64 steps, positive-mean products", 0, 64, 0.f, 1.f},
      {"x6, 1 step", 1, 1, 0.f, 0.f},
      {"x6, 64 steps", 1, 64, 0.f, 0.f},
      {"x6, 64 steps, positive-mean products", 1, 64, 0.f, 1.f},
      {"x6 -(x6(-a,b,-c)), 64 steps", 5, 64, 0.f, 0.f},
      {"x6 alternate-sign accumulators, 64 steps", 3, 64, 0.f, 0.f},
      {"x6 alternate-sign accumulators, pos-mean", 3, 64, 0.f, 1.f},
      {"x6 hi*hi / small-terms accumulators, 64", 4, 64, 0.f, 0.f},
      {"x6 hi*hi / small-terms accs, pos-mean", 4, 64, 0.f, 1.f},
      {"fp32 MFMA, 64 steps", 2, 64, 0.f, 0.f},
      {"fp32 MFMA, 64 steps, positive-mean", 2, 64, 0.f, 1.f},
  };
  const int Smax = 64;
  float *da, *db, *dc, *dd;
  (void)hipMalloc(&da, sizeof(float) * 16 * Smax * (size_t)n);
  (void)hipMalloc(&db, sizeof(float) * 16 * Smax * (size_t)n);
  (void)hipMalloc(&dc, sizeof(float) * n);
  (void)hipMalloc(&dd, sizeof(float) * n);
  std::vector<float> a(16 * Smax * (size_t)n), b(16 * Smax * (size_t)n), c(n), d(n);
  for (const Case& cs : cases) {
    const size_t len = 16 * (size_t)cs.S * n;
    for (size_t i = 0; i < len; ++i) {
      a[i] = cs.amean + N01(rng), b[i] = 1.f + 0.5f * N01(rng);
      if (cs.amean == 0.f) b[i] = N01(rng);
      if (cs.mode == 0) a[i] = bf16_rne(a[i]), b[i] = bf16_rne(b[i]);  // one bf16 MFMA: bf16 inputs
    }
    for (int i = 0; i < n; ++i) c[i] = cs.cscale * N01(rng);
    (void)hipMemcpy(da, a.data(), sizeof(float) * len, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, b.data(), sizeof(float) * len, hipMemcpyHostToDevice);
    (void)hipMemcpy(dc, c.data(), sizeof(float) * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(round_kernel, dim3(n), dim3(64), 0, 0, cs.mode, cs.S, da, db, dc, dd);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("kernel failed\n");
      return 1;
    }
    (void)hipMemcpy(d.data(), dd, sizeof(float) * n, hipMemcpyDeviceToHost);
    // error in ulps of the case's scale |c| + sum |a b| (no blow-up on cancelling sums), by the result's sign
    double sp = 0, sn = 0, sa = 0;
    long np = 0, nn = 0;
    for (int i = 0; i < n; ++i) {
      __float128 ex = c[i], sc = fabsf(c[i]);
      for (size_t k = 0; k < 16 * (size_t)cs.S; ++k) {
        const __float128 p = (__float128)a[16 * (size_t)cs.S * i + k] * (__float128)b[16 * (size_t)cs.S * i + k];
        ex += p;
        sc += p < 0 ? -p : p;
      }
      const double u = ulp_of((float)sc), e = (double)((__float128)d[i] - ex) / u;
      sa += fabs(e);
      if (ex >= 0) sp += e, ++np; else sn += e, ++nn;
    }
    printf("%-44s mean err (ulp of scale): results > 0 %+.4f (%ld)  results < 0 %+.4f (%ld)  all %+.4f  "
           "mean |err| %.4f\n", cs.name, np ? sp / np : 0.0, np, nn ? sn / nn : 0.0, nn, (sp + sn) / n, sa / n);
  }
  return 0;
}
