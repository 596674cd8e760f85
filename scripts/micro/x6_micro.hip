// Where does the split-bf16 GEMM loop spend its time?  Stand-alone microbenchmark of the k-tile loop
// of gemm_x6_kernel<256,128> (8 waves, wave tile 64x64, 48 bf16 MFMAs per wave per 32-deep tile):
//   mode 0: MFMAs only (fragments in registers)
//   mode 1: + the 24 ds_read_b128 fragment reads per tile
//   mode 2: + split + ds_write of a register tile (the next k tile) per iteration
//   mode 3: + one barrier per iteration
//   mode 4: + the real global loads (A 8192 x 8192 and B 8192 x 8192 fp32, 256 x 128 tiles, XCD-aware
//           tile order), issued at the top of an iteration and split at its end
//   mode 5: as 4 with the loads two iterations ahead (two register sets)
// hipcc -O3 --offload-arch=gfx950 x6_micro.hip -o x6_micro && ./x6_micro
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

template <int MODE>
__global__ void __launch_bounds__(512) loop_kernel(int iters, float* out, const float4* src, const float* A,
                                                   const float* B) {
  constexpr int BK = 32, APL = 256 * BK, BPL = 128 * BK, STAGE = 3 * (APL + BPL);
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w / 2, wn = w % 2, h = lane >> 5, l32 = lane & 31;
  for (int i = threadIdx.x; i < 2 * STAGE; i += 512) smem[i] = (__bf16)(float)(i & 7);
  __syncthreads();
  floatx16 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  bf16x8 fa[3][2], fb[3][2];
  for (int p = 0; p < 3; ++p)
    for (int i = 0; i < 2; ++i) {
      fa[p][i] = *reinterpret_cast<const bf16x8*>(smem + p * APL + (wm * 64 + i * 32 + l32) * BK + h * 8);
      fb[p][i] = *reinterpret_cast<const bf16x8*>(smem + 3 * APL + p * BPL + (wn * 64 + i * 32 + l32) * BK + h * 8);
    }
  float4 r[6], r2[6];
  for (int i = 0; i < 6; ++i) r[i] = r2[i] = src[threadIdx.x + 512 * i];
  // tile of this block (XCD-aware order of gemm_x6_kernel): 32 x 64 tiles of 256 x 128 over 8192^2
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b & 7, q = nwg >> 3;
  const int tile = (xcd * q + (b >> 3)) % 2048;
  const int tmi = tile / 64, tni = tile % 64;
  int offs[6];
  for (int i = 0; i < 6; ++i) {
    const int idx = threadIdx.x + 512 * i;
    if (i < 4) offs[i] = (tmi * 256 + idx / 8) * 8192 + (idx % 8) * 4;
    else offs[i] = (tni * 128 + (idx - 2048) / 8) * 8192 + ((idx - 2048) % 8) * 4;
  }
  auto gload = [&](float4 (&d)[6], int it) {
    const int k0 = (it * 32) & 8191;
    for (int i = 0; i < 6; ++i) d[i] = *reinterpret_cast<const float4*>((i < 4 ? A : B) + offs[i] + k0);
  };
  if (MODE >= 4) gload(r, 0);
  if (MODE >= 5) gload(r2, 1);
  int cur = 0;
  for (int it = 0; it < iters; ++it) {
    if (MODE == 4) gload(r, it + 1);
    if (MODE == 5) {
      if (it & 1) gload(r2, it + 2); else gload(r, it + 2);
    }
    const __bf16* a_s = smem + cur * STAGE;
    const __bf16* b_s = a_s + 3 * APL;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (MODE >= 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = wm * 64 + i * 32 + l32;
          const int off = row * BK + (((2 * s + h) ^ ((row >> 2) & 3)) << 3);
#pragma unroll
          for (int p = 0; p < 3; ++p) fa[p][i] = *reinterpret_cast<const bf16x8*>(a_s + p * APL + off);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = wn * 64 + j * 32 + l32;
          const int off = row * BK + (((2 * s + h) ^ ((row >> 2) & 3)) << 3);
#pragma unroll
          for (int p = 0; p < 3; ++p) fb[p][j] = *reinterpret_cast<const bf16x8*>(b_s + p * BPL + off);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2][i], fb[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
        }
    }
    if (MODE >= 2) {
      __bf16* nx = smem + (cur ^ 1) * STAGE;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int idx = threadIdx.x + 512 * i;
        const int rr = idx / 8, k4 = (idx % 8) * 4;
        const float4 rv = (MODE == 5 && (it & 1)) ? r[i] : (MODE == 5 ? r2[i] : r[i]);
        const float v[4] = {rv.x, rv.y, rv.z, rv.w};
        bf16x4 hh, mm, ll;
        for (int e = 0; e < 4; ++e) {
          __bf16 a, b, c;
          split3(v[e], a, b, c);
          hh[e] = a;
          mm[e] = b;
          ll[e] = c;
        }
        const int off = rr * BK + (((k4 >> 3) ^ ((rr >> 2) & 3)) << 3) + (k4 & 7);
        *reinterpret_cast<bf16x4*>(nx + off) = hh;
        *reinterpret_cast<bf16x4*>(nx + APL + off) = mm;
        *reinterpret_cast<bf16x4*>(nx + 2 * APL + off) = ll;
        if (MODE < 4) r[i].x += 1.f;
      }
      cur ^= 1;
    }
    if (MODE >= 3) __syncthreads();
  }
  float s = 0.f;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int e = 0; e < 16; ++e) s += acc[i][j][e];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int MODE>
void run(float* out, const float4* src, const float* A, const float* B) {
  const int iters = 2000, blocks = 256 * 4;
  hipLaunchKernelGGL(loop_kernel<MODE>, dim3(blocks), dim3(512), 0, 0, 10, out, src, A, B);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, 0);
  hipLaunchKernelGGL(loop_kernel<MODE>, dim3(blocks), dim3(512), 0, 0, iters, out, src, A, B);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double mfma = (double)blocks * 8 * iters * 48;  // wave MFMAs
  const double flop = mfma * 32 * 32 * 16 * 2;
  printf("mode %d: %.3f ms  %.1f bf16 TF/s  (fp32-equivalent %.1f TF/s)  cycles/k-tile/SIMD at 2.4 GHz %.0f\n", MODE, ms,
         flop / ms / 1e9, flop / 6 / ms / 1e9, ms * 1e-3 * 2.4e9 / ((double)blocks / 256 * iters));
}

int main() {
  float* out;
  float4* src;
  hipMalloc(&out, 1024 * 512 * 4 * 4);
  hipMalloc(&src, 512 * 6 * 16);
  hipMemset(src, 0, 512 * 6 * 16);
  float *A, *B;
  hipMalloc(&A, 8192ll * 8192 * 4);
  hipMalloc(&B, 8192ll * 8192 * 4);
  hipMemset(A, 0, 8192ll * 8192 * 4);
  hipMemset(B, 0, 8192ll * 8192 * 4);
  run<0>(out, src, A, B);
  run<1>(out, src, A, B);
  run<2>(out, src, A, B);
  run<3>(out, src, A, B);
  run<4>(out, src, A, B);
  run<5>(out, src, A, B);
  return 0;
}
