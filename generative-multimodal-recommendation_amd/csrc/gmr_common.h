// Shared helpers for the gfx950 kernels of libgmr_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gmr.h"

namespace gmr {
void set_error(const char* fn, const char* msg);
int hip_status(const char* fn, hipError_t e);

constexpr int kWave = 64;

__device__ __forceinline__ float4 f4_fma(float a, float4 x, float4 acc) {
  acc.x = fmaf(a, x.x, acc.x);
  acc.y = fmaf(a, x.y, acc.y);
  acc.z = fmaf(a, x.z, acc.z);
  acc.w = fmaf(a, x.w, acc.w);
  return acc;
}

__device__ __forceinline__ float4 f4_add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__device__ __forceinline__ float4 f4_scale(float s, float4 a) { return make_float4(s * a.x, s * a.y, s * a.z, s * a.w); }

__device__ __forceinline__ float4 shfl_xor_f4(float4 v, int m) {
  return make_float4(__shfl_xor(v.x, m), __shfl_xor(v.y, m), __shfl_xor(v.z, m), __shfl_xor(v.w, m));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m));
  return v;
}

// Counter-based RNG (Philox-4x32-10) for in-kernel noise / dropout / sampling.
struct Philox {
  __device__ static uint4 round(uint4 c, uint2 k) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    return make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
  }
  __device__ static uint4 gen(uint64_t seed, uint64_t subseq, uint64_t offset) {
    uint4 c = make_uint4((uint32_t)offset, (uint32_t)(offset >> 32), (uint32_t)subseq, (uint32_t)(subseq >> 32));
    uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      c = round(c, k);
      k.x += 0x9E3779B9u;
      k.y += 0xBB67AE85u;
    }
    return c;
  }
};

__device__ __forceinline__ float u32_to_unit(uint32_t x) {  // (0, 1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float2 box_muller(uint32_t a, uint32_t b) {
  float u1 = u32_to_unit(a);
  float u2 = u32_to_unit(b);
  float r = sqrtf(-2.0f * logf(u1));
  float s, c;
  sincosf(6.283185307179586f * u2, &s, &c);
  return make_float2(r * c, r * s);
}

inline int grid_for(int64_t n, int per_block, int cap = 1 << 30) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace gmr

#define GMR_ARG(cond, msg)                       \
  do {                                           \
    if (!(cond)) {                               \
      gmr::set_error(__func__, msg);             \
      return GMR_ERR_ARG;                        \
    }                                            \
  } while (0)

#define GMR_LAUNCHED()                                              \
  do {                                                              \
    hipError_t e__ = hipGetLastError();                             \
    if (e__ != hipSuccess) return gmr::hip_status(__func__, e__);   \
  } while (0)
