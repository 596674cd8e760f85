// Random row-gather microbenchmark (standalone, no torch): what rate can gfx950 sustain for
// 128-byte row gathers from tables of different sizes / row strides?  Used to bound the SpMM.
// build: hipcc -O3 --offload-arch=gfx950 -o gather_bench gather_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// each 8-lane group gathers G rows (indices from idx), 16 in flight, sums, writes one float4
template <int INFL>
__global__ void __launch_bounds__(256) gather(const float* __restrict__ tab, int64_t stride_f, const int* __restrict__ idx,
                                              int per_group, float* __restrict__ out) {
  const int gid = (blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int sub = threadIdx.x & 7;
  const int* ip = idx + (int64_t)gid * per_group;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int j = 0; j < per_group; j += INFL) {
    float4 xs[INFL];
#pragma unroll
    for (int u = 0; u < INFL; ++u) {
      int r = ip[j + u];  // same address for the 8 lanes
      xs[u] = *reinterpret_cast<const float4*>(tab + (int64_t)r * stride_f + sub * 4);
    }
#pragma unroll
    for (int u = 0; u < INFL; ++u) { acc.x += xs[u].x; acc.y += xs[u].y; acc.z += xs[u].z; acc.w += xs[u].w; }
  }
  reinterpret_cast<float4*>(out)[(int64_t)gid * 8 + sub] = acc;
}

int main() {
  const int groups = 1 << 17;  // 131072 groups of 8 lanes = 16384 waves
  const int per_group = 32;
  const int64_t n_idx = (int64_t)groups * per_group;
  std::vector<int> h(n_idx);
  int* d_idx; float* d_out; float* d_tab;
  CK(hipMalloc(&d_idx, n_idx * 4));
  CK(hipMalloc(&d_out, (int64_t)groups * 32 * 4));
  const int64_t max_bytes = 256ll << 20;
  CK(hipMalloc(&d_tab, max_bytes));
  CK(hipMemset(d_tab, 0, max_bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::mt19937 rng(1);
  printf("%10s %8s %10s %10s %10s\n", "table_MB", "stride_B", "us", "GB/s", "Mrow/s");
  for (int64_t mb : {1, 4, 16, 64, 256}) {
    for (int stride_b : {128, 512}) {
      int64_t rows = (mb << 20) / stride_b;
      if (rows * stride_b > max_bytes) continue;
      std::uniform_int_distribution<int> dist(0, (int)rows - 1);
      for (auto& v : h) v = dist(rng);
      CK(hipMemcpy(d_idx, h.data(), n_idx * 4, hipMemcpyHostToDevice));
      for (int it = 0; it < 3; ++it)
        hipLaunchKernelGGL(gather<16>, dim3(groups * 8 / 256), dim3(256), 0, 0, d_tab, stride_b / 4, d_idx, per_group, d_out);
      CK(hipEventRecord(a));
      const int reps = 10;
      for (int it = 0; it < reps; ++it)
        hipLaunchKernelGGL(gather<16>, dim3(groups * 8 / 256), dim3(256), 0, 0, d_tab, stride_b / 4, d_idx, per_group, d_out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      double us = 1e3 * ms / reps;
      double bytes = (double)n_idx * 128;
      printf("%10lld %8d %10.1f %10.0f %10.0f\n", (long long)mb, stride_b, us, bytes / us / 1e3, n_idx / us);
    }
  }
  return 0;
}
