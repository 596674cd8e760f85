#include <hip/hip_runtime.h>
template <int J>
__device__ __forceinline__ int grp_bcast(int x) {
  int a = __builtin_amdgcn_update_dpp(0, x, 0x150 + J, 0xf, 0xf, false);
  int b = __builtin_amdgcn_update_dpp(0, x, 0x150 + 8 + J, 0xf, 0xf, false);
  return (threadIdx.x & 8) ? b : a;
}
__global__ void k(const int* in, int* out) {
  int x = in[threadIdx.x];
  int acc = grp_bcast<0>(x) + 2 * grp_bcast<1>(x) + 3 * grp_bcast<5>(x) + 4 * grp_bcast<7>(x);
  out[threadIdx.x] = acc;
}
int main() {
  int h[64], *d, *o; hipMalloc(&d, 256); hipMalloc(&o, 256);
  for (int i = 0; i < 64; ++i) h[i] = i;
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, o);
  hipMemcpy(h, o, 256, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) { int g = i & ~7; int want = g + 2 * (g + 1) + 3 * (g + 5) + 4 * (g + 7); if (h[i] != want) { ++bad; if (bad < 5) printf("lane %d got %d want %d\n", i, h[i], want);} }
  printf("bad %d\n", bad);
  return 0;
}
