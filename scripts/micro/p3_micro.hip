// Prototype: fp32 GEMM on the bf16 matrix cores from PRE-SPLIT operands.  A and B arrive as three bf16
// planes each (x = hi + mid + lo exactly, written once by their producers), k-contiguous with rows padded
// to a multiple of 32 k (zero pad), so the k loop has no VALU split and no tail: every 32-deep k tile goes
// global -> LDS by global_load_lds_dwordx4 (16 rows x 64 B of one plane per wave instruction) and the
// waves run the six bf16 MFMA products per 32x32x16 block (hi.hi + hi.mid + mid.hi + hi.lo + lo.hi +
// mid.mid) on fragments read with ds_read_b128.  Measures the rebuild products of DiffMM at baby shape:
//   p_sample hidden   19445 x 1000 x 7050 (N = 1000, K = 7050)
//   p_sample output   19445 x 7050 x 1000 (N = 7050, K = 1000)
// hipcc -O3 -std=c++17 --offload-arch=gfx950 p3_micro.hip -o p3_micro && ./p3_micro
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                     \
    }                                                              \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;
constexpr int BK = 32;

__device__ __forceinline__ int swz(int r) { return (r >> 2) & 3; }

__device__ __forceinline__ void glds16(const void* src, void* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_void*)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// one operand tile: 3 planes x R rows x 32 k of bf16 -> LDS [plane][row][4 chunks], chunk c of row r at c ^ swz(r)
template <int R, int NW>
__device__ __forceinline__ void glds_planes(const __bf16* __restrict__ p, int64_t ld, int64_t pstride, int64_t r0,
                                            int64_t nrows, int64_t k0, __bf16* img, int w, int lane) {
  constexpr int NI = 3 * R / 16;  // 1 KiB wave instructions
  static_assert(NI % NW == 0, "glds instructions split evenly over the waves");
#pragma unroll
  for (int i = 0; i < NI / NW; ++i) {
    const int j = w + NW * i;
    const int plane = j / (R / 16), rb = (j % (R / 16)) * 16;
    const int r = rb + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    const int64_t row = min(r0 + r, nrows - 1);
    glds16(p + plane * pstride + row * ld + k0 + 8 * c, img + (plane * R + rb) * BK);
  }
}

template <int BM, int BN, int WGM, int WGN, int OCC, int NBUF>
__global__ void __launch_bounds__(64 * WGM * WGN, OCC) p3_kernel(int64_t M, int64_t N, int64_t Kp, const __bf16* A,
                                                             int64_t lda, int64_t psa, const __bf16* B, int64_t ldb,
                                                             int64_t psb, float* C, int64_t ldc, int tiles_n, int G) {
  constexpr int NW = WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN, TM = WTM / 32, TN = WTN / 32;
  constexpr int APL = BM * BK, BPL = BN * BK, STAGE = 3 * (APL + BPL);
  constexpr int GPW = 3 * (BM + BN) / 16 / NW;
  __shared__ __attribute__((aligned(16))) __bf16 smem[NBUF * STAGE];
  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int tiles_m = (int)((M + BM - 1) / BM);
  int tmi, tni;
  if (G <= 1) {
    tmi = tile / tiles_n;
    tni = tile % tiles_n;
  } else {
    const int per = G * tiles_n, g = tile / per, first = g * G;
    const int gs = min(tiles_m - first, G), rem = tile - g * per;
    tni = rem / gs;
    tmi = first + rem - tni * gs;
  }
  const int64_t m0 = (int64_t)tmi * BM, n0 = (int64_t)tni * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w / WGN, wn = w % WGN, h = lane >> 5, l32 = lane & 31;
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int nk = (int)(Kp / BK);
  auto issue = [&](int t) {
    __bf16* img = smem + (NBUF == 2 ? (t & 1) * STAGE : 0);
    glds_planes<BM, NW>(A, lda, psa, m0, M, (int64_t)t * BK, img, w, lane);
    glds_planes<BN, NW>(B, ldb, psb, n0, N, (int64_t)t * BK, img + 3 * APL, w, lane);
  };
  issue(0);
  vm_wait<0>();
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const bool more = t + 1 < nk;
    if (NBUF == 2 && more) issue(t + 1);
    const __bf16* a_s = smem + (NBUF == 2 ? (t & 1) * STAGE : 0);
    const __bf16* b_s = a_s + 3 * APL;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fb[3][TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WTN + j * 32 + l32;
        const int off = row * BK + (((2 * s + h) ^ swz(row)) << 3);
#pragma unroll
        for (int p = 0; p < 3; ++p) fb[p][j] = *reinterpret_cast<const bf16x8*>(b_s + p * BPL + off);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        bf16x8 fa[3];
        const int row = wm * WTM + i * 32 + l32;
        const int off = row * BK + (((2 * s + h) ^ swz(row)) << 3);
#pragma unroll
        for (int p = 0; p < 3; ++p) fa[p] = *reinterpret_cast<const bf16x8*>(a_s + p * APL + off);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0][j], acc[i][j], 0, 0, 0);
        }
      }
    }
    if (NBUF == 2) {
      if (more) vm_wait<0>();
      __syncthreads();
    } else {
      __syncthreads();  // every wave is done with the single buffer
      if (more) {
        issue(t + 1);
        vm_wait<0>();
        __syncthreads();
      }
    }
  }
  // plain fp32 store of the fragments (prototype epilogue)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t n = n0 + wn * WTN + j * 32 + l32;
      if (n >= N) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + wm * WTM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (m < M) C[m * ldc + n] = acc[i][j][e];
      }
    }
}

static uint16_t bf16_rne(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

struct Planes {
  int64_t rows, K, Kp, ps;
  std::vector<float> x;
  std::vector<uint16_t> p;  // [3][rows][Kp]
};
static Planes make(int64_t rows, int64_t K, int seed) {
  Planes q;
  q.rows = rows, q.K = K, q.Kp = (K + 31) / 32 * 32, q.ps = rows * q.Kp;
  std::mt19937 rng(seed);
  std::normal_distribution<float> nd(0.f, 1.f);
  q.x.resize(rows * K);
  for (auto& v : q.x) v = nd(rng);
  q.p.assign(3 * q.ps, 0);
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t k = 0; k < K; ++k) {
      const float v = q.x[r * K + k];
      const uint16_t h = bf16_rne(v);
      const float r1 = v - bf2f(h);
      const uint16_t m = bf16_rne(r1);
      const uint16_t l = bf16_rne(r1 - bf2f(m));
      q.p[r * q.Kp + k] = h;
      q.p[q.ps + r * q.Kp + k] = m;
      q.p[2 * q.ps + r * q.Kp + k] = l;
    }
  return q;
}

template <int BM, int BN, int WGM, int WGN, int OCC, int NBUF>
static void run(const char* name, int64_t M, int64_t N, int64_t K, int G) {
  Planes a = make(M, K, 1), b = make(N, K, 2);
  __bf16 *dA, *dB;
  float* dC;
  CK(hipMalloc(&dA, a.p.size() * 2));
  CK(hipMalloc(&dB, b.p.size() * 2));
  CK(hipMalloc(&dC, M * N * 4));
  CK(hipMemcpy(dA, a.p.data(), a.p.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, b.p.data(), b.p.size() * 2, hipMemcpyHostToDevice));
  const int tm = (int)((M + BM - 1) / BM), tn = (int)((N + BN - 1) / BN);
  const dim3 grid(tm * tn), blk(64 * WGM * WGN);
  auto launch = [&] {
    hipLaunchKernelGGL((p3_kernel<BM, BN, WGM, WGN, OCC, NBUF>), grid, blk, 0, 0, M, N, a.Kp, dA, a.Kp, a.ps, dB, b.Kp,
                       b.ps, dC, N, tn, G);
  };
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> C(M * N);
  CK(hipMemcpy(C.data(), dC, M * N * 4, hipMemcpyDeviceToHost));
  double worst = 0;
  std::mt19937 rng(5);
  for (int s = 0; s < 256; ++s) {
    const int64_t m = rng() % M, n = rng() % N;
    double ref = 0, mag = 0;
    for (int64_t k = 0; k < K; ++k) {
      ref += (double)a.x[m * K + k] * b.x[n * K + k];
      mag += fabs((double)a.x[m * K + k] * b.x[n * K + k]);
    }
    worst = fmax(worst, fabs(C[m * N + n] - ref) / mag);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(e0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1e3 * ms / reps;
  printf("%-34s %dx%d/%d G%-2d %6lld x %5lld x %5lld  %8.1f us  %6.1f TF/s  max err/sum|ab| %.2e\n", name, BM, BN, NBUF, G,
         (long long)M, (long long)N, (long long)K, us, 2.0 * M * N * K / us / 1e6, worst);
  CK(hipFree(dA));
  CK(hipFree(dB));
  CK(hipFree(dC));
}

int main() {
  for (int G : {0, 8}) {
    run<256, 128, 4, 2, 1, 2>("hidden  p3", 19445, 1000, 7050, G);
    run<128, 128, 2, 2, 1, 2>("hidden  p3", 19445, 1000, 7050, G);
    run<128, 128, 2, 2, 3, 1>("hidden  p3", 19445, 1000, 7050, G);
    run<256, 128, 4, 2, 1, 2>("output  p3", 19445, 7050, 1000, G);
    run<128, 128, 2, 2, 1, 2>("output  p3", 19445, 7050, 1000, G);
    run<128, 128, 2, 2, 3, 1>("output  p3", 19445, 7050, 1000, G);
    run<128, 256, 2, 4, 1, 2>("output  p3", 19445, 7050, 1000, G);
  }
  run<256, 128, 4, 2, 1, 2>("square  p3", 8192, 8192, 8192, 8);
  return 0;
}
