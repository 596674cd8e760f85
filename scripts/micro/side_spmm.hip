// Side-split SpMM microbenchmark (standalone, no torch): Y = A X for a bipartite A = [[0, R], [R^T, 0]]
// (DiffMM norm_adj, models/diffmm.py:88-107) with X row-major N x d, d = 64 * NB.
//
// Idea: a user row gathers only item rows of X and an item row only user rows, so each XCD is given
// ONE side's rows and ONE 32-column slice (128-B lines): its L2 then holds just the other side's
// slice (items 7,050 x 128 B = 0.9 MB, users 19,445 x 128 B = 2.5 MB at baby) and every gather is a
// whole line.  d = 128: 4 slices x 2 sides = 8 groups, one per XCD; d = 64: 4 groups, 2 XCDs each
// (rows split); d = 256: 16 groups, two phases per XCD.
// mode 0 = side split, mode 1 = slice only (every XCD walks both sides of its slice).
// build: hipcc -O3 --offload-arch=gfx950 -o side_spmm side_spmm.hip
// run:   ./side_spmm graph.bin   (scripts/micro/dump_graph.py)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("err %s line %d\n", hipGetErrorString(e_), __LINE__);                  \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

struct SidePlan {
  const int4* desc;  // {row, beg, end, 0}
  int hub_beg[2], hub_end[2], sh_beg[2], sh_end[2];
};

__device__ __forceinline__ float4 f4_fma(float a, float4 x, float4 c) {
  c.x = fmaf(a, x.x, c.x);
  c.y = fmaf(a, x.y, c.y);
  c.z = fmaf(a, x.z, c.z);
  c.w = fmaf(a, x.w, c.w);
  return c;
}
__device__ __forceinline__ float4 f4_add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 shx(float4 v, int m) {
  return make_float4(__shfl_xor(v.x, m), __shfl_xor(v.y, m), __shfl_xor(v.z, m), __shfl_xor(v.w, m));
}

template <int EB, int NS>
__global__ void __launch_bounds__(256) side_kernel(const int* __restrict__ col, const float* __restrict__ val, SidePlan p,
                                                   const float* __restrict__ lo, const float* __restrict__ hi, int64_t ldx,
                                                   int split, float* __restrict__ Y, int64_t ldy, int wpx, int mode,
                                                   int nt) {
  constexpr int G = 2 * NS;
  constexpr int EPL = EB / 8;
  __shared__ float4 s_red[4][8];
  const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane >> 3, sub = lane & 7, gbase = grp * 8;
  // mode 0: (side, slice) groups; mode 1: slice groups over both sides
  const bool sidesplit = !(mode & 1), do_hub = !(mode & 4), do_short = !(mode & 8);
  const int ngroups = sidesplit ? G : NS;
  const int phases = ngroups > 8 ? ngroups / 8 : 1;
  const int P = ngroups >= 8 ? 1 : 8 / ngroups;
  for (int ph = 0; ph < phases; ++ph) {
    const int g = ngroups >= 8 ? xcd + 8 * ph : xcd % ngroups;
    const int part = ngroups >= 8 ? 0 : xcd / ngroups;
    const int slice = sidesplit ? g % NS : g;
    const int s0 = sidesplit ? g / NS : 0, s1 = sidesplit ? s0 + 1 : 2;
    const int c0 = slice * 32 + sub * 4;
    const float* L = lo + c0;
    const float* H = hi + c0;
    float* Yc = Y + c0;
    const int W = P * wpx, w = part * wpx + k;
    auto walk = [&](int e0, int end, int step) -> float4 {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      int cc[EPL];
      float vv[EPL];
#pragma unroll
      for (int q = 0; q < EPL; ++q) {
        const int i = e0 + q * 8 + sub;
        cc[q] = i < end ? col[i] : 0;
        vv[q] = i < end ? val[i] : 0.f;
      }
      for (int e = e0; e < end; e += step) {
        float4 xs[EB];
        float vs[EB];
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          const int c = __shfl(cc[u / 8], gbase + u % 8);
          vs[u] = __shfl(vv[u / 8], gbase + u % 8);
          xs[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (e + u < end) xs[u] = *reinterpret_cast<const float4*>(c < split ? L + (int64_t)c * ldx : H + (int64_t)(c - split) * ldx);
        }
        const int en = e + step;
#pragma unroll
        for (int q = 0; q < EPL; ++q) {
          const int i = en + q * 8 + sub;
          cc[q] = i < end ? col[i] : 0;
          vv[q] = i < end ? val[i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < EB; ++u) acc = f4_fma(vs[u], xs[u], acc);
      }
      return acc;
    };
    auto store = [&](int row, float4 o) {
      float* yp = Yc + (int64_t)row * ldy;
      if (nt) {
        typedef float v4 __attribute__((ext_vector_type(4)));
        v4 ov = {o.x, o.y, o.z, o.w};
        __builtin_nontemporal_store(ov, reinterpret_cast<v4*>(yp));
      } else {
        *reinterpret_cast<float4*>(yp) = o;
      }
    };
    for (int s = s0; s < s1; ++s) {
      // hubs: one workgroup per row, 32 lane groups striding EB-entry batches
      for (int h = p.hub_beg[s] + w; do_hub && h < p.hub_end[s]; h += W) {
        const int4 d = p.desc[h];
        float4 acc = walk(d.y + (wid * 8 + grp) * EB, d.z, 32 * EB);
        acc = f4_add(acc, shx(acc, 8));
        acc = f4_add(acc, shx(acc, 16));
        acc = f4_add(acc, shx(acc, 32));
        if (grp == 0) s_red[wid][sub] = acc;
        __syncthreads();
        if (threadIdx.x < 8) {
          float4 t = s_red[0][sub];
          t = f4_add(t, s_red[1][sub]);
          t = f4_add(t, s_red[2][sub]);
          t = f4_add(t, s_red[3][sub]);
          store(d.x, t);
        }
        __syncthreads();
      }
      // short rows: one lane group each, rows in descending degree
      const int n = do_short ? p.sh_end[s] - p.sh_beg[s] : 0;
      const int stride = W * 32;
      int b = (w * 4 + wid) * 8 + grp;
      int4 d = b < n ? p.desc[p.sh_beg[s] + b] : make_int4(-1, 0, 0, 0);
      for (; b - grp < n; b += stride) {
        const int bn = b + stride;
        const int4 dn = bn < n ? p.desc[p.sh_beg[s] + bn] : make_int4(-1, 0, 0, 0);
        const float4 acc = walk(d.y, d.z, EB);
        if (d.x >= 0) store(d.x, acc);
        d = dn;
      }
    }
  }
}

struct Graph {
  int n, split;
  int64_t nnz;
  std::vector<int> rp, col;
  std::vector<float> val;
};

static Graph load(const char* fn) {
  Graph g;
  FILE* f = fopen(fn, "rb");
  if (!f) {
    printf("cannot open %s\n", fn);
    exit(1);
  }
  int64_t h[3];
  if (fread(h, 8, 3, f) != 3) exit(1);
  g.n = (int)h[0];
  g.split = (int)h[1];
  g.nnz = h[2];
  g.rp.resize(g.n + 1);
  g.col.resize(g.nnz);
  g.val.resize(g.nnz);
  if (fread(g.rp.data(), 4, g.n + 1, f) != (size_t)g.n + 1) exit(1);
  if (fread(g.col.data(), 4, g.nnz, f) != (size_t)g.nnz) exit(1);
  if (fread(g.val.data(), 4, g.nnz, f) != (size_t)g.nnz) exit(1);
  fclose(f);
  return g;
}

// per side: hub rows (deg > L) longest first, then short rows by descending degree
static std::vector<int4> build_plan(const Graph& g, int L, SidePlan& p) {
  std::vector<int4> desc;
  for (int s = 0; s < 2; ++s) {
    const int r0 = s == 0 ? 0 : g.split, r1 = s == 0 ? g.split : g.n;
    std::vector<int> hub, sh;
    for (int r = r0; r < r1; ++r) (g.rp[r + 1] - g.rp[r] > L ? hub : sh).push_back(r);
    auto bydeg = [&](int a, int b) {
      int da = g.rp[a + 1] - g.rp[a], db = g.rp[b + 1] - g.rp[b];
      return da != db ? da > db : a < b;
    };
    std::sort(hub.begin(), hub.end(), bydeg);
    std::sort(sh.begin(), sh.end(), bydeg);
    p.hub_beg[s] = desc.size();
    for (int r : hub) desc.push_back(make_int4(r, g.rp[r], g.rp[r + 1], 0));
    p.hub_end[s] = desc.size();
    p.sh_beg[s] = desc.size();
    for (int r : sh) desc.push_back(make_int4(r, g.rp[r], g.rp[r + 1], 0));
    p.sh_end[s] = desc.size();
  }
  return desc;
}

template <int EB, int NS>
static void launch(const int* col, const float* val, SidePlan p, const float* X, int64_t ldx, int split, float* Y,
                   int64_t ldy, int wpx, int mode, int nt) {
  hipLaunchKernelGGL((side_kernel<EB, NS>), dim3(8 * wpx), dim3(256), 0, 0, col, val, p, X, X + (int64_t)split * ldx, ldx,
                     split, Y, ldy, wpx, mode, nt);
}

int main(int argc, char** argv) {
  Graph g = load(argc > 1 ? argv[1] : "graph.bin");
  const int n = g.n;
  printf("graph n=%d split=%d nnz=%lld\n", n, g.split, (long long)g.nnz);
  int *d_col, *d_col_hot;
  float *d_val, *d_X, *d_Y;
  CK(hipMalloc(&d_col, g.nnz * 4));
  CK(hipMalloc(&d_col_hot, g.nnz * 4));
  CK(hipMalloc(&d_val, g.nnz * 4));
  CK(hipMalloc(&d_X, (int64_t)n * 256 * 4));
  CK(hipMalloc(&d_Y, (int64_t)n * 256 * 4));
  CK(hipMemcpy(d_col, g.col.data(), g.nnz * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_val, g.val.data(), g.nnz * 4, hipMemcpyHostToDevice));
  // "hot": every gather hits one of 64 rows per side (L1/L2-hot: the issue-bound floor)
  std::vector<int> hot(g.nnz);
  for (int64_t e = 0; e < g.nnz; ++e) hot[e] = g.col[e] < g.split ? g.col[e] % 64 : g.split + (g.col[e] - g.split) % 64;
  CK(hipMemcpy(d_col_hot, hot.data(), g.nnz * 4, hipMemcpyHostToDevice));
  std::vector<float> hX((int64_t)n * 256);
  std::mt19937 rng(3);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  for (auto& x : hX) x = U(rng);
  CK(hipMemcpy(d_X, hX.data(), hX.size() * 4, hipMemcpyHostToDevice));
  SidePlan p;
  std::vector<int4> desc = build_plan(g, 32, p);
  int4* d_desc;
  CK(hipMalloc(&d_desc, desc.size() * 16));
  CK(hipMemcpy(d_desc, desc.data(), desc.size() * 16, hipMemcpyHostToDevice));
  p.desc = d_desc;
  printf("hubs: users %d items %d\n", p.hub_end[0] - p.hub_beg[0], p.hub_end[1] - p.hub_beg[1]);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> hY((int64_t)n * 256);
  printf("%4s %4s %3s %4s %3s %4s %9s %9s %8s %9s\n", "d", "mode", "EB", "wpx", "nt", "hot", "us", "GB/s", "frac", "maxrel");
  for (int NB : {1, 2, 4}) {
    const int d = 64 * NB;
    const int64_t ld = d;
    // CPU reference (double)
    std::vector<double> ref((int64_t)n * d, 0.0);
    for (int r = 0; r < n; ++r)
      for (int e = g.rp[r]; e < g.rp[r + 1]; ++e) {
        const float* x = hX.data() + (int64_t)g.col[e] * ld;
        double* y = ref.data() + (int64_t)r * d;
        for (int c = 0; c < d; ++c) y[c] += (double)g.val[e] * x[c];
      }
    // X is read with ld = d from the same random buffer
    const double bytes = 8.0 * g.nnz + 4.0 * (n + 1) + 8.0 * d * n;
    for (int hotv : {0})
      for (int mode : {0, 1, 4, 8})
        for (int EB : {8, 16})
          for (int wpx : {256})
            for (int nt : {1}) {
              const int* cptr = hotv ? d_col_hot : d_col;
              auto run = [&]() {
                if (NB == 1) {
                  if (EB == 8) launch<8, 2>(cptr, d_val, p, d_X, ld, g.split, d_Y, ld, wpx, mode, nt);
                  else launch<16, 2>(cptr, d_val, p, d_X, ld, g.split, d_Y, ld, wpx, mode, nt);
                } else if (NB == 2) {
                  if (EB == 8) launch<8, 4>(cptr, d_val, p, d_X, ld, g.split, d_Y, ld, wpx, mode, nt);
                  else launch<16, 4>(cptr, d_val, p, d_X, ld, g.split, d_Y, ld, wpx, mode, nt);
                } else {
                  if (EB == 8) launch<8, 8>(cptr, d_val, p, d_X, ld, g.split, d_Y, ld, wpx, mode, nt);
                  else launch<16, 8>(cptr, d_val, p, d_X, ld, g.split, d_Y, ld, wpx, mode, nt);
                }
              };
              CK(hipMemset(d_Y, 0, (int64_t)n * d * 4));
              for (int i = 0; i < 5; ++i) run();
              CK(hipDeviceSynchronize());
              double maxrel = 0;
              if (!hotv) {
                CK(hipMemcpy(hY.data(), d_Y, (int64_t)n * d * 4, hipMemcpyDeviceToHost));
                for (int64_t i = 0; i < (int64_t)n * d; ++i)
                  maxrel = std::max(maxrel, std::fabs(hY[i] - ref[i]) / (std::fabs(ref[i]) + 1e-3));
              }
              const int reps = 50;
              CK(hipEventRecord(a));
              for (int i = 0; i < reps; ++i) run();
              CK(hipEventRecord(b));
              CK(hipEventSynchronize(b));
              float ms;
              CK(hipEventElapsedTime(&ms, a, b));
              const double us = 1e3 * ms / reps;
              printf("%4d %4d %3d %4d %3d %4d %9.2f %9.0f %8.3f %9.2e\n", d, mode, EB, wpx, nt, hotv, us, bytes / us / 1e3,
                     bytes / us / 1e3 / 8000.0, maxrel);
            }
  }
  return 0;
}
