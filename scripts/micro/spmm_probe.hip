// SpMM probe (standalone, no torch): what bounds the side-split graph-conv SpMM at baby shape?
// Times, on the real norm_adj column pattern (scripts/micro/dump_graph.py), kernels that do a
// growing part of the SpMM's work with the side-split XCD mapping of csrc/spmm_side.hip
// (XCD x -> side x / NS... d = 128: side = x / 4, 32-column slice = x % 4):
//   V0 empty kernel over the same grid (dispatch + drain floor);
//   V1 entries only: lane groups stream fixed 16-entry chunks of their side's CSR entries, sum the
//      values, store one float4 per chunk (the entry stream + stores, no gathers);
//   V2 gathers: V1 plus the 16 whole-line gathers of X per chunk (no row logic: the gather floor);
//   V3 V2 with CH chunks per lane group per pass (CH x 16 gathers in flight);
//   V4 V2 with the chunk's entries loaded as one 16-B load per lane (int4 = 2 entries).
// build: hipcc -O3 --offload-arch=gfx950 -o spmm_probe spmm_probe.hip
// run:   ./spmm_probe graph.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

__device__ __forceinline__ float4 f4_fma(float a, float4 x, float4 c) {
  c.x = fmaf(a, x.x, c.x);
  c.y = fmaf(a, x.y, c.y);
  c.z = fmaf(a, x.z, c.z);
  c.w = fmaf(a, x.w, c.w);
  return c;
}

struct Args {
  const int2* ent;  // {col, val} in CSR order
  int side_beg[2], side_end[2];  // entry ranges of the user / item side
  const float* X;
  int64_t ldx;
  float* out;
  int wpx;
};

__global__ void v0_empty(Args a) {}

// MODE 1 = entries only, 2 = + gathers; CH chunks per pass; W16: one 16-B entry load per lane
// SM (store mode, MODE 2): 0 one float4 per chunk; 1 a store at every simulated row end (every 6th entry,
// offset per lane group: divergent across the wave's groups, like the side kernel's short rows);
// 2 the same row ends uniform across the wave; 3 as 1 with non-temporal stores; 4 as 1 staged in LDS,
// flushed once per chunk (one store per staged row, all groups together)
template <int MODE, int CH, bool W16, int SM = 0>
__global__ void __launch_bounds__(256) v_chunks(Args a) {
  __shared__ float4 stage[4][8][4][8];  // [wave][group][slot][lane]
  const int xcd = blockIdx.x & 7, k = blockIdx.x >> 3;
  const int lane = threadIdx.x & 63, grp = lane >> 3, sub = lane & 7;
  const int side = xcd >> 2, slice = xcd & 3;
  const int n_lg = a.wpx * 32;
  const int lg = k * 32 + (threadIdx.x >> 3);
  const int beg = a.side_beg[side], end = a.side_end[side];
  const int nch = (end - beg + 15) / 16;
  const float* Xs = a.X + slice * 32 + sub * 4;
#pragma unroll 1
  for (int c0 = lg * CH; c0 < nch; c0 += n_lg * CH) {
    int2 e[CH][2];
#pragma unroll
    for (int h = 0; h < CH; ++h) {
      const int base = beg + (c0 + h) * 16;
      if (W16) {
        const int i = base + 2 * sub;
        int4 q = make_int4(0, 0, 0, 0);
        if (c0 + h < nch && i + 1 < end) q = *reinterpret_cast<const int4*>(a.ent + i);
        else if (c0 + h < nch && i < end) q = make_int4(a.ent[i].x, a.ent[i].y, 0, 0);
        e[h][0] = make_int2(q.x, q.y);
        e[h][1] = make_int2(q.z, q.w);
      } else {
        const int i0 = base + sub, i1 = base + 8 + sub;
        e[h][0] = (c0 + h < nch && i0 < end) ? a.ent[i0] : make_int2(0, 0);
        e[h][1] = (c0 + h < nch && i1 < end) ? a.ent[i1] : make_int2(0, 0);
      }
    }
    float4 acc[CH];
#pragma unroll
    for (int h = 0; h < CH; ++h) acc[h] = make_float4(0, 0, 0, 0);
    if (MODE == 1) {
#pragma unroll
      for (int h = 0; h < CH; ++h) {
        acc[h].x = __int_as_float(e[h][0].y) + __int_as_float(e[h][1].y);
        acc[h].y = (float)(e[h][0].x + e[h][1].x);
      }
    } else {
      float4 xs[CH][16];
#pragma unroll
      for (int h = 0; h < CH; ++h)
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int src = W16 ? (u >> 1) : (u & 7);
          const int which = W16 ? (u & 1) : (u >> 3);
          const int c = __shfl(e[h][which].x, grp * 8 + src);
          const int i = (c0 + h) * 16 + u;
          xs[h][u] = make_float4(0, 0, 0, 0);
          if (i < end - beg) xs[h][u] = *reinterpret_cast<const float4*>(Xs + (int64_t)c * a.ldx);
        }
#pragma unroll
      for (int h = 0; h < CH; ++h) {
        int nst = 0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int src = W16 ? (u >> 1) : (u & 7);
          const int which = W16 ? (u & 1) : (u >> 3);
          const float v = __int_as_float(__shfl(e[h][which].y, grp * 8 + src));
          acc[h] = f4_fma(v, xs[h][u], acc[h]);
          if (SM != 0 && c0 + h < nch) {
            const bool end = SM == 2 ? (u % 6 == 5) : ((u + 3 * grp) % 6 == 5);
            if (end) {
              float* o = a.out + (((int64_t)(side * 4 + slice) * nch + c0 + h) * 16 + u) * 32 + sub * 4;
              if (SM == 4) {
                stage[threadIdx.x >> 6][grp][nst & 3][sub] = acc[h];
                ++nst;
              } else if (SM == 3) {
                typedef float f32x4v __attribute__((ext_vector_type(4)));
                f32x4v ov = {acc[h].x, acc[h].y, acc[h].z, acc[h].w};
                __builtin_nontemporal_store(ov, reinterpret_cast<f32x4v*>(o));
              } else {
                *reinterpret_cast<float4*>(o) = acc[h];
              }
              acc[h] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
          }
        }
        if (SM == 4 && c0 + h < nch) {  // flush: slot j of every group in one store instruction
          for (int j = 0; j < 3; ++j)
            if (j < nst) {
              float* o = a.out + (((int64_t)(side * 4 + slice) * nch + c0 + h) * 16 + j) * 32 + sub * 4;
              *reinterpret_cast<float4*>(o) = stage[threadIdx.x >> 6][grp][j][sub];
            }
        }
      }
    }
#pragma unroll
    for (int h = 0; h < CH; ++h)
      if (c0 + h < nch)
        *reinterpret_cast<float4*>(a.out + ((int64_t)(side * 4 + slice) * nch + c0 + h) * 32 + sub * 4) = acc[h];
  }
}

int main(int argc, char** argv) {
  Graph g = load(argc > 1 ? argv[1] : "graph.bin");
  const int n = g.n;
  printf("graph n=%d split=%d nnz=%lld\n", n, g.split, (long long)g.nnz);
  // the item side's entries start at a 16-entry boundary (aligned 16-B entry loads)
  const int64_t n0 = g.rp[g.split], off1 = (n0 + 15) / 16 * 16;
  std::vector<int2> ent(off1 + (g.nnz - n0), make_int2(0, 0));
  for (int64_t i = 0; i < g.nnz; ++i)
    ent[i < n0 ? i : off1 + (i - n0)] = make_int2(g.col[i], __builtin_bit_cast(int, g.val[i]));
  int2* d_ent;
  float *d_X, *d_out;
  const int64_t ldx = 128;
  CK(hipMalloc(&d_ent, ent.size() * 8 + 64));
  CK(hipMalloc(&d_X, (int64_t)n * ldx * 4));
  CK(hipMalloc(&d_out, (int64_t)(g.nnz / 16 + 64) * 8 * 32 * 4 * 16));
  CK(hipMemcpy(d_ent, ent.data(), ent.size() * 8, hipMemcpyHostToDevice));
  std::vector<float> hX((int64_t)n * ldx);
  std::mt19937 rng(3);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  for (auto& x : hX) x = U(rng);
  CK(hipMemcpy(d_X, hX.data(), hX.size() * 4, hipMemcpyHostToDevice));
  Args a;
  a.ent = d_ent;
  a.side_beg[0] = 0;
  a.side_end[0] = g.rp[g.split];
  a.side_beg[1] = (int)off1;
  a.side_end[1] = (int)(off1 + g.nnz - n0);
  a.X = d_X;
  a.ldx = ldx;
  a.out = d_out;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double gbytes = (double)g.nnz * 4 * 128;  // the gathered lines: 4 slices x 128 B per entry
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 5; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 100;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    printf("%-34s %8.2f us   gathered %6.2f TB/s\n", name, us, gbytes / us / 1e6);
  };
  for (int wpx : {32, 64, 128, 256}) {
    a.wpx = wpx;
    const dim3 grid(8 * wpx), blk(256);
    char nm[64];
    snprintf(nm, 64, "V0 empty            wpx %3d", wpx);
    time(nm, [&] { hipLaunchKernelGGL(v0_empty, grid, blk, 0, 0, a); });
    snprintf(nm, 64, "V1 entries          wpx %3d", wpx);
    time(nm, [&] { hipLaunchKernelGGL((v_chunks<1, 1, false>), grid, blk, 0, 0, a); });
    snprintf(nm, 64, "V2 gathers CH1      wpx %3d", wpx);
    time(nm, [&] { hipLaunchKernelGGL((v_chunks<2, 1, false>), grid, blk, 0, 0, a); });
    snprintf(nm, 64, "V3 gathers CH2      wpx %3d", wpx);
    time(nm, [&] { hipLaunchKernelGGL((v_chunks<2, 2, false>), grid, blk, 0, 0, a); });
    snprintf(nm, 64, "V4 gathers CH1 w16  wpx %3d", wpx);
    time(nm, [&] { hipLaunchKernelGGL((v_chunks<2, 1, true>), grid, blk, 0, 0, a); });
    snprintf(nm, 64, "V5 + rowend st div  wpx %3d", wpx);
    time(nm, [&] { hipLaunchKernelGGL((v_chunks<2, 1, false, 1>), grid, blk, 0, 0, a); });
    snprintf(nm, 64, "V6 + rowend st uni  wpx %3d", wpx);
    time(nm, [&] { hipLaunchKernelGGL((v_chunks<2, 1, false, 2>), grid, blk, 0, 0, a); });
    snprintf(nm, 64, "V7 + rowend NT div  wpx %3d", wpx);
    time(nm, [&] { hipLaunchKernelGGL((v_chunks<2, 1, false, 3>), grid, blk, 0, 0, a); });
    snprintf(nm, 64, "V8 + rowend LDS+fl  wpx %3d", wpx);
    time(nm, [&] { hipLaunchKernelGGL((v_chunks<2, 1, false, 4>), grid, blk, 0, 0, a); });
  }
  return 0;
}
