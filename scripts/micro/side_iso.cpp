// Isolation probe of the production side-split SpMM (libgmr_hip.so, csrc/spmm_side.hip): times the
// whole launch and the launch with parts of its plan switched off (hub wave tasks only, short-row
// tasks only, one side only) by editing copies of the plan header, at several launch widths and task
// sizes.  Standalone (no torch): links the library and calls its C-ABI.
// build: hipcc -O2 -o side_iso side_iso.cpp -L../../generative-multimodal-recommendation_amd/gmr -lgmr_hip -Wl,-rpath,...
// run:   ./side_iso graph.bin          (graph from scripts/micro/dump_graph.py)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/gmr.h"

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                     \
    }                                                              \
  } while (0)
#define OK(x)                                                              \
  do {                                                                     \
    if ((x) != 0) {                                                        \
      printf("gmr error %s line %d\n", gmr_last_error_string(), __LINE__); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

enum { H_MAGIC, H_NROWS, H_SPLIT, H_T, H_TASK, H_NT0, H_NT1, H_EMPTY, H_NE0, H_NE1, H_HUB, H_NHUB, H_SLOT, H_NSLOT,
       H_PACKED, H_NNZ, H_WAVE, H_NW0, H_NW1, H_TW, H_DC, H_CLS };

int main(int argc, char** argv) {
  FILE* f = fopen(argc > 1 ? argv[1] : "graph.bin", "rb");
  if (!f) return 1;
  int64_t h[3];
  if (fread(h, 8, 3, f) != 3) return 1;
  const int n = (int)h[0], split = (int)h[1];
  const int64_t nnz = h[2];
  std::vector<int> rp(n + 1), col(nnz);
  std::vector<float> val(nnz);
  if (fread(rp.data(), 4, n + 1, f) != (size_t)n + 1 || fread(col.data(), 4, nnz, f) != (size_t)nnz ||
      fread(val.data(), 4, nnz, f) != (size_t)nnz)
    return 1;
  fclose(f);
  printf("graph n=%d split=%d nnz=%lld\n", n, split, (long long)nnz);
  int *d_rp, *d_col;
  float *d_val, *d_X, *d_Y;
  CK(hipMalloc(&d_rp, (n + 1) * 4));
  CK(hipMalloc(&d_col, nnz * 4));
  CK(hipMalloc(&d_val, nnz * 4));
  CK(hipMalloc(&d_X, (int64_t)n * 256 * 4));
  CK(hipMalloc(&d_Y, (int64_t)n * 256 * 4));
  CK(hipMemcpy(d_rp, rp.data(), (n + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_col, col.data(), nnz * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_val, val.data(), nnz * 4, hipMemcpyHostToDevice));
  {
    std::vector<float> hx((int64_t)n * 256);
    std::mt19937 rng(3);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    for (auto& x : hx) x = U(rng);
    CK(hipMemcpy(d_X, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int T : {16 | GMR_SIDE_CLASSES, 16, 32}) {
    const int32_t Tw = T | (32 << 16);
    const int64_t words = gmr_spmm_side_plan_words(rp.data(), n, split, Tw);
    std::vector<int32_t> plan(words);
    OK(gmr_spmm_side_plan_build(rp.data(), n, split, Tw, plan.data(), words));
    const int64_t sc = gmr_spmm_side_scratch_floats(plan.data());
    printf("T=%d%s: tasks %d/%d waves %d/%d hubs %d slots %d empty %d/%d\n", T & 0xFFFF,
           (T & GMR_SIDE_CLASSES) ? " classes" : "", plan[H_NT0], plan[H_NT1], plan[H_NW0],
           plan[H_NW1], plan[H_NHUB], plan[H_NSLOT], plan[H_NE0], plan[H_NE1]);
    int32_t* d_plan[5];
    const char* names[5] = {"full", "short tasks only", "hub waves only", "user side only", "item side only"};
    for (int v = 0; v < 5; ++v) {
      std::vector<int32_t> p = plan;
      if (v == 1) p[H_NW0] = p[H_NW1] = 0;
      if (v == 2) p[H_NT0] = p[H_NT1] = p[H_NE0] = p[H_NE1] = 0;
      if (v == 3) p[H_NT1] = p[H_NW1] = p[H_NE1] = 0;
      if (v == 4) p[H_NT0] = p[H_NW0] = p[H_NE0] = 0;
      if (p[H_DC]) {  // class jobs: the side's terminator record holds its job count
        if (v == 2 || v == 4) p[p[H_CLS] + 4 * 16] = 0;
        if (v == 2 || v == 3) p[p[H_CLS] + 4 * (17 + 16)] = 0;
      }
      CK(hipMalloc(&d_plan[v], words * 4));
      CK(hipMemcpy(d_plan[v], p.data(), words * 4, hipMemcpyHostToDevice));
      OK(gmr_spmm_side_pack(d_rp, d_col, d_val, n, nnz, p[H_PACKED], d_plan[v], nullptr));
      OK(gmr_spmm_side_pack_classes(d_rp, d_col, d_val, p.data(), d_plan[v], nullptr));
    }
    float* d_sc;
    CK(hipMalloc(&d_sc, sc * 4));
    CK(hipMemset(d_sc, 0, sc * 4));
    CK(hipDeviceSynchronize());
    for (int nb : {1, 2}) {
      const float* lo[4];
      const float* hi[4];
      float* y[4];
      int64_t ldl[4], ldh[4], ldy[4];
      for (int b = 0; b < nb; ++b) {
        lo[b] = d_X + 64 * b;
        hi[b] = d_X + (int64_t)split * 64 * nb + 64 * b;
        y[b] = d_Y + 64 * b;
        ldl[b] = ldh[b] = ldy[b] = 64 * nb;
      }
      for (int wpx : {64, 128, 256, 512}) {
        OK(gmr_spmm_side_tune(wpx, 16));
        for (int v = 0; v < 5; ++v) {
          auto launch = [&] {
            OK(gmr_spmm_side_f32(d_plan[v], nb, lo, ldl, hi, ldh, split, 1.f, 0.f, y, ldy, d_sc, wpx, nullptr));
          };
          for (int i = 0; i < 5; ++i) launch();
          CK(hipDeviceSynchronize());
          const int reps = 100;
          CK(hipEventRecord(e0));
          for (int i = 0; i < reps; ++i) launch();
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          printf("  T %2d%s d %3d wpx %3d %-18s %7.2f us\n", T & 0xFFFF, (T & GMR_SIDE_CLASSES) ? " cls" : "    ",
                 64 * nb, wpx, names[v], 1e3 * ms / reps);
        }
      }
    }
    for (int v = 0; v < 5; ++v) CK(hipFree(d_plan[v]));
    CK(hipFree(d_sc));
  }
  return 0;
}
