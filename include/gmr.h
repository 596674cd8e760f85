/* libgmr_hip.so — C-ABI of the MI355X-native GenMMRec hot path (gfx950).
 *
 * The reference (orangeai-research/Generative-Multimodal-Recommendation, GenMMRec/src) is pure
 * PyTorch: its hot path has no FFI.  The boundary it exposes is the Python module API
 * (GeneralRecommender.calculate_loss / full_sort_predict, the trainers' diffusion hooks);
 * every entry point below replaces the torch/ATen call sites named in its comment, and the
 * Python package `gmr` (generative-multimodal-recommendation_amd/gmr) binds them with ctypes.
 *
 * Conventions
 *   - all pointers are DEVICE pointers unless the comment says "host"; the caller owns every
 *     buffer (no allocation inside); workspaces are sized by the *_words and *_floats helpers;
 *   - matrices are row-major with an explicit leading dimension (elements);
 *   - every call is asynchronous on `stream` (a hipStream_t; NULL = legacy default stream);
 *   - return 0 on success, GMR_ERR_ARG for a rejected argument, or -(hipError_t);
 *     gmr_last_error_string() describes the last failure of the calling thread;
 *   - calls are stateless and re-entrant (safe from several threads on different streams).
 */
#ifndef GMR_H_
#define GMR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GMR_ABI_VERSION 2
#define GMR_OK 0
#define GMR_ERR_ARG (-1000)

/* GEMM epilogues (gmr_gemm_f32) */
#define GMR_EPI_NONE 0         /* C = alpha*acc + beta*C                                  */
#define GMR_EPI_BIAS 1         /* C = alpha*acc + bias + beta*C                           */
#define GMR_EPI_BIAS_TANH 2    /* C = tanh(alpha*acc + bias)            Denoise in_layers */
#define GMR_EPI_LEAKY 3        /* C = leaky_relu(alpha*acc + bias, slope)  modal projection */
#define GMR_EPI_POSTERIOR 4    /* C = c1*(alpha*acc + bias) + c2*aux[m,n], c1 = rv1 ? rv1[m] : slope,
                                  c2 = rv2 ? rv2[m] : beta            p_sample posterior mean */
#define GMR_EPI_DTANH 5        /* C = alpha*acc * (1 - aux[m,n]^2)      tanh backward      */
#define GMR_EPI_ROWSCALE_AUX 6 /* C = alpha*acc + bias + rv1[m]*aux[m,n]                  */
#define GMR_EPI_BIAS_RELU 7    /* C = relu(alpha*acc + bias)        TransformerDecoderLayer FF */
/* split-K workspaces start with this many int32 tile counters: zero them once when the buffer is
 * allocated (every gmr_gemm_f32 call leaves them zero); the partial slabs follow */
#define GMR_GEMM_COUNTER_WORDS 16384
#define GMR_GEMM_GLDS (1 << 22)      /* tile flag: stage operands by global_load_lds (the default) */
#define GMR_GEMM_REGSTAGE (1 << 23)  /* tile flag: stage operands through registers + ds_write */
#define GMR_GEMM_MFMA16 (1 << 24)
#define GMR_GEMM_MFMA32 (1 << 25)
#define GMR_GEMM_X6 (1 << 26)        /* tile flag: split-bf16 operands on the bf16 MFMA (six products, fp32-accurate) */
#define GMR_GEMM_F32 (1 << 27)       /* tile flag: force the fp32-input MFMA (overrides GMR_GEMM_X6=1 in the environment) */
#define GMR_EPI_DRELU 8        /* C = aux[m,n] > 0 ? alpha*acc : 0  ReLU (+ dropout) backward  */
#define GMR_EPI_LEAKY_NORM 9   /* C = leaky_relu(alpha*acc + bias, slope) and its row normalisation in the split-K
                                  reduce: aux (WRITTEN, ld_aux) = C[m] / max(|C[m]|, 1e-12), rowvec1 (WRITTEN) = that
                                  norm; N = 64 plans with split-K only (DiffMM modality projection + F.normalize,
                                  models/diffmm.py:115-127, 138-149) */
#define GMR_EPI_SCALE_BIAS 10  /* C = slope*(alpha*acc + bias): POSTERIOR with c2 = 0 without reading aux, bit for
                                  bit (the last p_sample step, t = 0, whose posterior mean is the x0 prediction) */

const char* gmr_last_error_string(void);
int gmr_version(void);
int gmr_device_name(char* buf /* host */, int32_t len);
int gmr_zero(void* ptr, int64_t bytes, void* stream);
/* host-layer stream plumbing: an event (timing disabled) and "record ev on from, make to wait" */
int gmr_event_create(void** ev /* host */);
int gmr_event_destroy(void* ev);
int gmr_stream_fork(void* from, void* to, void* ev);
/* test probe (no reference counterpart): a one-wave kernel that sleeps ~us microseconds on `stream`, used to
 * perturb side-stream timing in the stream-ordering tests */
int gmr_delay(int32_t us, void* stream);

/* ---------------------------------------------------------------- K1 graph convolution
 * Y = alpha * A * X + beta * Y for CSR A (int32 rowptr/col, fp32 val).
 * Replaces torch.spmm / torch.sparse.mm: models/diffmm.py:136,139,142,146,149,152,176,179,285;
 * lightgcn.py:120.  X is n_blocks (1,2,4) column blocks of 64 floats; block b reads source
 * row s from x_lo[b] + s*ld_lo[b] when s < split, else x_hi[b] + (s-split)*ld_hi[b]
 * (x_lo/x_hi/ld_* are HOST arrays of device pointers / strides).  A plan is built once per
 * matrix by gmr_spmm_plan_build; seg_nnz selects the schedule:
 *   64..448 (multiple of 64): segment plan — rows cut into <= seg_nnz segments, one wave per
 *            segment, hub rows combined in segment order by a second pass that reads
 *            `partial` (gmr_spmm_partial_rows(...) x (64*n_blocks) floats);
 *   512..8192: blocked plan — whole rows packed into ~seg_nnz-nnz blocks, one 1024-thread
 *            workgroup per block and XCD-pinned 32-column slice, rows cut by the in-block
 *            nnz split combined in LDS (no second pass, `partial` unused).
 *   GMR_SPMM_LANE_PLAN | L (L = 32, 64 or 128): lane plan — X cut into 16- or 32-column
 *            slices pinned one per XCD (L2-resident), one lane group per row of degree <= L
 *            (rows ordered by degree), one workgroup per hub row (degree > L); one launch,
 *            `partial` unused.
 *   GMR_SPMM_LANE_PLAN | GMR_SPMM_PACKED | 32: packed lane plan — as the lane plan, with the
 *            short rows' col/val copied into plan order by gmr_spmm_plan_pack (call it after
 *            gmr_spmm_plan_build, and again whenever col/val change): a row's entries are found
 *            from a degree-bucket table, so no descriptor load sits on the gather chain and the
 *            next rows' entries load while the current gathers land.  Same sums, bit for bit.
 *   GMR_SPMM_CHUNK_PLAN: chunk plan — rows of degree 1..128 cut in row order into tasks of whole
 *            rows holding <= 128 entries; a wave gathers a task's entries in one round whatever
 *            rows they belong to (no idle gather slots on short rows), row sums crossing lane
 *            groups meet in LDS in a fixed order; rows of degree > 128 take a workgroup each;
 *            X sliced per XCD as in the lane plan.  Needs gmr_spmm_plan_pack after the build.
 * All are deterministic.  flags: GMR_SPMM_NO_SPLIT_ROWS when the segment plan has no row
 * longer than seg_nnz (gmr_spmm_plan_info header word 1 == 0): the combine pass is skipped. */
#define GMR_SPMM_NO_SPLIT_ROWS 1
/* lane plans whose hub rows were split into segments (plan header word 2 >> 1 > 0): the launch
 * adds the segment partials (partial buffer of gmr_spmm_partial_rows x 256 floats) in order. */
#define GMR_SPMM_HUB_FIXUP 2
#define GMR_SPMM_LANE_PLAN (1 << 16)
#define GMR_SPMM_PACKED (1 << 17)
#define GMR_SPMM_CHUNK_PLAN (1 << 18)
int64_t gmr_spmm_plan_words(int64_t n_rows, int64_t nnz, int32_t seg_nnz);
int64_t gmr_spmm_partial_rows(int64_t n_rows, int64_t nnz, int32_t seg_nnz);
/* gmr_spmm_plan_build with row classes (non-packed lane plans): the short rows >= class_split are
 * scheduled before the rows < class_split, each class by descending degree (the item rows, then
 * the user rows of a bipartite graph: each phase gathers one side's X rows); 0 = one class.
 * Same sums as the one-class plan. */
int gmr_spmm_plan_build_split(const int32_t* rowptr, int64_t n_rows, int64_t nnz, int32_t seg_nnz,
                              int64_t class_split, int32_t* plan, void* stream);
int gmr_spmm_plan_build(const int32_t* rowptr, int64_t n_rows, int64_t nnz, int32_t seg_nnz, int32_t* plan,
                        void* stream);
/* Copies the 4-word plan header to the host (synchronises the stream): segment plan
 * {n_segments, n_split_rows, n_partials, 0}; blocked plan {n_blocks, 0, 0, seg_nnz};
 * lane plan {n_hub_descriptors, n_short_rows, packed | n_split_hub_rows << 1, L}; chunk plan
 * {n_hub_rows, n_tasks, n_empty_rows, n_packed_entries}. */
int gmr_spmm_plan_pack(const int32_t* rowptr, const int32_t* col, const float* val, int64_t n_rows, int64_t nnz,
                       int32_t seg_nnz, int32_t* plan, void* stream);
/* Lane-plan SpMM with X in column-panel layout: S contiguous panels of panel_rows x W floats
 * (W = 16 for n_blocks 1 and 2, 32 for 4; S = 64 * n_blocks / W), panel s holding columns
 * [s*W, (s+1)*W) of X, so each XCD's slice occupies whole cache lines.  Same sums as
 * gmr_spmm_csr_f32 on the row-major X. */
int gmr_spmm_panel_f32(const int32_t* col, const float* val, int64_t n_rows, int64_t nnz, const int32_t* plan,
                       int32_t seg_nnz, int32_t n_blocks, const float* x_panel, int64_t panel_rows, float alpha,
                       float beta, float* y, int64_t ldy, float* partial, int32_t flags, void* stream);
/* Lane-plan SpMM with one output per 64-column block: block b goes to y_blocks[b] (row stride
 * ld_y[b]; host arrays of device pointers / strides).  Fuses independent products of one matrix
 * (DiffMM's H and K2) into one launch; same sums as the separate gmr_spmm_csr_f32 calls. */
int gmr_spmm_multi_f32(const int32_t* col, const float* val, int64_t n_rows, int64_t nnz, const int32_t* plan,
                       int32_t seg_nnz, int32_t n_blocks, const float* const* x_lo, const int64_t* ld_lo,
                       const float* const* x_hi, const int64_t* ld_hi, int64_t split, float alpha, float beta,
                       float* const* y_blocks, const int64_t* ld_y, float* partial, int32_t flags, void* stream);
/* One launch for up to 4 independent lane-plan products, of one or several matrices (DiffMM's
 * Qi = iadj.[E0|nimg], Qt = tadj.[E0|ntxt] and G = adj.[nimg|ntxt] of forward_MM, models/diffmm.py:
 * 135-149; the backward's adj^T products of the contrastive and BPR gradients, and the UI-graph
 * transposes beside adj^T dE).  Job q is gmr_spmm_multi_f32's argument list; every job keeps its
 * own plan, sources, outputs, alpha/beta, partial buffer and flags, and its sums are exactly the
 * single-job call's.  All jobs of a launch need n_blocks in {1, 2} or all 4.  Hub-row fixups of
 * the jobs that need one (GMR_SPMM_HUB_FIXUP) follow in one second launch. */
typedef struct gmr_spmm_job {
  const int32_t* col;
  const float* val;
  const int32_t* plan;
  float* partial;
  int64_t n_rows, nnz;
  int32_t seg_nnz, n_blocks, flags, reserved;
  const float* x_lo[4];
  int64_t ld_lo[4];
  const float* x_hi[4];
  int64_t ld_hi[4];
  int64_t split;
  float alpha, beta;
  float* y[4];
  int64_t ld_y[4];
} gmr_spmm_job;
int gmr_spmm_jobs_f32(int32_t n_jobs, const gmr_spmm_job* jobs, void* stream);
int gmr_spmm_plan_info(const int32_t* plan, int32_t* host_hdr, void* stream);

/* Side-split SpMM (csrc/spmm_side.hip; the graph-conv products of models/diffmm.py:136-191, 285 and
 * common/trainer.py:464-485).  Rows [0, split) and [split, n) are the two sides of a bipartite
 * adjacency; each XCD serves one (side, 32-column slice) group, lane groups stream tasks of <= T
 * CSR entries (whole rows; hub rows cut into pieces whose partial rows the last-arriving piece adds
 * in order, in-launch).  Plan: built on the HOST from a host copy of rowptr (words from
 * gmr_spmm_side_plan_words), copied to the device, then gmr_spmm_side_pack writes the packed
 * (col, val) entries into it (packed_off = plan word 14).  scratch: gmr_spmm_side_scratch_floats
 * floats, zero before the first call (its counters re-arm themselves); two launches that may run
 * concurrently need separate scratch.  Y = alpha A X + beta Y with X / Y as gmr_spmm_multi_f32's
 * per-block split sources / outputs (16-byte aligned, strides multiples of 4).  A short row's sum
 * is its entries in CSR order; a hub row adds its pieces in piece order: deterministic. */
/* T: bits 0-15 = entries per short-row task (rows of degree > T are hub rows), bits 16-23 = entries
 * per lane group of a hub block (blocks of 8 x that; 0 = 32); | GMR_SIDE_CLASSES: degree-class plan —
 * rows of degree 1 .. 16 are grouped by degree (a wave takes 8 tasks of 16 / d whole rows of one degree
 * d, so every lane group's row ends fall on the same entry slots: full-width row stores), their
 * (col, val) copied in class order by gmr_spmm_side_pack_classes (after gmr_spmm_side_pack, with the
 * host plan); rows above 16 entries are hub rows.  Short-row sums keep CSR order from zero. */
#define GMR_SIDE_CLASSES (1 << 24)
int64_t gmr_spmm_side_plan_words(const int32_t* rowptr_host, int64_t n_rows, int64_t split, int32_t T);
int gmr_spmm_side_plan_build(const int32_t* rowptr_host, int64_t n_rows, int64_t split, int32_t T, int32_t* plan_host,
                             int64_t words);
int64_t gmr_spmm_side_scratch_floats(const int32_t* plan_host);
int gmr_spmm_side_pack(const int32_t* rowptr, const int32_t* col, const float* val, int64_t n_rows, int64_t nnz,
                       int64_t packed_off, int32_t* plan, void* stream);
int gmr_spmm_side_pack_classes(const int32_t* rowptr, const int32_t* col, const float* val, const int32_t* plan_host,
                               int32_t* plan, void* stream);
/* launch shape for tuning sweeps: workgroups per XCD and entries in flight per lane group (8 / 16);
 * defaults GMR_SPMM_SIDE_WPX / GMR_SPMM_SIDE_EB (64 / 16) */
int gmr_spmm_side_tune(int32_t wpx, int32_t eb);
/* wpx: workgroups per XCD of the launch (0 = GMR_SPMM_SIDE_WPX or 64); gmr_spmm_side_tune overrides it */
int gmr_spmm_side_f32(const int32_t* plan, int32_t n_blocks, const float* const* x_lo, const int64_t* ld_lo,
                      const float* const* x_hi, const int64_t* ld_hi, int64_t split, float alpha, float beta,
                      float* const* y_blocks, const int64_t* ld_y, float* scratch, int32_t wpx, void* stream);
/* The same product as Y = alpha A X + beta Z: z_blocks / ld_z (NULL: Z = Y) give the beta term's source, and
 * only_side 0 / 1 computes only the rows < split / >= split (the other rows of Y are left untouched; -1: all),
 * with all eight XCDs on that side.  DiffMM's backward (round 6, models/diffmm.py:141-195): Tcl and the
 * contrastive views' dC = dK + adj^T dK in one pass, and the second GCN hop's item rows T3i = T2i + adj^T T2u. */
int gmr_spmm_side2_f32(const int32_t* plan, int32_t n_blocks, const float* const* x_lo, const int64_t* ld_lo,
                       const float* const* x_hi, const int64_t* ld_hi, int64_t split, float alpha, float beta,
                       const float* const* z_blocks, const int64_t* ld_z, float* const* y_blocks, const int64_t* ld_y,
                       int32_t only_side, float* scratch, int32_t wpx, void* stream);
/* Up to 4 independent side-split products of the same width (n_blocks) in ONE launch (round 5; the forward's
 * Qi / Qt / G and the backward's UI-graph transposes, models/diffmm.py:129-195): job q has its own plan,
 * hub scratch, split and block arrays at entries [4 q, 4 q + n_blocks) of x_lo / ld_lo / x_hi / ld_hi / y /
 * ld_y.  Each job's sums are those of its own gmr_spmm_side_f32 call, bit for bit. */
int gmr_spmm_side_jobs_f32(int32_t njobs, const int32_t* const* plans, float* const* scratch, int32_t n_blocks,
                           const float* const* x_lo, const int64_t* ld_lo, const float* const* x_hi,
                           const int64_t* ld_hi, const int64_t* split, float alpha, float beta, float* const* y,
                           const int64_t* ld_y, int32_t wpx, void* stream);

int gmr_spmm_csr_f32(const int32_t* rowptr, const int32_t* col, const float* val, int64_t n_rows, int64_t nnz,
                     const int32_t* plan, int32_t seg_nnz, float* partial, int32_t n_blocks,
                     const float* const* x_lo, const int64_t* ld_lo, const float* const* x_hi, const int64_t* ld_hi,
                     int64_t split, float alpha, float beta, float* y, int64_t ldy, int32_t flags, void* stream);

/* ---------------------------------------------------------------- K9b fp16 scoring (opt-in)
 * C (E x I, fp32) = fp16(A) (E x 64) . fp16(B)^T, fp32 accumulation on v_mfma_f32_32x32x16_f16;
 * the fp16 MFMA scoring GEMM of BASELINE config 5, replacing the fp32 product of
 * GenRecV1.full_sort_predict (models/genrecv1.py:419-427) when scoring_dtype = fp16.  A and B
 * are fp32 and rounded on load.  d must be 64. */
int gmr_score_f16(int64_t E, int64_t I, int64_t d, const float* A, int64_t lda, const float* B, int64_t ldb,
                  float* C, int64_t ldc, void* stream);

/* ---------------------------------------------------------------- K11 graph construction
 * Symmetric-normalised bipartite adjacency (N = U + I) in CSR from a user->items CSR
 * (items ascending and distinct per user).  Replaces DiffMM.get_norm_adj_mat
 * (models/diffmm.py:88-107: self_loops=0, deg_eps=1e-7) and DiffMMTrainer.buildUIMatrix +
 * normalizeAdj (common/trainer.py:464-485: self_loops=1, deg_eps=0).  rowptr: N+1, col/val:
 * gmr_bipartite_nnz(...) entries, workspace: gmr_bipartite_workspace_ints(...) ints. */
int64_t gmr_bipartite_nnz(int64_t n_users, int64_t n_items, int64_t n_user_items, int32_t self_loops);
int64_t gmr_bipartite_workspace_ints(int64_t n_users, int64_t n_items);
int gmr_bipartite_symnorm_build(int64_t n_users, int64_t n_items, const int32_t* user_ptr, const int32_t* user_items,
                                int64_t n_user_items, int32_t self_loops, double deg_eps, int32_t* workspace,
                                int32_t* rowptr, int32_t* col, float* val, void* stream);
/* per-user top-k item lists (n_users x k, ld) -> user CSR with items sorted (trainer.py:545-562) */
int gmr_topk_to_user_csr(int64_t n_users, int32_t k, const int32_t* topk, int64_t ld, int32_t* user_ptr,
                         int32_t* user_items, void* stream);

/* ---------------------------------------------------------------- K3/K4/K6/K9 dense GEMM (fp32 operands)
 * C[M,N] = epilogue(alpha * op(A) op(B)); op(A) = A (M x K, lda) or A^T (A stored K x M);
 * op(B) = B (K x N, ldb) or B^T (B stored N x K).  bias[(bias_row ? bias_row[m] : 0)*ld_bias + n].
 * Replaces nn.Linear / torch.mm / matmul: diffmm.py:117,124,277,352-358,472-473; vbpr.py:70,105.
 * tile: 0 auto, 64, 128, 256, 256128 (256 x 128), 128256 or 12864 (128 x 64, fp32 kernel only), optionally | GMR_GEMM_MFMA16 (v_mfma_f32_16x16x4_f32)
 * or | GMR_GEMM_MFMA32 (v_mfma_f32_32x32x2_f32) to force the matrix instruction, | GMR_GEMM_REGSTAGE /
 * GMR_GEMM_GLDS to force register or global_load_lds operand staging (same sums, bit for bit);
 * split_k: 0 auto, else >= 1.
 * gmr_gemm_workspace_floats returns the exact scratch the same call needs (GMR_GEMM_COUNTER_WORDS
 * tile counters + splits*M*N floats of split-K partials, 0 when it does not split); the counter
 * words must be zero before the first call (they are left zero).  The split slabs are summed in
 * slab order by a reduce pass; the environment switch GMR_GEMM_FIXUP=1 instead has the last slice
 * of each tile sum them in-launch (same order and bits; slower on gfx950).
 * GMR_GEMM_GROUP=G (tuning) walks G tile rows per column inside each XCD's tile range.
 * Split-bf16 products (gemm_x6.hip): NT calls (trans_a = 0, trans_b = 1) with 16-byte aligned A / B and
 * lda, ldb multiples of 4 on a >= 128^2 tile run on the bf16 matrix cores with every fp32 operand split
 * exactly into three bf16 terms and six products accumulated in fp32 (fp32-accurate: error vs fp64 within
 * the fp32-MFMA kernel's bound, tests/test_kernels_gpu.py); | GMR_GEMM_X6 forces it, | GMR_GEMM_F32 (or
 * any staging / MFMA-shape flag) keeps the fp32-input MFMA, and the environment variable GMR_GEMM_X6=0
 * turns it off for every call.  gmr_gemm_kernel_kind returns the matrix path a call with these
 * arguments takes: 6 (split-bf16), 32 (v_mfma_f32_32x32x2_f32) or 16 (v_mfma_f32_16x16x4_f32). */
int32_t gmr_gemm_kernel_kind(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K, int32_t tile,
                             int32_t split_k, int32_t aligned);
int64_t gmr_gemm_workspace_floats(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K, int32_t tile,
                                  int32_t split_k);
int gmr_gemm_f32(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                 int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc, int32_t epilogue,
                 const float* bias, const int32_t* bias_row, int64_t ld_bias, const float* aux, int64_t ld_aux,
                 const float* rowvec1, const float* rowvec2, float slope, int32_t tile, int32_t split_k,
                 float* workspace, int64_t workspace_floats, void* stream);

/* bf16 plane sets (csrc/planes.hip): an fp32 matrix as three bf16 matrices (uint16 storage) [3][rows][ld]
 * with plane stride ps, x = hi + mid + lo exactly for every fp32 x (the split of GMR_GEMM_X6); ld is a
 * multiple of 32 and the columns [cols, ld) are zero.  gmr_split3_planes writes one from an fp32 matrix
 * (the item table of gmr_score_topk_x6).  (Round 4's pre-split GEMM gmr_gemm_p3_f32 was removed in round 5:
 * slower in the epoch and less accurate at K = 7,050 than the on-the-fly split of gmr_gemm_f32.) */
int gmr_split3_planes(int64_t rows, int64_t cols, const float* src, int64_t ld_src, uint16_t* dst, int64_t ld_dst,
                      int64_t plane_stride, void* stream);

/* ---------------------------------------------------------------- DiffMM rec step (diffmm.py:129-258)
 * Fused row kernels of forward_MM / forward_cl_MM / calculate_loss and their backward
 * (layouts in csrc/diffmm.hip). */
int gmr_dmm_combine_fwd(int64_t n, float* G, const float* H, const float* Qi, const float* Qt, const float* mw,
                        float lam, float* M, void* stream);
int gmr_dmm_final_fwd(int64_t n, const float* M, const float* L, float ris, float* Emb, float* nrm, void* stream);
int gmr_dmm_cl_fwd(int64_t n, const float* Qi, const float* Qt, const float* K2, float* CLN, float* nrm,
                   void* stream);
int gmr_dmm_final_bwd(int64_t n, const float* dEmb, const float* T1, const float* M, const float* nrmM, float ris,
                      const float* E, const float* mw, float* dE, float* partials, void* stream);
int64_t gmr_dmm_final_bwd_partials(int64_t n);
int gmr_dmm_mw_grad(int64_t nparts, const float* partials, const float* mw, float* dmw, int32_t accumulate,
                    void* stream);
int gmr_dmm_dg(int64_t n, int64_t U, const float* dE, const float* T2, float* dG, void* stream);
int gmr_dmm_cl_bwd(int64_t n, const float* dK, const float* T, const float* dE, float lam, float* Ri, float* Rt,
                   void* stream);
int gmr_dmm_assemble(int64_t n, int64_t U, const float* T2, const float* T3, const float* Ri, const float* Rt,
                     const float* E0, float reg2, float* dE0, float* dNF, void* stream);
/* Round 6: the rec step's small passes folded into their neighbours (same reference lines).
 * final_bwd2: clear != 0 zeroes dEmb after reading it (its last reader; the next step's sorted scatter adds onto
 *   zeros, so no fill pass); Ri / Rt (both or neither): also write lam * dE_img / lam * dE_txt into their left
 *   halves (what gmr_dmm_cl_bwd writes there).
 * cl_bwd2: clear != 0 zeroes dK[:, :64] after reading it; left = 0 leaves Ri / Rt's left halves alone.
 * assemble2: dNF leaves through the modality projections' normalize + leaky-ReLU backward (NF = the normalised
 *   projections I x 128, nrmF = their norms [2][I], slope) - gmr_normalize_rows_bwd_f32 on each half, same bits;
 *   dK_clear (N x 128, optional): its [:, :64] half is zeroed (the contrastive view gradient's last reader);
 *   t3u_from_t2: T3's user rows are read from T2 (they are equal: adj is bipartite) - T3 holds item rows only.
 * bpr_sqnorm: gmr_bpr_fwd_bwd and gmr_sqnorm_part_f32(n_sq, x, sq_parts) in one launch (same bits).
 * loss_mw: gmr_dmm_loss_total (+ acc[0] += loss when acc is not NULL: the trainer's epoch-loss sum) and
 *   gmr_dmm_mw_grad (accumulate 0) in one two-block launch. */
int gmr_dmm_final_bwd2(int64_t n, float* dEmb, const float* T1, const float* M, const float* nrmM, float ris,
                       const float* E, const float* mw, float* dE, float* partials, int32_t clear, float lam, float* Ri,
                       float* Rt, void* stream);
int gmr_dmm_cl_bwd2(int64_t n, float* dK, const float* T, const float* dE, float lam, float* Ri, float* Rt,
                    int32_t clear, int32_t left, void* stream);
int gmr_dmm_assemble2(int64_t n, int64_t U, const float* T2, const float* T3, const float* Ri, const float* Rt,
                      const float* E0, float reg2, float* dE0, float* dNF, const float* NF, const float* nrmF,
                      float slope, float* dK_clear, int32_t t3u_from_t2, void* stream);
int gmr_dmm_bpr_sqnorm(int32_t B, int64_t U, const float* Emb, const int32_t* users, const int32_t* pos,
                       const int32_t* neg, float* loss, float* contrib, float inv_norm, int64_t n_sq, const float* x,
                       double* sq_parts, void* stream);
int gmr_dmm_loss_mw(int64_t B, const float* loss_bpr, float inv_nr, const double* parts, int64_t nparts,
                    float reg_scale, const float* loss_cu, const float* loss_ci, float ssl_scale, float* out,
                    float* acc, int64_t n_mw_parts, const float* mw_parts, const float* mw, float* dmw, void* stream);

/* F.normalize (p=2, eps=1e-12) over rows and its backward (optionally fused with leaky-ReLU backward) */
int gmr_normalize_rows_f32(int64_t n, int32_t cols, const float* x, int64_t ldx, float* y, int64_t ldy, float* nrm,
                           void* stream);
int gmr_normalize_rows_bwd_f32(int64_t n, int32_t cols, const float* y, int64_t ldy, const float* nrm, const float* dy,
                               int64_t lddy, float* dx, int64_t lddx, float slope, int32_t accumulate, void* stream);

/* K7 BPR: -log(1e-10 + sigmoid(<a,p> - <a,n>)) with gathers; per-row loss + 3B contribution rows
 * (diffmm.py:220-227, common/loss.py:33-37) */
int gmr_bpr_fwd_bwd(int32_t B, int64_t U, const float* Emb, const int32_t* users, const int32_t* pos,
                    const int32_t* neg, float* loss, float* contrib, float inv_norm, void* stream);
/* K8 InfoNCE pieces (diffmm.py:251-258): in-place row softmax of logits with log-sum-exp out,
 * and the per-row terms of the gathered batch */
/* VBPR calculate_loss (models/vbpr.py:76-97; common/loss.py BPRLoss + EmbLoss): rows of one
 * (U + I) x D table (items at item_off); loss = mean -log(1e-10 + sigmoid(<u,p> - <u,n>)) +
 * reg_weight * (||U||_F + ||P||_F + ||N||_F) / B; contrib = [dU; dP; dN] (3B x D) for
 * gmr_scatter_sorted_f32.  Workspaces: x_ws B floats, sq_ws 3B doubles, coef_ws 3 floats. */
int gmr_vbpr_loss_fwd_bwd(int32_t B, int32_t D, const float* table, int64_t ldt, const int32_t* users,
                          const int32_t* pos, const int32_t* neg, int64_t item_off, float reg_weight, float* x_ws,
                          double* sq_ws, float* coef_ws, float* loss, float* contrib, int64_t ldc, void* stream);
int gmr_fill2d_f32(int64_t rows, int64_t cols, float* p, int64_t ld, float value, void* stream);
int gmr_row_softmax_f32(int64_t rows, int64_t cols, float* L, int64_t ld, float coef, float* lse, void* stream);
int gmr_contrast_rows(int32_t B, const float* CLN, const int32_t* nodes, int64_t node_off, const float* lse,
                      float inv_temp, float coef, float* loss, float* contrib, int64_t ld_contrib, void* stream);
/* K8 fused InfoNCE: forward + backward of DiffMM.contrastLoss (models/diffmm.py:251-258) for one
 * gathered batch, replacing the logits GEMM + row softmax + two gradient GEMMs.  P = view-1 rows of
 * the batch (B x 64, ldp; P_i = CLN[node_off + nodes[i], 0:64]), T = the view-2 table (n x 64, ldt),
 * CLN = the N x 128 [view 1 | view 2] table.  Writes loss[i] = log sum_j exp(<P_i,T_j>/temp) -
 * <P_i,T_node(i)>/temp; contrib[i, 0:64] = dL/dP_i and contrib[i, 64:128] = -coef/temp P_i (the
 * T_node(i) term, for the caller's scatter); dT (n x 64, ld_dt, overwritten) = the dense table
 * gradient; gradients scaled by coef.  No B x n matrix in HBM; f32 MFMA; deterministic.
 * P = NULL (round 6): the passes read P_i = CLN[node_off + nodes[i], 0:64] in place, ldp = CLN's leading
 * dimension (no gathered copy; the default pipelined split-bf16 passes only, else an argument error).
 * workspace: gmr_contrast_workspace_floats(B, n) floats. */
int64_t gmr_contrast_workspace_floats(int32_t B, int64_t n);
int gmr_contrast_fused_f32(int32_t B, int64_t n, const float* P, int64_t ldp, const float* T, int64_t ldt,
                           const float* CLN, const int32_t* nodes, int64_t node_off, float inv_temp, float coef,
                           float* loss, float* contrib, int64_t ld_contrib, float* dT, int64_t ld_dt, float* workspace,
                           int64_t workspace_floats, void* stream);
/* The same with dT taken through the normalize backward of the table's view in the reduce pass (y = the
 * normalised table rows n x 64, ldy; nrm = their norms): dT = nbwd(dense gradient).  DiffMM: the dense part of
 * dK[:, 64:] (contrastLoss's F.normalize, diffmm.py:252-253); the sparse part goes through
 * gmr_scatter_sorted_nbwd_f32 (the normalize backward is linear in its input). */
int gmr_contrast_fused_nbwd_f32(int32_t B, int64_t n, const float* P, int64_t ldp, const float* T, int64_t ldt,
                                const float* CLN, const int32_t* nodes, int64_t node_off, float inv_temp, float coef,
                                float* loss, float* contrib, int64_t ld_contrib, float* dT, int64_t ld_dt,
                                const float* y, int64_t ldy, const float* nrm, float* workspace,
                                int64_t workspace_floats, void* stream);
/* K2 gather / deterministic scatter-add through a sorted (key << 32 | slot) plan */
int gmr_gather_rows_f32(int32_t B, int32_t cols, const float* src, int64_t lds, const int32_t* idx, int64_t off,
                        float* out, int64_t ldo, void* stream);
int gmr_scatter_sorted_f32(int32_t n, int32_t cols, const uint64_t* plan, const float* contrib, int64_t ldc,
                           float* dst, int64_t ldd, void* stream);
/* 128-wide contribution rows through the plan, each 64-column half taken through the normalize backward of the
 * contrastive view it belongs to (y = CLN, N x 128; nrm = [2][n_nodes] norms) and ADDED to dK (N x 128):
 * dK[key] += [nbwd(s[:64]) | nbwd(s[64:])]  (DiffMM contrastLoss's sparse terms, diffmm.py:252-258) */
int gmr_scatter_sorted_nbwd_f32(int32_t n, const uint64_t* plan, const float* contrib, int64_t ldc, const float* y,
                                const float* nrm, int64_t n_nodes, float* dK, void* stream);
int gmr_sort_batch_keys(int64_t n_batches, const int32_t* keys, const int64_t* offsets, const int32_t* key_add,
                        int32_t n_keysets, int64_t key_stride, uint64_t* out, int64_t out_stride, int32_t pow2,
                        void* stream);
/* deterministic reductions */
int gmr_sum_f32(int64_t n, const float* x, float scale, float* out, int32_t accumulate, void* stream);
#define GMR_SQNORM_PARTS 1024 /* workspace doubles of gmr_sqnorm_f32 */
int gmr_sqnorm_f32(int64_t n, const float* x, float scale, float* out, int32_t accumulate, double* workspace,
                   void* stream);
/* The same as two steps: per-block fp64 partials (gmr_sqnorm_nparts(n) of them) into workspace,
 * then gmr_dmm_loss_total sums them in order with the other loss terms of DiffMM.calculate_loss
 * (models/diffmm.py:203-249): out = sum(bpr)*inv_nr + reg*|x|^2 + ssl*(sum(cu) + sum(ci)), one
 * launch and the same float value as the four separate reductions. */
int64_t gmr_sqnorm_nparts(int64_t n);
int gmr_sqnorm_part_f32(int64_t n, const float* x, double* workspace, void* stream);
int gmr_dmm_loss_total(int64_t B, const float* loss_bpr, float inv_nr, const double* parts, int64_t nparts,
                       float reg_scale, const float* loss_cu, const float* loss_ci, float ssl_scale, float* out,
                       void* stream);
int gmr_sum_f64(int64_t n, const double* x, double scale, double* out, int32_t accumulate, void* stream);
int gmr_colsum_f32(int64_t rows, int64_t cols, const float* x, int64_t ld, const int32_t* group, int32_t n_groups,
                   float* out, int32_t accumulate, void* stream);

/* column sums over few columns with the rows split 32 ways (fixed-order partials; workspace
 * gmr_colsum_split_floats(cols) floats) — bias gradients of the B x 512 transformer products */
int64_t gmr_colsum_split_floats(int64_t cols);
int gmr_colsum_split_f32(int64_t rows, int64_t cols, const float* x, int64_t ld, float* out, int32_t accumulate,
                         float* workspace, int64_t workspace_floats, void* stream);

/* ---------------------------------------------------------------- BPR epoch sampler (dataloader.py:218-275)
 * shuffled interactions + one rejection-sampled negative from `all_items` per interaction (redrawn while
 * in the user's history); rows still without a true negative after 4096 draws are added to
 * *n_fallback (may be NULL; the caller zeroes it) and keep their last draw. */
int gmr_sample_epoch(int64_t n_inter, const int32_t* inter_user, const int32_t* inter_item, const int32_t* user_rowptr,
                     const int32_t* user_items, const int32_t* all_items, int64_t n_all_items, uint64_t seed,
                     uint64_t epoch, int32_t* out_users, int32_t* out_pos, int32_t* out_neg, int32_t* n_fallback,
                     void* stream);
/* random permutation of [0, n) (DataLoader(shuffle=True) over users, trainer.py:462) */
int gmr_permutation(int64_t n, uint64_t seed, uint64_t epoch, int32_t* out, void* stream);

/* ---------------------------------------------------------------- K5/K6 diffusion (diffmm.py:408-484, diffrec.py:182-310)
 * x_t = sqrt_ac[t]*x0 + sqrt_1mac[t]*eps, times the Denoise input dropout keep/keep_prob when
 * dropout != 0; x0 rows come from the user's train items.  noise/keep may be NULL (Philox).
 * row0: index of row 0 inside the global batch — the Philox draws of a row depend on
 * (seed, step, row0 + b) only, so a batch split over data-parallel ranks draws what one
 * process drawing the whole batch would (trainer.py:491-527). */
int gmr_diff_sample_t(int32_t B, int32_t T, uint64_t seed, uint64_t step, int64_t row0, int32_t* t, void* stream);
int gmr_diff_qsample(int32_t B, int32_t I, const int32_t* users, const int32_t* user_ptr, const int32_t* user_items,
                     const int32_t* t, const float* sqrt_ac, const float* sqrt_1mac, const float* noise,
                     int64_t ld_noise, const float* keep, int64_t ld_keep, float keep_prob, int32_t dropout,
                     uint64_t seed, uint64_t step, int64_t row0, float* x, int64_t ldx, void* stream);
int gmr_diff_densify(int32_t B, int32_t I, const int32_t* users, const int32_t* user_ptr, const int32_t* user_items,
                     float* x, int64_t ldx, void* stream);
int gmr_diff_time_bias(int32_t T, int32_t E, const float* emb_W, const float* emb_b, const float* W1, int64_t ld_w1,
                       int64_t col_off, const float* b1, int32_t H, float* EB, float* temb_out, float* emb_out,
                       void* stream);
int gmr_diff_loss_rows(int32_t B, int32_t I, const int32_t* users, const int32_t* user_ptr, const int32_t* user_items,
                       const int32_t* t, const double* wtab, const float* pt, float* out, int64_t ld, float grad_scale,
                       double* mse_out, double* diff_out, double* loss_out, int32_t write_grad, void* stream);
/* out[c][r] = in[r][c] for a rows x cols fp32 matrix. */
int gmr_transpose_f32(int64_t rows, int64_t cols, const float* in, int64_t ldi, float* out, int64_t ldo,
                      void* stream);
/* First p_sample step on binary x0 rows (models/diffmm.py:408-426 with steps = 0, the loop's
 * first model call): h[b] = tanh(sum over the user's items i of W1T[i, :] + eb), W1T = W1[:, :I]^T
 * (I x H) — the sparse form of the hidden GEMM. */
int gmr_diff_sparse_hidden(int32_t B, int32_t H, const int32_t* users, const int32_t* user_ptr,
                           const int32_t* user_items, const float* W1T, int64_t ldw, const float* eb, float* h,
                           int64_t ldh, void* stream);
/* Folded p_sample chain (round 5; the same p_sample, models/diffmm.py:408-451 and models/diffrec.py:291-310,
 * carried as the hidden pre-activation a = x_t W1[:, :I]^T instead of x_t: a_i = c1_i (h_i P^T + v) +
 * c2_i a_{i+1} with P = W1[:, :I] W2 (H x H), v = W1[:, :I] b2; gmr/denoise.py p_sample_fold).
 * gmr_diff_sparse_pre: the first step from binary x0 rows, a[b] = sum over the user's items of W1T[i, :]
 * and h[b] = tanh(a[b] + eb) (h bit-identical to gmr_diff_sparse_hidden).
 * gmr_tanh_bias_f32: h = tanh(a + bias) per row (rows x cols, cols % 4 == 0, 16-byte aligned). */
int gmr_diff_sparse_pre(int32_t B, int32_t H, const int32_t* users, const int32_t* user_ptr, const int32_t* user_items,
                        const float* W1T, int64_t ldw, const float* eb, float* a, int64_t lda, float* h, int64_t ldh,
                        void* stream);
int gmr_tanh_bias_f32(int64_t rows, int32_t cols, const float* a, int64_t lda, const float* bias, float* h,
                      int64_t ldh, void* stream);
/* DiffRec importance sampling of t (models/diffrec.py:234-250): uniform t and pt = 1 until every
 * t has hist_len recorded losses, then t ~ (1-up) sqrt(mean(hist^2))/sum + up/T, pt = p[t]*T. */
int gmr_diff_sample_t_importance(int32_t B, int32_t T, int32_t hist_len, const double* hist, const int32_t* count,
                                 double uniform_prob, uint64_t seed, uint64_t step, int64_t row0, int32_t* t,
                                 float* pt, void* stream);
/* Lt_history / Lt_count update (models/diffrec.py:279-286), rows applied in batch order; t < 0 skips. */
int gmr_diff_history_update(int32_t B, int32_t T, int32_t hist_len, const int32_t* t, const double* loss,
                            double* hist, int32_t* count, void* stream);
int gmr_diff_gc_rows(int32_t B, const int32_t* users, const int32_t* user_ptr, const int32_t* user_items,
                     const float* item_embeds, int64_t ld_ie, const float* Z, int64_t ldz, float gscale, float* G,
                     int64_t ldg, double* gc_out, void* stream);
int gmr_diff_time_bwd(int32_t T, int32_t E, int32_t H, const float* S, const float* temb, const float* emb,
                      const float* W1, int64_t ld_w1, int64_t col_off, float* dW1, float* db1, float* d_emb_W,
                      float* d_emb_b, int32_t accumulate, void* stream);

/* ---------------------------------------------------------------- K10/K12 eval tail (trainer.py:369-388)
 * ties -> lowest index; k <= 64 */
int gmr_mask_scores_f32(int64_t n, const int32_t* rows, const int32_t* cols, float* scores, int64_t ld, float fill,
                        void* stream);
int gmr_topk_rows_f32(int64_t n_rows, int64_t n_cols, const float* scores, int64_t ld, int32_t k, int32_t* out_idx,
                      int64_t ld_idx, float* out_val, void* stream);
/* K9 + K10 fused (common/trainer.py:379-386 with models/diffmm.py:276-277): per eval row r,
 * scores = user_table[users[r]] . item_table^T (users NULL: row r is user r), the row's train positives
 * mask_cols[mask_ptr[r] .. mask_ptr[r+1]) (sorted ascending within a row) set to `fill` (-1e10), then
 * the top-k item indices (score desc, ties -> lowest index) into out_idx[r * ld_idx + j] and,
 * if out_val is not NULL, their scores.  No n_rows x n_items buffer; dim 64 or 128; k <= 64.
 * mask_ptr holds n_rows + 1 absolute offsets into mask_cols (pass &ptr[first row] for a slice). */
int gmr_score_topk_f32(int64_t n_rows, const int32_t* users, const float* user_table, int64_t ld_user, int64_t n_items,
                       const float* item_table, int64_t ld_item, int64_t dim, const int64_t* mask_ptr,
                       const int32_t* mask_cols, float fill, int32_t k, int32_t* out_idx, int64_t ld_idx,
                       float* out_val, void* stream);
/* The same with the scores on the bf16 matrix cores (round 4): the item table as a plane set
 * (gmr_split3_planes: item_planes[p * plane_stride + i * ld_plane + c], x = hi + mid + lo exactly) and
 * the six-product split of GMR_GEMM_X6 (fp32-accurate sums, 2.7x the fp32 MFMA rate); the user
 * table stays fp32 and is split in registers.  dim 64; ld_plane a multiple of 8. */
int gmr_score_topk_x6(int64_t n_rows, const int32_t* users, const float* user_table, int64_t ld_user, int64_t n_items,
                      const uint16_t* item_planes, int64_t ld_plane, int64_t plane_stride, int64_t dim,
                      const int64_t* mask_ptr, const int32_t* mask_cols, float fill, int32_t k, int32_t* out_idx,
                      int64_t ld_idx, float* out_val, void* stream);
/* Recall/NDCG/Precision/MAP sums over users at ks (topk_evaluator.py:107-120, metrics.py):
 * out_sums[metric*8 + j], metric 0 recall 1 ndcg 2 precision 3 map, j < n_ks (fp64). */
int64_t gmr_eval_metrics_partials(int64_t n_users);
int gmr_eval_metrics(int64_t n_users, const int32_t* topk, int64_t ld_topk, int32_t K, const int64_t* pos_ptr,
                     const int32_t* pos_items, int32_t n_ks, const int32_t* ks, double* partials, double* out_sums,
                     void* stream);
/* The same sums over the eval-user rows sel[0 .. n_sel) only, each scored against its own row of
 * (pos_ptr, pos_items): the test-time group metrics (Pop/Niche positives, Cold/Warm users,
 * topk_evaluator.py:122-200).  partials: gmr_eval_metrics_partials(n_sel) doubles. */
int gmr_eval_metrics_sel(int64_t n_sel, const int32_t* sel, const int32_t* topk, int64_t ld_topk, int32_t K,
                         const int64_t* pos_ptr, const int32_t* pos_items, int32_t n_ks, const int32_t* ks,
                         double* partials, double* out_sums, void* stream);
/* counts[j * n_items + i] = times item i appears in the first ks[j] columns of topk (ks ascending, <= 64, n_ks <= 8):
 * Coverage / Gini / Tail% (topk_evaluator.py:212-270). */
int gmr_topk_item_counts(int64_t n_users, const int32_t* topk, int64_t ld_topk, int32_t n_ks, const int32_t* ks,
                         int64_t n_items, int32_t* counts, void* stream);

/* ---------------------------------------------------------------- GenRecV1 rec step (models/genrecv1.py:225-427)
 * Tables are rows x 64 fp32.  BatchNorm1d(64) (eps, momentum as nn.BatchNorm1d): train mode uses
 * batch statistics and updates run_mean/run_var (unbiased var); eval mode uses them.  Fused:
 * y = act(BN(z)) [* keep * keep_scale] (act 0 none, 1 leaky(slope), 2 sigmoid, 3 tanh) and the
 * post op: 0 none, 1 out2 = rs[0]*aux + y (res_scale residual, :229), 2 out2 = aux*y (gate product,
 * :268), 3 rowdot[r] = <y_r, aux[0:64]> (Linear(64, 1, bias=False), :88).
 * Replaces nn.BatchNorm1d + activation + Dropout chains at genrecv1.py:84-89,155-164,166-222.
 * parts: gmr_bn_parts_doubles(rows) doubles; mean/invstd: 64 floats each (saved for backward). */
int64_t gmr_bn_parts_doubles(int64_t rows);
int gmr_bn_fwd_f32(int64_t rows, const float* z, int64_t ldz, int32_t train, float eps, float momentum, float* run_mean,
                   float* run_var, double* parts, float* mean, float* invstd, const float* w, const float* b,
                   int32_t act, float slope, const uint8_t* keep, int64_t ld_keep, float keep_scale, float* y,
                   int64_t ldy, int32_t post, const float* aux, int64_t ld_aux, const float* rs, float* out2,
                   int64_t ld2, float* rowdot, void* stream);
/* backward of the above (train mode): upstream = dy (* mul) or, for post 3, da[r] * v[c]; writes
 * dz (accumulated if asked), dw/db (and dv for post 3; accumulated if asked); sums: 128 floats. */
int gmr_bn_bwd_f32(int64_t rows, const float* z, int64_t ldz, const float* mean, const float* invstd, const float* w,
                   const float* b, int32_t act, float slope, const uint8_t* keep, int64_t ld_keep, float keep_scale,
                   const float* dy, int64_t lddy, const float* mul, int64_t ld_mul, const float* da, const float* v,
                   double* parts, float* sums, float* dw, float* db, float* dv, int32_t accumulate_params, float* dz,
                   int64_t lddz, int32_t accumulate_dz, void* stream);
/* content = w0 (E + A1)/2 + w1 (E + A2)/2, w = softmax(origin_weight, generation_weight) (:255-264,:332-336)
 * and its backward (T_k = A_k^T dC; dE += ... + reg2 E; d(ow, gw) accumulated); parts: gmr_gr_parts doubles */
int64_t gmr_gr_parts(int64_t n);
int gmr_gr_content_fwd(int64_t n, const float* E, const float* A1, const float* A2, const float* ow, const float* gw,
                       float* C, void* stream);
int gmr_gr_content_bwd(int64_t n, const float* E, const float* A1, const float* A2, const float* dC, const float* T1,
                       const float* T2, const float* ow, const float* gw, float reg2, double* parts, float* dE,
                       float* dow, float* dgw, void* stream);
/* gate_attention_fusion + prefer gates (:309-353): SIDE = (PI (IMG-COM) + PT (TXT-COM) + COM)/4 */
int gmr_gr_fusion_fwd(int64_t n, const float* IMG, const float* TXT, const float* aI, const float* aT,
                      const float* PI, const float* PT, float* SIDE, float* alpha, void* stream);
int gmr_gr_fusion_bwd(int64_t n, const float* IMG, const float* TXT, const float* alpha, const float* PI,
                      const float* PT, const float* dSIDE, float* dIMG, float* dTXT, float* daI, float* daT,
                      float* dPI, float* dPT, void* stream);
/* out (+)= scale * a * b (rows x 64); out = sum(a * b) * scale (+ out), deterministic (parts >= 1024 doubles) */
int gmr_mul64_f32(int64_t rows, const float* a, int64_t lda, const float* b, int64_t ldb, float* out, int64_t ldo,
                  float scale, int32_t accumulate, void* stream);
int gmr_dot64_f32(int64_t rows, const float* a, int64_t lda, const float* b, int64_t ldb, double* parts, float scale,
                  float* out, int32_t accumulate, void* stream);
/* InfoNCE rows on L = v1 v2^T / temp (B x B, in place; :407-414): loss[r] = lse(L_r) - L_rr and
 * L <- coef (softmax - I) for the two gradient GEMMs (coef 0: loss only) */
int gmr_nce_rows_f32(int64_t B, float* L, int64_t ld, float coef, float* loss, void* stream);
/* the same for a data-parallel rank's block: rows [diag_off, diag_off + rows) of the global batch
 * against all cols keys (row r's positive at column diag_off + r; genrecv1.py:407-414 over the
 * global batch) */
int gmr_nce_rows_off_f32(int64_t rows, int64_t cols, float* L, int64_t ld, int64_t diag_off, float coef, float* loss,
                         void* stream);
/* GenRecV1's in-batch InfoNCE terms through gmr_contrast_fused_f32 (round 4; genrecv1.py:389-397): term k
 * pairs the normalised query table i1[k] with key table i2[k] of nv [4][tab][64] (i1 / i2: host arrays of
 * nterms <= 4 entries; Bg rows used per table).  gmr_nce_pairs_f32 writes the (query, positive) pair rows
 * CLN [nterms][ct][128] of the rank's rows [row0, row0 + B); after one contrast call per term (contrib
 * [nterms][ct][128], dT [nterms][dts][64]) gmr_nce_combine_f32 writes every nv row's gradient g [4][tab][64],
 * summed in term order. */
int gmr_nce_pairs_f32(int32_t nterms, int64_t B, int64_t Bg, int64_t row0, const int32_t* i1, const int32_t* i2,
                      const float* nv, int64_t tab, float* cln, int64_t ct, void* stream);
int gmr_nce_combine_f32(int32_t nterms, int64_t B, int64_t Bg, int64_t row0, const int32_t* i1, const int32_t* i2,
                        const float* contrib, int64_t ct, const float* dT, int64_t dts, float* g, int64_t tab,
                        void* stream);
/* BPR with log-sigmoid (:377-380) over one (U + I) x 64 table; contrib = [dU; dP; dN] */
int gmr_bpr_logsigmoid_f32(int32_t B, int64_t U, const float* C, const int32_t* users, const int32_t* pos,
                           const int32_t* neg, float* loss, float* contrib, float inv_norm, void* stream);

/* y += alpha[0] x (device scalar); out = a * b (flat); Bernoulli(p_keep) keep bytes (nn.Dropout masks) */
int gmr_axpy_dev_f32(int64_t n, const float* alpha, const float* x, float* y, void* stream);
int gmr_mul_f32(int64_t n, const float* a, const float* b, float* out, void* stream);
/* keep byte i uses Philox counter ctr0 + i (a data-parallel rank's rows: ctr0 = first global row x row length) */
int gmr_keep_mask_u8(int64_t n, float p_keep, uint64_t seed, uint64_t step, uint64_t ctr0, uint8_t* out, void* stream);

/* ---------------------------------------------------------------- GenRecV1 graphs (§8a G2, G6)
 * CSR transpose (columns ascending in every output row, values carried); workspace 2*n_cols ints,
 * stage_col/stage_val nnz entries.  Backward of the non-symmetric SpMMs (dropped UI graph, kNN, R). */
int gmr_csr_transpose(int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t* rowptr, const int32_t* col,
                      const float* val, int32_t* workspace, int32_t* t_rowptr, int32_t* t_col, float* t_val,
                      int32_t* stage_col, float* stage_val, void* stream);
/* SpAdjDropEdge (:443-457): keep e iff floor(u_e + keep_rate) >= 1 (Philox u, or keep[e]); values / keep_rate.
 * Two calls: counts + out_rowptr (workspace n_rows ints), then the compaction.  transposed = 1 on a
 * structurally symmetric matrix gives (dropped A)^T directly (entry (r, c) takes the flag of (c, r)). */
int gmr_csr_drop_count(int64_t n_rows, const int32_t* rowptr, const int32_t* col, int32_t transposed,
                       const uint8_t* keep, float keep_rate, uint64_t seed, uint64_t step, int32_t* workspace,
                       int32_t* out_rowptr, void* stream);
int gmr_csr_drop_write(int64_t n_rows, const int32_t* rowptr, const int32_t* col, const float* val,
                       int32_t transposed, const uint8_t* keep, float keep_rate, uint64_t seed, uint64_t step,
                       const int32_t* out_rowptr, int32_t* out_col, float* out_val, void* stream);
/* kNN graph from per-row top-k (idx, sim) (utils/utils.py:184-197, 'sym'): deg = row sums of the
 * kept sims (top-k order), w = d_r v d_c, d = deg^-1/2 (inf -> 0); rowptr n+1, col/val n*k */
int gmr_knn_symnorm_csr(int64_t n, int32_t k, const int32_t* topi, int64_t ldi, const float* topv, int64_t ldv,
                        float* dis_ws, int32_t* rowptr, int32_t* col, float* val, void* stream);
/* rebuild (common/trainer.py:752-754): den = x0 with the gen_topk positions taken from xs */
int gmr_gen_mask(int32_t B, int32_t I, int32_t k, const int32_t* topi, int64_t ldt, const float* x0, const float* xs,
                 int64_t ld, float* den, void* stream);
/* InterestDebiase (interest_cluster.py:186-332): exact-n uniform picks of 0->1 / 1->0 flips among the
 * gen_topk positions (n = int(count * ratio)); picks[type][max_picks][2] = (row, item), n_picks[2];
 * then the cluster rules (labels < 64) applied to den in place */
int gmr_debias_select(int32_t B, int32_t k, const int32_t* topi, int64_t ldt, const float* x0, const float* xs,
                      int64_t ld, float ratio, uint64_t seed, uint64_t step, uint64_t* keys_ws /* 2*B*k */,
                      int32_t* picks, int32_t max_picks, int32_t* n_picks, void* stream);
int gmr_debias_apply(int32_t type, const int32_t* picks, const int32_t* n_picks, int32_t max_picks, const float* x0,
                     int64_t ld0, int32_t I, const int32_t* labels, float* den, int64_t ldd, void* stream);
/* K-means pieces (interest_cluster.py:60-79 — StandardScaler + KMeans): distances and centroid sums
 * are GEMMs (gmr_gemm_f32) between these calls */
int gmr_kmeans_standardize(int64_t n, int32_t d, const float* X, int64_t ldx, float* mean, float* scale, float* Y,
                           int64_t ldy, float* sq, void* stream);
int gmr_kmeans_pp_pick(int64_t n, const float* mind, uint64_t seed, uint64_t step, int32_t* out, void* stream);
int gmr_kmeans_take_center(int32_t d, const float* X, int64_t ldx, const int32_t* idx, float* C, int64_t ldc,
                           int32_t j, const float* xsq, float* csq, void* stream);
/* greedy k-means++ step (sklearn's default seeding: L = 2 + floor(ln k) candidates, round 4): given dots =
 * X . Cc^T (n x L) of the candidate rows Cc and their squared norms ccsq, picks the candidate of the lowest
 * potential sum_r min(mind[r], |x_r - c|^2) (fixed-order sums, ties -> lowest), copies it to C[j], sets
 * csq[j] and lowers mind. */
int gmr_kmeans_pp_greedy(int64_t n, int32_t L, const float* xsq, const float* dots, int64_t ldd, const float* ccsq,
                         float* mind, const float* Cc, int64_t ldcc, int32_t d, float* C, int64_t ldc, int32_t j,
                         float* csq, void* stream);
int gmr_kmeans_min_dist(int64_t n, const float* xsq, const float* dots, int64_t ld_dots, const float* csq, int32_t j,
                        float* mind, int32_t first, void* stream);
int64_t gmr_kmeans_parts(int64_t n);
int gmr_kmeans_assign(int64_t n, int32_t k, const float* dots, int64_t ldd, const float* csq, const float* xsq,
                      int32_t* label, float* onehot_t, int64_t ldo, int32_t* changed, double* inertia_parts,
                      void* stream);
int gmr_kmeans_centroids(int32_t k, int32_t d, const float* sums, int64_t lds, const float* onehot_t, int64_t ldo,
                         int64_t n, float* C, int64_t ldc, float* csq, void* stream);

/* ---------------------------------------------------------------- GenRecV1 generation (§8a G4, G5)
 * FlipInterestDiffusion (models/genrecv1.py:460-648).  tables = [gamma_cum (T) | eps_cum (T) |
 * pos_weight | sparsity] from the batch users' history sizes (get_cum, :480-498). */
int gmr_flip_schedule(int32_t B, const int32_t* users, const int32_t* user_ptr, int32_t I, int32_t T, float* tables,
                      void* stream);
/* q_sample (:512-526): x_t = x0 xor Bernoulli(sigmoid((a_t - u) temp)); flip (0/1 bytes) replaces the draws.
 * Draws are keyed by (step, global row row0 + b, item), so a data-parallel rank holding rows
 * [row0, row0 + B) of a batch draws what one process holding the whole batch draws. */
int gmr_flip_qsample(int32_t B, int32_t I, const float* x0, int64_t ld0, const int32_t* t, int32_t t_const,
                     const float* tables, int32_t T, float temp, const uint8_t* flip, int64_t ld_flip, uint64_t seed,
                     uint64_t step, int64_t row0, float* xt, int64_t ldt, void* stream);
/* one p_sample step on the model logits (:536-548); probs may be NULL; draws keyed as gmr_flip_qsample */
int gmr_flip_step(int32_t B, int32_t I, const float* z, int64_t ldz, const float* tables, int32_t T, int32_t qi,
                  int32_t last,
                  const uint8_t* draws, int64_t ldd, uint64_t seed, uint64_t step, int64_t row0, float* x, int64_t ldx,
                  float* probs, int64_t ldp, void* stream);
/* BCE(pos_weight) + curriculum KL rows (:550-627); dz = grad_scale * dBCE/dz (may alias z) */
int gmr_flip_loss_rows(int32_t B, int32_t I, const float* x0, int64_t ld0, const float* z, int64_t ldz,
                       const int32_t* t, const float* tables, int32_t T, float grad_scale, float* dz, int64_t lddz,
                       double* bce_row, double* kl_row, void* stream);
/* [bce, kl, cl, bce + kl + w_cl cl] (training_losses total, :604) */
int gmr_flip_total(const double* bce_kl, const float* cl, float w_cl, float* out4, void* stream);
/* ModalDenoiseTransformer rows (:650-710).  LayerNorm over D (64..1024) of s = a + keep*scale*b
 * (b a matrix, or a broadcast row when ldb == 0; keep may be NULL), optional exact GELU after;
 * saves s, mean, rstd.  Backward: dx (+)=, dw/db (+)= through parts (gmr_layernorm_parts_floats). */
int gmr_layernorm_fwd(int64_t rows, int32_t D, const float* a, int64_t lda, const float* b, int64_t ldb,
                      const uint8_t* keep, int64_t ld_keep, float keep_scale, const float* w, const float* bias,
                      float eps, int32_t gelu, float* y, int64_t ldy, float* s_out, int64_t lds, float* mean,
                      float* rstd, void* stream);
/* The same with the residual-branch dropout drawn in the kernel (nn.Dropout on the decoder layer's branch,
 * :650-710): keep_out[r][c] = (Philox(seed, step, ctr0 + r D + c).x >> 8) / 2^24 < p_keep (gmr_keep_mask_u8's
 * key, so the bytes equal a gmr_keep_mask_u8 draw of rows x D at ctr0) is stored and applied; one launch
 * instead of the mask launch + gmr_layernorm_fwd.  b must be a matrix (ldb > 0). */
int gmr_layernorm_drop_fwd(int64_t rows, int32_t D, const float* a, int64_t lda, const float* b, int64_t ldb,
                           float p_keep, uint64_t seed, uint64_t step, uint64_t ctr0, uint8_t* keep_out,
                           int64_t ld_keep, float keep_scale, const float* w, const float* bias, float eps,
                           int32_t gelu, float* y, int64_t ldy, float* s_out, int64_t lds, float* mean, float* rstd,
                           void* stream);
int64_t gmr_layernorm_parts_floats(int64_t rows, int32_t D);
int gmr_layernorm_bwd(int64_t rows, int32_t D, const float* s, int64_t lds, const float* mean, const float* rstd,
                      const float* w, const float* bias, int32_t gelu, const float* dy, int64_t lddy, float* dx,
                      int64_t lddx, int32_t accumulate_dx, float* parts, float* dw, float* db,
                      int32_t accumulate_params, void* stream);
/* adaLN (:702-703): h1 = h0 (1 + scale[t]) + shift[t], S = T x 2D [shift | scale]; backward writes
 * dh0 and prod = dh1 * h0 (grouped column sums give dscale / dshift, gmr_colsum_f32) */
int gmr_adaln_fwd(int64_t rows, int32_t D, const float* h0, int64_t ld0, const int32_t* t, int32_t t_const,
                  const float* S, int64_t lds, float* h1, int64_t ld1, void* stream);
int gmr_adaln_bwd(int64_t rows, int32_t D, const float* h0, int64_t ld0, const float* dh1, int64_t ldd,
                  const int32_t* t, const float* S, int64_t lds, float* dh0, int64_t ldo, float* prod, int64_t ldp,
                  void* stream);
/* dropout with keep probability p_keep, one draw per (row, column / group) (group = head size for
 * the attention-weight dropout of a length-1 sequence); mask_in replays a mask, mask_out records it */
int gmr_dropout_f32(int64_t rows, int32_t D, int32_t group, const float* x, int64_t ldx, float p_keep,
                    const uint8_t* mask_in, uint8_t* mask_out, int64_t ldm, uint64_t seed, uint64_t step, int64_t row0,
                    float* y, int64_t ldy, void* stream);
/* Cross-attention of the decoder layers on their all-zero memory (models/genrecv1.py:650-710): head h
 * outputs the value bias bv'_h on every row, so with head dropout the block is, per row, a mixture of
 * nhead fixed vectors.  gmr_xattn_table_f32: P[l][h][j] = sum_{c in head h} Wo_l[j][c] bv'_l[c] / p_keep
 * for the L layers (layer l's tensors at woc0 / bvc0 + l * layer_stride floats; Wo row-major, ld D).
 * gmr_xattn_fwd_f32: CA[r] = b_o + sum_h keep[r][h] P[h] (keep drawn as gmr_dropout_f32 with group
 * D / nhead draws it, or read from mask_in; mask_out records it).  gmr_xattn_bwd_f32: from dCA (B x D)
 * and the masks, dWo += Gs[h(c)][j] bv'[c] / p_keep and dbv' += sum_j Wo[j][c] Gs[h(c)][j] / p_keep,
 * Gs[h][j] = sum_r keep[r][h] dCA[r][j]; nhead <= 16; ws of gmr_xattn_bwd_workspace_floats floats.
 * They replace the B x D x D out-projection GEMM, its transposed-operand gradient and dBc products. */
int gmr_xattn_table_f32(int32_t L, int32_t D, int32_t nhead, const float* woc0, const float* bvc0,
                        int64_t layer_stride, float p_keep, float* P, void* stream);
int gmr_xattn_fwd_f32(int64_t rows, int32_t D, int32_t nhead, const float* P, const float* bo, float p_keep,
                      const uint8_t* mask_in, uint8_t* mask_out, int64_t ldm, uint64_t seed, uint64_t step, int64_t row0,
                      float* CA, int64_t ldc, void* stream);
int64_t gmr_xattn_bwd_workspace_floats(int64_t rows, int32_t D, int32_t nhead);
int gmr_xattn_bwd_f32(int64_t rows, int32_t D, int32_t nhead, const float* dCA, int64_t ld, const uint8_t* mask,
                      int64_t ldm, const float* wo, const float* bv, float p_keep, float* g_wo, float* g_bv, float* ws,
                      int64_t ws_floats, void* stream);
/* (Round 4's one-launch decoder stack, gmr_decoder_fwd_f32 / _masks_u8 / _split_f32, was removed in round 6:
 * opt-in, slower than the layer-by-layer path at the GenRecV1 batch in every round it was measured.) */
/* The same L decoder layers layer by layer, issued from C++ (csrc/decoder_host.hip, round 5): the kernels and
 * arguments of gmr/transformer.py's Python layer loop (gmr_gemm_f32 NT products with `tile`, gmr_dropout_f32,
 * gmr_layernorm_[drop_]fwd, gmr_xattn_fwd_f32 in train mode; the constant cross-attention row cav = b_v' Wo^T +
 * b_o, recomputed unless reuse_cav, in eval mode), bit-identical to it, without its per-launch Python cost.
 * offsets: 17 slab offsets of layer 0 (Wv = in_proj rows 2D..3D, bv, Wo, bo, norm1 w/b, b_v' = cross in_proj
 * bias + 2D, Wo', bo', norm2 w/b, W1, b1, W2, b2, norm3 w/b), layer l at + l * layer_stride.  bufs: 22 device
 * pointers of the activation workspace with Bmax rows per layer (h [L+1], V, SAin, SA, s1, h1, LN1 stats
 * [L][3][Bmax], CA, s2, h2, F1, F2, s3, LN2 / LN3 stats, cav [L][D], masks a / c [L][Bmax][nhead], masks
 * 1 / 2 / 3 / f [L][Bmax][D]; SAin, CA and the masks may be NULL in eval mode); h[0] is the input, h[L] the
 * output.  gemm_ws: >= gmr_gemm_workspace_floats of the B x D x D and 1 x D x D products (zeroed counters). */
int gmr_decoder_layers_fwd_f32(int64_t B, int64_t Bmax, int32_t L, int32_t D, int32_t nhead, const float* slab,
                               const int64_t* offsets, int64_t layer_stride, int32_t train_drop, float p_keep,
                               uint64_t seed, uint64_t step, int64_t row0, int32_t reuse_cav, const float* xP,
                               void* const* bufs, int32_t tile, float* gemm_ws, int64_t gemm_ws_floats, void* stream);
/* sinusoidal time embedding table T x E (:692-696); SiLU (dy == NULL) or its backward */
int gmr_time_embedding(int32_t T, int32_t E, float* out, void* stream);
int gmr_silu_f32(int64_t n, const float* x, const float* dy, float* y, void* stream);

/* ---------------------------------------------------------------- optimizer (torch.optim.Adam, trainer.py:125-142)
 * flat fp32 slabs; step_size = lr / (1 - b1^t), bias_correction2_sqrt = sqrt(1 - b2^t) */
int gmr_adam_f32(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, float beta1,
                 float beta2, float eps, float weight_decay, float step_size, float bias_correction2_sqrt,
                 void* stream);

/* (Round 5's native executor of a captured HIP graph, gmr_graph_exec_*, was removed in round 6: its replayed
 * step ran slower on the GPU than eager issue; the host tape of gmr/tape.py removes the Python issue cost and
 * keeps the eager streams and order.) */

#ifdef __cplusplus
}
#endif
#endif /* GMR_H_ */
