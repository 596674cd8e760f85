// Native issue of the GenRecV1 decoder layers (models/genrecv1.py:650-710, ModalDenoiseTransformer's
// nn.TransformerDecoder on a length-1 sequence): the layer-by-layer forward of gmr/transformer.py moved from
// Python to C++.  Host code only - it issues the same kernels with the same arguments as the Python loop
// (gmr_gemm_f32, gmr_dropout_f32, gmr_layernorm_[drop_]fwd, gmr_xattn_fwd_f32), so results are bit-identical.
//
// Why: GenRecV1's epoch issues ~7,000 launches and is host-issue-bound (profiles/r05s_genrecv1_host_profile.txt:
// ~7 us of Python + ctypes per launch on top of the ~5 us HIP launch).  The decoder layers are ~60 of the
// ~100 launches of each of the 55 denoiser forwards per epoch; issuing them from here removes their Python
// cost.  (The fused one-launch stack, csrc/decoder.hip, removes the launches too but runs slower on the GPU at
// the 2,048-row batch)
#include "gmr_common.h"

namespace {

// per-layer tensors of the slab, as float offsets of layer 0 (layer l adds l * layer_stride)
enum Off {
  O_WV,   // self_attn_in_proj_weight + 2 D^2 (the value rows)
  O_BV,   // self_attn_in_proj_bias + 2 D
  O_WO,   // self_attn_out_proj_weight
  O_BO,   // self_attn_out_proj_bias
  O_N1W,
  O_N1B,
  O_BVC,  // multihead_attn_in_proj_bias + 2 D
  O_WOC,  // multihead_attn_out_proj_weight
  O_BOC,  // multihead_attn_out_proj_bias
  O_N2W,
  O_N2B,
  O_L1W,
  O_L1B,
  O_L2W,
  O_L2B,
  O_N3W,
  O_N3B,
  O_COUNT
};

// activation / mask buffers of transformer.py's workspace (rows of Bmax per layer)
enum Buf {
  B_H,      // (L + 1, Bmax, D): h[0] in, h[l + 1] out of layer l
  B_V,      // (L, Bmax, D)
  B_SAIN,   // (L, Bmax, D)
  B_SA,     // (L, Bmax, D)
  B_S1,     // (L, Bmax, D)
  B_H1,     // (L, Bmax, D)
  B_M1,     // (L, 3, Bmax): mean, rstd
  B_CA,     // (L, Bmax, D)
  B_S2,
  B_H2,
  B_F1,
  B_F2,
  B_S3,
  B_M2,     // (L, 3, Bmax)
  B_M3,     // (L, 3, Bmax)
  B_CAV,    // (L, D)
  B_MASK_A, // u8 (L, Bmax, nhead)
  B_MASK_C, // u8 (L, Bmax, nhead)
  B_MASK_1, // u8 (L, Bmax, D)
  B_MASK_2,
  B_MASK_3,
  B_MASK_F,
  B_COUNT
};

inline uint64_t site_step(uint64_t step, int l, int site) {  // transformer.py _site_step, site in "ac123f"
  return ((step * 64 + (uint64_t)l) * 8 + (uint64_t)site) & 0xFFFFFFFFFFFFull;
}

}  // namespace

#define DH_CALL(x)              \
  do {                          \
    const int r__ = (x);        \
    if (r__ != GMR_OK) return r__; \
  } while (0)

extern "C" int gmr_decoder_layers_fwd_f32(int64_t B, int64_t Bmax, int32_t L, int32_t D, int32_t nhead,
                                          const float* slab, const int64_t* offsets, int64_t layer_stride,
                                          int32_t train_drop, float p_keep, uint64_t seed, uint64_t step, int64_t row0,
                                          int32_t reuse_cav, const float* xP, void* const* bufs, int32_t tile,
                                          float* gemm_ws, int64_t gemm_ws_floats, void* stream) {
  GMR_ARG(B > 0 && B <= Bmax && L > 0 && D > 0 && nhead > 0 && D % nhead == 0, "bad decoder shape");
  GMR_ARG(slab && offsets && bufs, "null slab / offsets / buffers");
  GMR_ARG(!train_drop || (xP && p_keep > 0.f && p_keep <= 1.f), "training mode needs the head tables and 0 < p_keep <= 1");
  for (int i = 0; i < B_COUNT; ++i) GMR_ARG(bufs[i] || (!train_drop && (i == B_SAIN || i == B_CA || i >= B_MASK_A)),
                                            "null activation buffer");
  auto F = [&](int b) { return static_cast<float*>(bufs[b]); };
  auto U8 = [&](int b) { return static_cast<uint8_t*>(bufs[b]); };
  const int64_t lay = Bmax * D;     // floats between two layers' (Bmax, D) activations
  const int64_t lay3 = 3 * Bmax;    // ... of the (3, Bmax) LayerNorm statistics
  const float inv_keep = 1.0f / p_keep;
  const int64_t dD = D;
  auto gemm = [&](const float* A, const float* W, float* C, int64_t M, int32_t epi, const float* bias) {
    return gmr_gemm_f32(0, 1, M, dD, dD, 1.0f, A, dD, W, dD, 0.0f, C, dD, epi, bias, nullptr, 0, nullptr, 0, nullptr,
                        nullptr, 0.0f, tile, 0, gemm_ws, gemm_ws_floats, stream);
  };
  for (int l = 0; l < L; ++l) {
    const float* P = slab + (int64_t)l * layer_stride;
    auto p = [&](int o) { return P + offsets[o]; };
    const float* h = F(B_H) + (int64_t)l * lay;
    float* V = F(B_V) + l * lay;
    float* SA = F(B_SA) + l * lay;
    float* h1 = F(B_H1) + l * lay;
    float* h2 = F(B_H2) + l * lay;
    float* hn = F(B_H) + (int64_t)(l + 1) * lay;
    float* m1 = F(B_M1) + l * lay3;
    float* m2 = F(B_M2) + l * lay3;
    float* m3 = F(B_M3) + l * lay3;
    // self-attention on the length-1 sequence: out_proj(dropout_head(V))
    DH_CALL(gemm(h, p(O_WV), V, B, GMR_EPI_BIAS, p(O_BV)));
    const float* SAin = V;
    if (train_drop) {
      float* sain = F(B_SAIN) + l * lay;
      DH_CALL(gmr_dropout_f32(B, D, D / nhead, V, dD, p_keep, nullptr, U8(B_MASK_A) + (int64_t)l * Bmax * nhead, nhead,
                              seed, site_step(step, l, 0), row0, sain, dD, stream));
      SAin = sain;
    }
    DH_CALL(gemm(SAin, p(O_WO), SA, B, GMR_EPI_BIAS, p(O_BO)));
    if (train_drop)
      DH_CALL(gmr_layernorm_drop_fwd(B, D, h, dD, SA, dD, p_keep, seed, site_step(step, l, 2), (uint64_t)row0 * D,
                                     U8(B_MASK_1) + l * lay, dD, inv_keep, p(O_N1W), p(O_N1B), 1e-5f, 0, h1, dD,
                                     F(B_S1) + l * lay, dD, m1, m1 + Bmax, stream));
    else
      DH_CALL(gmr_layernorm_fwd(B, D, h, dD, SA, dD, nullptr, 0, inv_keep, p(O_N1W), p(O_N1B), 1e-5f, 0, h1, dD,
                                F(B_S1) + l * lay, dD, m1, m1 + Bmax, stream));
    // cross-attention on the all-zero memory
    if (train_drop) {
      float* CA = F(B_CA) + l * lay;
      DH_CALL(gmr_xattn_fwd_f32(B, D, nhead, xP + (int64_t)l * nhead * D, p(O_BOC), p_keep, nullptr,
                                U8(B_MASK_C) + (int64_t)l * Bmax * nhead, nhead, seed, site_step(step, l, 1), row0, CA,
                                dD, stream));
      DH_CALL(gmr_layernorm_drop_fwd(B, D, h1, dD, CA, dD, p_keep, seed, site_step(step, l, 3), (uint64_t)row0 * D,
                                     U8(B_MASK_2) + l * lay, dD, inv_keep, p(O_N2W), p(O_N2B), 1e-5f, 0, h2, dD,
                                     F(B_S2) + l * lay, dD, m2, m2 + Bmax, stream));
    } else {
      float* cav = F(B_CAV) + (int64_t)l * D;
      if (!reuse_cav) DH_CALL(gemm(p(O_BVC), p(O_WOC), cav, 1, GMR_EPI_BIAS, p(O_BOC)));
      DH_CALL(gmr_layernorm_fwd(B, D, h1, dD, cav, 0, nullptr, 0, inv_keep, p(O_N2W), p(O_N2B), 1e-5f, 0, h2, dD,
                                F(B_S2) + l * lay, dD, m2, m2 + Bmax, stream));
    }
    // feed-forward
    float* F1 = F(B_F1) + l * lay;
    float* F2 = F(B_F2) + l * lay;
    DH_CALL(gemm(h2, p(O_L1W), F1, B, GMR_EPI_BIAS_RELU, p(O_L1B)));
    if (train_drop)
      DH_CALL(gmr_dropout_f32(B, D, 1, F1, dD, p_keep, nullptr, U8(B_MASK_F) + l * lay, dD, seed, site_step(step, l, 5),
                              row0, F1, dD, stream));
    DH_CALL(gemm(F1, p(O_L2W), F2, B, GMR_EPI_BIAS, p(O_L2B)));
    if (train_drop)
      DH_CALL(gmr_layernorm_drop_fwd(B, D, h2, dD, F2, dD, p_keep, seed, site_step(step, l, 4), (uint64_t)row0 * D,
                                     U8(B_MASK_3) + l * lay, dD, inv_keep, p(O_N3W), p(O_N3B), 1e-5f, 0, hn, dD,
                                     F(B_S3) + l * lay, dD, m3, m3 + Bmax, stream));
    else
      DH_CALL(gmr_layernorm_fwd(B, D, h2, dD, F2, dD, nullptr, 0, inv_keep, p(O_N3W), p(O_N3B), 1e-5f, 0, hn, dD,
                                F(B_S3) + l * lay, dD, m3, m3 + Bmax, stream));
  }
  return GMR_OK;
}
