"""ModalDenoiseTransformer on MI355X — models/genrecv1.py:650-710 of the reference.

A post-norm nn.TransformerDecoder (ReLU feed-forward) applied to a length-1 target with an
all-zero memory.  On such a sequence the attention softmax is exactly 1, so
  self-attention  = out_proj(dropout_head(V)),  V = h W_v^T + b_v   (Q/K projections inert)
  cross-attention = out_proj(dropout_head(b_v'))                     (memory = 0 -> V = bias)
and the block is a chain of B x D GEMMs (MFMA, gemm.hip) and fused row kernels (LayerNorm with
residual + dropout [+ GELU], adaLN, dropout masks; gendiff.hip).  The time embedding takes only T
values, so time_emb / adaLN / the input projection's time columns are T-row tables recomputed
once per call.  Forward keeps every activation the hand-derived backward needs.

Parameters live in one Slab under the reference's parameter names ('.' -> '_'); Q/K rows of the
in_proj matrices and the unused `time_emb` MLP are kept (zero gradient) so state dicts line up.
"""
import copy
import ctypes
import math
import os

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from . import kernels as K
from .kernels import ptr, stream
from .slab import Slab


def _round4(n):
    return (n + 3) // 4 * 4


# (round 4's one-launch decoder stack, GMR_DEC_FUSED, lost to the layer-by-layer path at the 2,048-row batch -
# 1.49 ms per call vs ~0.7 ms, epoch 165 vs 121 ms, profiles/r04s_genrecv1_ab.txt - and was removed in round 6)
# the layer-by-layer decoder issued from C++ (gmr_decoder_layers_fwd_f32, csrc/decoder_host.hip): the same kernels
# and arguments as the Python loop below (bit-identical), without its ~7 us of Python per launch; GMR_DEC_NATIVE=0
# keeps the Python loop (A/B, and the path that takes injected masks)
DEC_NATIVE = os.environ.get("GMR_DEC_NATIVE", "1") != "0"
_DEC_OFFSETS = ("self_attn_in_proj_weight", "self_attn_in_proj_bias", "self_attn_out_proj_weight",
                "self_attn_out_proj_bias", "norm1_weight", "norm1_bias", "multihead_attn_in_proj_bias",
                "multihead_attn_out_proj_weight", "multihead_attn_out_proj_bias", "norm2_weight", "norm2_bias",
                "linear1_weight", "linear1_bias", "linear2_weight", "linear2_bias", "norm3_weight", "norm3_bias")
_DEC_BUFS = ("h", "V", "SAin", "SA", "s1", "h1", "m1", "CA", "s2", "h2", "F1", "F2", "s3", "m2", "m3", "cav",
             "mask_a", "mask_c", "mask_1", "mask_2", "mask_3", "mask_f")


class TransformerDenoiser:
    def __init__(self, in_dims, out_dims, emb_size, device, nhead=8, num_layers=6, dim_feedforward=512,
                 dropout=0.2):
        if in_dims != out_dims:
            raise NotImplementedError("GenRecV1 denoises interaction rows: in_dims == out_dims")
        I, E, D = in_dims, emb_size, dim_feedforward
        if D not in (64, 128, 256, 512, 1024) or D % nhead:
            raise NotImplementedError("dim_feedforward must be a power of two 64..1024 divisible by nhead")
        self.I, self.E, self.D, self.nhead, self.L, self.p = I, E, D, nhead, num_layers, float(dropout)
        self.device = device
        self.ld_in = _round4(I + E)
        specs = [("time_emb_0_weight", (4 * E, E), None), ("time_emb_0_bias", (4 * E,), None),
                 ("time_emb_2_weight", (E, 4 * E), None), ("time_emb_2_bias", (E,), None),
                 ("emb_layer_weight", (E, E), None), ("emb_layer_bias", (E,), None),
                 ("input_proj_weight", (D, I + E), self.ld_in), ("input_proj_bias", (D,), None)]
        for l in range(num_layers):
            p = f"transformer_decoder_layers_{l}_"
            specs += [(p + "self_attn_in_proj_weight", (3 * D, D), None), (p + "self_attn_in_proj_bias", (3 * D,), None),
                      (p + "self_attn_out_proj_weight", (D, D), None), (p + "self_attn_out_proj_bias", (D,), None),
                      (p + "multihead_attn_in_proj_weight", (3 * D, D), None),
                      (p + "multihead_attn_in_proj_bias", (3 * D,), None),
                      (p + "multihead_attn_out_proj_weight", (D, D), None),
                      (p + "multihead_attn_out_proj_bias", (D,), None),
                      (p + "linear1_weight", (D, D), None), (p + "linear1_bias", (D,), None),
                      (p + "linear2_weight", (D, D), None), (p + "linear2_bias", (D,), None)]
            for n in (1, 2, 3):
                specs += [(p + f"norm{n}_weight", (D,), None), (p + f"norm{n}_bias", (D,), None)]
        H2 = D // 2
        self.H2 = H2
        specs += [("output_proj_0_weight", (H2, D), None), ("output_proj_0_bias", (H2,), None),
                  ("output_proj_1_weight", (H2,), None), ("output_proj_1_bias", (H2,), None),
                  ("output_proj_3_weight", (I, H2), None), ("output_proj_3_bias", (I,), None),
                  ("adaLN_modulation_1_weight", (2 * D, E), None), ("adaLN_modulation_1_bias", (2 * D,), None)]
        self.names = [s[0] for s in specs]
        self.slab = Slab(specs, device)
        # floats between one decoder layer's tensors and the next's (the same spec list per layer)
        o = self.slab.offsets
        self.layer_stride = (o["transformer_decoder_layers_1_linear1_weight"] - o["transformer_decoder_layers_0_linear1_weight"]
                             if num_layers > 1 else 0)
        self._cache = None  # (T, train_drop, keep) of the time tables / cross-attention tables held
        # layer 0's slab offsets for gmr_decoder_layers_fwd_f32 (value rows / bias of in_proj: + 2 D)
        p0 = "transformer_decoder_layers_0_"
        self._lay_off = (ctypes.c_int64 * len(_DEC_OFFSETS))(*[
            o[p0 + n] + (2 * D * D if n == "self_attn_in_proj_weight" else 2 * D if n.endswith("in_proj_bias") else 0)
            for n in _DEC_OFFSETS])
        self._lay_bufs = None
        self.training = True
        self._ws = None
        self._temb = None
        self._seed = 0
        self._call = 0

    def twin(self):
        """A second denoiser over the same slab (weights and gradients shared) with private work buffers and
        table caches: a forward issued on another stream beside this one's work (GenRecV1's value-only
        p_sample beside the training backward, the rebuild chunks) touches none of this one's buffers."""
        t = copy.copy(self)
        t._ws, t._cache, t._lay_bufs, t._last = None, None, None, None
        return t

    # ------------------------------------------------------------------ parameters
    def v(self, name):
        return self.slab.view(name)

    def g(self, name):
        return self.slab.gview(name)

    def load_state(self, params):
        """params: {reference name with '.' -> '_': tensor}."""
        for n in self.names:
            if n in params:
                self.slab.load(n, torch.as_tensor(params[n], dtype=torch.float32))

    def init_like_reference(self, seed=None):
        """Initial weights with the reference's construction order (ModalDenoiseTransformer.__init__,
        :651-689): the torch modules are built on the CPU only to draw the same initial values."""
        twin = _reference_init_twin(self.I, self.E, self.nhead, self.L, self.D, self.p)
        self.load_state({k.replace(".", "_"): v.detach() for k, v in twin.named_parameters()})

    def train(self, mode=True):
        self.training = mode

    def eval(self):
        self.training = False

    def parameters(self):
        return [self.slab.data]

    # ------------------------------------------------------------------ buffers
    def _work(self, B):
        if self._ws is not None and self._ws["B"] >= B:
            return self._ws
        D, I, L, H2, T = self.D, self.I, self.L, self.H2, 16
        dev = self.device
        f = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)  # noqa: E731
        u8 = lambda *s: torch.empty(s, dtype=torch.uint8, device=dev)  # noqa: E731
        w = {"B": B, "h0": f(B, D), "h": f(L + 1, B, D), "V": f(L, B, D), "SAin": f(L, B, D),
             "SA": f(L, B, D), "s1": f(L, B, D), "h1": f(L, B, D), "m1": f(L, 3, B),
             "CA": f(L, B, D), "s2": f(L, B, D), "h2": f(L, B, D),
             "F1": f(L, B, D), "F2": f(L, B, D), "s3": f(L, B, D), "m2": f(L, 3, B), "m3": f(L, 3, B),
             "o1": f(B, H2), "og": f(B, H2), "mo": f(2, B),
             "mask_a": u8(L, B, self.nhead), "mask_c": u8(L, B, self.nhead), "mask_1": u8(L, B, D),
             "mask_2": u8(L, B, D), "mask_3": u8(L, B, D), "mask_f": u8(L, B, D),
             # backward scratch
             "dh": f(B, D), "dA": f(B, D), "dB": f(B, D), "dC": f(B, D), "dg": f(B, H2), "do1": f(B, H2),
             "prod": f(B, D), "ln_parts": f(int(_lib.load().gmr_layernorm_parts_floats(B, D))),
             "te": f(T, self.E), "ste": f(T, self.E), "TB": f(T, D), "S": f(T, 2 * D), "cav": f(L, D),
             "dS": f(2 * T, D), "dTB": f(T, D), "dte": f(T, self.E), "col": f(2 * D),
             "xP": f(L, self.nhead, D),
             "xws": f(int(_lib.load().gmr_xattn_bwd_workspace_floats(B, D, self.nhead)))}
        self._ws = w
        return w

    def _tables(self, T, reuse=False):
        """te = emb_layer(temb(t)), TB = te W_in[:, I:]^T + b_in, S = SiLU(te) W_ada^T + b_ada, t < T.
        reuse: the caller guarantees the weights are those of the previous forward (a p_sample step after
        its first), so tables of the same T are kept."""
        w = self._work(1)
        I, E, D = self.I, self.E, self.D
        if reuse and self._cache is not None and self._cache[0] == T:
            return w["te"][:T], w["ste"][:T], w["TB"][:T], w["S"][:T]
        if self._temb is None or self._temb.shape[0] != T:
            self._temb = torch.empty((T, E), dtype=torch.float32, device=self.device)
            _lib.call("gmr_time_embedding", T, E, ptr(self._temb), stream())
        te, ste, TB, S = w["te"][:T], w["ste"][:T], w["TB"][:T], w["S"][:T]
        K.gemm(self._temb, self.v("emb_layer_weight"), te, trans_b=True, epi=K.EPI_BIAS, bias=self.v("emb_layer_bias"))
        win = self.v("input_proj_weight")
        K.gemm(te, win[:, I:], TB, trans_b=True, epi=K.EPI_BIAS, bias=self.v("input_proj_bias"))
        _lib.call("gmr_silu_f32", T * E, ptr(te), None, ptr(ste), stream())
        K.gemm(ste, self.v("adaLN_modulation_1_weight"), S, trans_b=True, epi=K.EPI_BIAS,
               bias=self.v("adaLN_modulation_1_bias"))
        return te, ste, TB, S

    # ------------------------------------------------------------------ forward
    def forward(self, x, t_rows=None, t_const=None, T=5, out=None, masks=None, seed=None, step=0, row0=0,
                reuse_tables=False, keep_acts=True):
        """logits = model(x, t) for x (B x I, fp32, ld % 4 == 0) and per-row t (int32 device tensor) or
        a constant t.  Train mode draws the dropout masks (Philox seed/step, keyed by the global row
        row0 + r, so a data-parallel rank draws what one process holding the whole batch draws) unless
        `masks` gives them ({'a','c','1','2','3','f'} -> uint8 (L, B, ...)); returns out (B x I).
        reuse_tables: the weights are the previous forward's (p_sample steps after the first): the time
        tables and the cross-attention tables of the same T and mode are kept.  keep_acts is accepted for the
        callers of the removed fused stack (every layer's activations are kept)."""
        B = x.shape[0]
        w = self._work(B)
        D, I, L, H2 = self.D, self.I, self.L, self.H2
        train_drop = self.training and self.p > 0.0
        keep = 1.0 - self.p
        mode = (T, train_drop, keep)
        reuse = reuse_tables and self._cache == mode
        te, ste, TB, S = self._tables(T, reuse)
        self._T = T
        if train_drop and not reuse:  # cross-attention head tables of the L layers (gmr_xattn_table_f32)
            p0 = "transformer_decoder_layers_0_"
            _lib.call("gmr_xattn_table_f32", L, D, self.nhead, ptr(self.v(p0 + "multihead_attn_out_proj_weight")),
                      ptr(self.v(p0 + "multihead_attn_in_proj_bias")[2 * D:]), self.layer_stride,
                      keep if train_drop else 1.0, ptr(w["xP"]), stream())
        seed = self._seed if seed is None else seed
        win = self.v("input_proj_weight")
        h0 = w["h0"][:B]
        if t_rows is not None:
            K.gemm(x, win[:, :I], h0, trans_b=True, epi=K.EPI_BIAS, bias=TB, bias_row=t_rows, ld_bias=D)
        else:
            K.gemm(x, win[:, :I], h0, trans_b=True, epi=K.EPI_BIAS, bias=TB[t_const])
        h = w["h"][0, :B]
        _lib.call("gmr_adaln_fwd", B, D, ptr(h0), D, ptr(t_rows), -1 if t_rows is not None else int(t_const), ptr(S),
                  2 * D, ptr(h), D, stream())
        native = DEC_NATIVE and masks is None
        if native:
            h = self._decoder_native(w, B, train_drop, keep, seed, step, row0, reuse)
        for l in range(L if not native else 0):
            p = f"transformer_decoder_layers_{l}_"
            wv = self.v(p + "self_attn_in_proj_weight")[2 * D:]
            bv = self.v(p + "self_attn_in_proj_bias")[2 * D:]
            V, SAin, SA = w["V"][l, :B], w["SAin"][l, :B], w["SA"][l, :B]
            K.gemm(h, wv, V, trans_b=True, epi=K.EPI_BIAS, bias=bv)
            if train_drop:
                self._drop(V, SAin, "a", l, masks, keep, seed, step, row0, group=D // self.nhead)
            else:
                SAin = V
            K.gemm(SAin, self.v(p + "self_attn_out_proj_weight"), SA, trans_b=True, epi=K.EPI_BIAS,
                   bias=self.v(p + "self_attn_out_proj_bias"))
            h1 = w["h1"][l, :B]
            m1 = w["m1"][l]
            self._ln(h, SA, D, w["mask_1"][l, :B] if train_drop else None, "1", l, masks, keep, seed, step, row0,
                     self.v(p + "norm1_weight"), self.v(p + "norm1_bias"), h1, w["s1"][l, :B], m1[0, :B], m1[1, :B])
            # cross-attention on the zero memory: out_proj(dropout_head(b_v)) (+ b_o)
            bvc = self.v(p + "multihead_attn_in_proj_bias")[2 * D:]
            woc = self.v(p + "multihead_attn_out_proj_weight")
            boc = self.v(p + "multihead_attn_out_proj_bias")
            h2 = w["h2"][l, :B]
            m2 = w["m2"][l]
            if train_drop:
                # out_proj(dropout_head(b_v)) + b_o as a per-row mixture of the layer's head vectors
                CA = w["CA"][l, :B]
                mbuf = w["mask_c"][l, :B]
                given = masks.get("c") if masks else None
                if given is not None:
                    mbuf.copy_(given[l])
                _lib.call("gmr_xattn_fwd_f32", B, D, self.nhead, ptr(w["xP"][l]), ptr(boc), keep,
                          ptr(mbuf) if given is not None else None, ptr(mbuf) if given is None else None,
                          mbuf.stride(0), seed, self._site_step(step, l, "c"), int(row0), ptr(CA), K._ld(CA), stream())
                self._ln(h1, CA, D, w["mask_2"][l, :B], "2", l, masks, keep, seed, step, row0, self.v(p + "norm2_weight"),
                         self.v(p + "norm2_bias"), h2, w["s2"][l, :B], m2[0, :B], m2[1, :B])
            else:
                cav = w["cav"][l:l + 1]
                if not reuse:
                    K.gemm(bvc.view(1, D), woc, cav, trans_b=True, epi=K.EPI_BIAS, bias=boc)
                self._ln(h1, cav, 0, None, "2", l, masks, keep, seed, step, row0, self.v(p + "norm2_weight"),
                         self.v(p + "norm2_bias"), h2, w["s2"][l, :B], m2[0, :B], m2[1, :B])
            F1, F2 = w["F1"][l, :B], w["F2"][l, :B]
            K.gemm(h2, self.v(p + "linear1_weight"), F1, trans_b=True, epi=K.EPI_BIAS_RELU,
                   bias=self.v(p + "linear1_bias"))
            if train_drop:
                self._drop(F1, F1, "f", l, masks, keep, seed, step, row0, group=1)
            K.gemm(F1, self.v(p + "linear2_weight"), F2, trans_b=True, epi=K.EPI_BIAS,
                   bias=self.v(p + "linear2_bias"))
            m3 = w["m3"][l]
            hn = w["h"][l + 1, :B]
            self._ln(h2, F2, D, w["mask_3"][l, :B] if train_drop else None, "3", l, masks, keep, seed, step, row0,
                     self.v(p + "norm3_weight"), self.v(p + "norm3_bias"), hn, w["s3"][l, :B], m3[0, :B], m3[1, :B])
            h = hn
        o1, og = w["o1"][:B], w["og"][:B]
        K.gemm(h, self.v("output_proj_0_weight"), o1, trans_b=True, epi=K.EPI_BIAS, bias=self.v("output_proj_0_bias"))
        _lib.call("gmr_layernorm_fwd", B, H2, ptr(o1), H2, None, 0, None, 0, 1.0, ptr(self.v("output_proj_1_weight")),
                  ptr(self.v("output_proj_1_bias")), 1e-5, 1, ptr(og), H2, None, 0, ptr(w["mo"][0, :B]),
                  ptr(w["mo"][1, :B]), stream())
        if out is None:
            out = torch.empty((B, _round4(I)), dtype=torch.float32, device=self.device)[:, :I]
        K.gemm(og, self.v("output_proj_3_weight"), out, trans_b=True, epi=K.EPI_BIAS,
               bias=self.v("output_proj_3_bias"))
        self._last = (B, x, t_rows, t_const, train_drop, keep)
        self._cache = mode
        return out

    def _decoder_native(self, w, B, train_drop, keep, seed, step, row0, reuse):
        """The L decoder layers issued from C++ (gmr_decoder_layers_fwd_f32): the Python loop of forward()
        with the same kernels and arguments.  Returns the last layer's rows w['h'][L, :B]."""
        D, L = self.D, self.L
        if self._lay_bufs is None or self._lay_bufs[0] is not w:
            self._lay_bufs = (w, (ctypes.c_void_p * len(_DEC_BUFS))(*[w[k].data_ptr() for k in _DEC_BUFS]))
        tile = K.GEMM_TILE_FLAGS
        lib = _lib.load()
        need = max(lib.gmr_gemm_workspace_floats(0, 1, B, D, D, tile, 0), lib.gmr_gemm_workspace_floats(0, 1, 1, D, D,
                                                                                                        tile, 0))
        ws = K.workspace(need, self.device) if need > 0 else None
        _lib.call("gmr_decoder_layers_fwd_f32", B, w["B"], L, D, self.nhead, ptr(self.slab.data),
                  ctypes.cast(self._lay_off, ctypes.c_void_p), self.layer_stride, int(train_drop), keep, seed, step,
                  int(row0), int(bool(reuse)), ptr(w["xP"]), ctypes.cast(self._lay_bufs[1], ctypes.c_void_p), tile,
                  ptr(ws), ws.numel() if ws is not None else 0, stream())
        return w["h"][L, :B]

    def _drop(self, x, y, site, l, masks, keep, seed, step, row0, group, ldx=None):
        w = self._ws
        B = y.shape[0]
        D = self.D
        mbuf = w["mask_" + site][l, :B]
        given = masks.get(site) if masks else None
        mask_in = given[l] if given is not None else None
        if mask_in is not None:
            mbuf.copy_(mask_in)
        _lib.call("gmr_dropout_f32", B, D, group, ptr(x), K._ld(x) if ldx is None else ldx, keep,
                  ptr(mbuf) if mask_in is not None else None, ptr(mbuf) if mask_in is None else None,
                  mbuf.stride(0), seed, self._site_step(step, l, site), int(row0), ptr(y), K._ld(y), stream())

    def _site_step(self, step, l, site):
        return ((step * 64 + l) * 8 + "ac123f".index(site)) & 0xFFFFFFFFFFFF

    def _ln(self, a, b, ldb, mbuf, site, l, masks, keep, seed, step, row0, wt, bs, y, s, mean, rstd):
        B = a.shape[0]
        D = self.D
        if mbuf is not None:
            given = masks.get(site) if masks else None
            if given is not None:
                mbuf.copy_(given[l])
            else:  # the residual-branch dropout mask drawn by the LN kernel itself (gmr_keep_mask_u8's keys)
                assert mbuf.stride(0) == D and ldb > 0
                _lib.call("gmr_layernorm_drop_fwd", B, D, ptr(a), K._ld(a), ptr(b), ldb, keep, seed,
                          self._site_step(step, l, site), int(row0) * D, ptr(mbuf), D, 1.0 / keep, ptr(wt), ptr(bs),
                          1e-5, 0, ptr(y), K._ld(y), ptr(s), D, ptr(mean), ptr(rstd), stream())
                return
        _lib.call("gmr_layernorm_fwd", B, D, ptr(a), K._ld(a), ptr(b), ldb, ptr(mbuf), mbuf.stride(0) if mbuf is not None
                  else 0, 1.0 / keep, ptr(wt), ptr(bs), 1e-5, 0, ptr(y), K._ld(y), ptr(s), D, ptr(mean), ptr(rstd),
                  stream())

    # ------------------------------------------------------------------ backward
    def backward(self, dout, accumulate=False):
        """Gradients of every parameter from dL/dlogits (B x I) of the last forward (into slab.grad,
        added to what is there when accumulate)."""
        B, x, t_rows, t_const, train_drop, keep = self._last
        if t_rows is None:
            raise NotImplementedError("training steps use per-row t")
        w = self._ws
        D, I, L, H2, T = self.D, self.I, self.L, self.H2, self._T
        if not accumulate:
            self.slab.zero_grad()
        inv_keep = 1.0 / keep if train_drop else 1.0
        lnp = w["ln_parts"]
        og, o1 = w["og"][:B], w["o1"][:B]
        # output head
        K.gemm(dout, og, self.g("output_proj_3_weight"), trans_a=True, beta=1.0)
        K.colsum(dout, self.g("output_proj_3_bias"), accumulate=True)
        dg = w["dg"][:B]
        K.gemm(dout, self.v("output_proj_3_weight"), dg)
        do1 = w["do1"][:B]
        _lib.call("gmr_layernorm_bwd", B, H2, ptr(o1), H2, ptr(w["mo"][0, :B]), ptr(w["mo"][1, :B]),
                  ptr(self.v("output_proj_1_weight")), ptr(self.v("output_proj_1_bias")), 1, ptr(dg), H2, ptr(do1), H2,
                  0, ptr(lnp), ptr(self.g("output_proj_1_weight")), ptr(self.g("output_proj_1_bias")), 1, stream())
        hL = w["h"][L, :B]
        K.gemm(do1, hL, self.g("output_proj_0_weight"), trans_a=True, beta=1.0)
        K.colsum(do1, self.g("output_proj_0_bias"), accumulate=True)
        dh = w["dh"][:B]
        K.gemm(do1, self.v("output_proj_0_weight"), dh)
        dA, dB, dC = w["dA"][:B], w["dB"][:B], w["dC"][:B]
        for l in reversed(range(L)):
            p = f"transformer_decoder_layers_{l}_"
            m1, m2, m3 = w["m1"][l], w["m2"][l], w["m3"][l]
            # norm3: s3 = h2 + drop(F2)
            self._ln_bwd(w["s3"][l, :B], m3, p + "norm3", dh, dA)              # dA = d s3
            dF2 = self._mask_grad(dA, w["mask_3"][l, :B] if train_drop else None, keep, dB)
            F1, h2 = w["F1"][l, :B], w["h2"][l, :B]
            K.gemm(dF2, F1, self.g(p + "linear2_weight"), trans_a=True, beta=1.0)
            K.colsum(dF2, self.g(p + "linear2_bias"), accumulate=True)
            K.gemm(dF2, self.v(p + "linear2_weight"), dC, epi=K.EPI_DRELU, aux=F1, alpha=inv_keep)  # dF1 (pre-ReLU)
            K.gemm(dC, h2, self.g(p + "linear1_weight"), trans_a=True, beta=1.0)
            K.colsum(dC, self.g(p + "linear1_bias"), accumulate=True)
            K.gemm(dC, self.v(p + "linear1_weight"), dA, beta=1.0)            # d h2 = d s3 + dF1 W1
            # norm2: s2 = h1 + drop(CA)
            self._ln_bwd(w["s2"][l, :B], m2, p + "norm2", dA, dh)              # dh = d s2
            woc = self.v(p + "multihead_attn_out_proj_weight")
            bvc = self.v(p + "multihead_attn_in_proj_bias")[2 * D:]
            gbvc = self.g(p + "multihead_attn_in_proj_bias")[2 * D:]
            if train_drop:
                dCA = self._mask_grad(dh, w["mask_2"][l, :B], keep, dB)
                mc = w["mask_c"][l, :B]
                xws = w["xws"]
                _lib.call("gmr_xattn_bwd_f32", B, D, self.nhead, ptr(dCA), K._ld(dCA), ptr(mc), mc.stride(0), ptr(woc),
                          ptr(bvc), keep, ptr(self.g(p + "multihead_attn_out_proj_weight")), ptr(gbvc), ptr(xws),
                          xws.numel(), stream())
                K.colsum(dCA, self.g(p + "multihead_attn_out_proj_bias"), accumulate=True)
            else:
                col = w["col"][:D].view(1, D)
                K.colsum(dh, col)
                K.gemm(col, bvc.view(1, D), self.g(p + "multihead_attn_out_proj_weight"), trans_a=True, beta=1.0)
                K.gemm(col, woc, gbvc.view(1, D), beta=1.0)
                K.colsum(dh, self.g(p + "multihead_attn_out_proj_bias"), accumulate=True)
            # norm1: s1 = h + drop(SA)
            self._ln_bwd(w["s1"][l, :B], m1, p + "norm1", dh, dA)              # dA = d s1 (-> d h_l)
            dSA = self._mask_grad(dA, w["mask_1"][l, :B] if train_drop else None, keep, dB)
            SAin = w["SAin"][l, :B] if train_drop else w["V"][l, :B]
            K.gemm(dSA, SAin, self.g(p + "self_attn_out_proj_weight"), trans_a=True, beta=1.0)
            K.colsum(dSA, self.g(p + "self_attn_out_proj_bias"), accumulate=True)
            K.gemm(dSA, self.v(p + "self_attn_out_proj_weight"), dC)            # d SAin
            dV = self._mask_grad(dC, w["mask_a"][l, :B] if train_drop else None, keep, dC, group=D // self.nhead)
            hl = w["h"][l, :B]
            K.gemm(dV, hl, self.g(p + "self_attn_in_proj_weight")[2 * D:], trans_a=True, beta=1.0)
            K.colsum(dV, self.g(p + "self_attn_in_proj_bias")[2 * D:], accumulate=True)
            K.gemm(dV, self.v(p + "self_attn_in_proj_weight")[2 * D:], dA, beta=1.0)
            dh, dA = dA, dh
        # adaLN + input projection + time tables
        h0 = w["h0"][:B]
        prod = w["prod"][:B]
        dh0 = dB
        S = w["S"][:T]
        _lib.call("gmr_adaln_bwd", B, D, ptr(h0), D, ptr(dh), D, ptr(t_rows), ptr(S), 2 * D, ptr(dh0), D, ptr(prod), D,
                  stream())
        dshift, dscale = w["dS"][:T, :D], w["dS"][T:2 * T, :D]
        _lib.call("gmr_colsum_f32", B, D, ptr(dh), D, ptr(t_rows), T, ptr(dshift), 0, stream())
        _lib.call("gmr_colsum_f32", B, D, ptr(prod), D, ptr(t_rows), T, ptr(dscale), 0, stream())
        gwin = self.g("input_proj_weight")
        K.gemm(dh0, x, gwin[:, :I], trans_a=True, beta=1.0)
        dTB = w["dTB"][:T]
        _lib.call("gmr_colsum_f32", B, D, ptr(dh0), D, ptr(t_rows), T, ptr(dTB), 0, stream())
        K.colsum(dTB, self.g("input_proj_bias"), accumulate=True)
        te, ste = w["te"][:T], w["ste"][:T]
        K.gemm(dTB, te, gwin[:, I:], trans_a=True, beta=1.0)
        # adaLN Linear(SiLU(te)): [shift | scale] halves of its weight / bias
        wa, gwa, gba = self.v("adaLN_modulation_1_weight"), self.g("adaLN_modulation_1_weight"), \
            self.g("adaLN_modulation_1_bias")
        K.gemm(dshift, ste, gwa[:D], trans_a=True, beta=1.0)
        K.gemm(dscale, ste, gwa[D:], trans_a=True, beta=1.0)
        K.colsum(dshift, gba[:D], accumulate=True)
        K.colsum(dscale, gba[D:], accumulate=True)
        dte = w["dte"][:T]
        K.gemm(dshift, wa[:D], dte)
        K.gemm(dscale, wa[D:], dte, beta=1.0)
        _lib.call("gmr_silu_f32", T * self.E, ptr(te), ptr(dte), ptr(dte), stream())   # through SiLU
        K.gemm(dTB, self.v("input_proj_weight")[:, I:], dte, beta=1.0)              # + input_proj time columns
        K.gemm(dte, self._temb, self.g("emb_layer_weight"), trans_a=True, beta=1.0)
        K.colsum(dte, self.g("emb_layer_bias"), accumulate=True)

    def _ln_bwd(self, s, m, name, dy, dx):
        B = dy.shape[0]
        D = self.D
        _lib.call("gmr_layernorm_bwd", B, D, ptr(s), D, ptr(m[0, :B]), ptr(m[1, :B]), ptr(self.v(name + "_weight")),
                  ptr(self.v(name + "_bias")), 0, ptr(dy), K._ld(dy), ptr(dx), K._ld(dx), 0, ptr(self._ws["ln_parts"]),
                  ptr(self.g(name + "_weight")), ptr(self.g(name + "_bias")), 1, stream())

    def _mask_grad(self, g, mask, keep, out, group=1):
        if mask is None:
            return g
        B = g.shape[0]
        _lib.call("gmr_dropout_f32", B, self.D, group, ptr(g), K._ld(g), keep, ptr(mask), None, mask.stride(0), 0, 0, 0,
                  ptr(out), K._ld(out), stream())
        return out


def _reference_init_twin(I, E, nhead, L, D, p):
    """CPU module with ModalDenoiseTransformer's construction order (models/genrecv1.py:651-689),
    used only to draw identical initial parameters under the caller's torch seed."""
    class Twin(nn.Module):
        def __init__(self):
            super().__init__()
            self.time_emb = nn.Sequential(nn.Linear(E, 4 * E), nn.SiLU(), nn.Linear(4 * E, E))
            self.emb_layer = nn.Linear(E, E)
            self.input_proj = nn.Linear(I + E, D)
            layer = nn.TransformerDecoderLayer(d_model=D, nhead=nhead, dim_feedforward=D, dropout=p, batch_first=True)
            self.transformer_decoder = nn.TransformerDecoder(layer, num_layers=L)
            self.output_proj = nn.Sequential(nn.Linear(D, D // 2), nn.LayerNorm(D // 2), nn.GELU(),
                                             nn.Linear(D // 2, I))
            self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(E, 2 * D))

            def init(m):
                if isinstance(m, nn.Linear):
                    nn.init.xavier_uniform_(m.weight)
                    if m.bias is not None:
                        nn.init.constant_(m.bias, 0.01)
            self.apply(init)
    return Twin()
