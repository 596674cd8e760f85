"""MLP denoiser of the Gaussian diffusion over interaction vectors, on flat slabs + HIP GEMMs.

Reference: Denoise (models/diffmm.py:303-360) / DNN (models/diffrec.py:16-91), one hidden
layer (dims = [H]):  h = tanh([drop(x), emb(t)] @ W1^T + b1);  out = h @ W2^T + b2.
The time embedding takes only T values, so emb(t) @ W1[:, I:]^T + b1 is precomputed as a
T x H table (gmr_diff_time_bias) and added by the first GEMM's epilogue.
State-dict names follow the reference: emb_layer.{weight,bias}, in_layers.0.*, out_layers.0.*.
"""
import math
import os

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from . import dist
from . import kernels as K
from .kernels import ptr, stream
from .slab import Slab


def _r4(n):
    return (n + 3) // 4 * 4


# GMR_PSAMPLE_FOLD (default 1): p_sample chains (the DiffMM graph rebuild, DiffRec's prediction) carry the
# hidden pre-activation a = x_t W1[:, :I]^T instead of x_t (p_sample_fold): every step but the last is one
# B x H x H product instead of a B x H x I and a B x I x H one.  0 restores the step-by-step chain.
PSAMPLE_FOLD = os.environ.get("GMR_PSAMPLE_FOLD", "1") != "0"


class _Linear(nn.Module):
    def __init__(self, weight, bias):
        super().__init__()
        self.weight = weight
        self.bias = bias


class Denoiser(nn.Module):
    PARAM_NAMES = ("emb_W", "emb_b", "W1", "b1", "W2", "b2")

    def __init__(self, n_items, hidden, emb_size, device, dropout=0.5, norm=False):
        super().__init__()
        if norm:
            raise NotImplementedError("Denoise(norm=True) is not on the configured hot path")
        I, H, E = n_items, hidden, emb_size
        self.I, self.H, self.E = I, H, E
        self.ld_w1 = _r4(I + E)
        self.keep_prob = 1.0 - dropout
        self.slab = Slab([("emb_W", (E, E), None), ("emb_b", (E,), None), ("W1", (H, I + E), self.ld_w1),
                          ("b1", (H,), None), ("W2", (I, H), _r4(H)), ("b2", (I,), None)], device)
        self.emb_layer = _Linear(self.slab.parameter("emb_W"), self.slab.parameter("emb_b"))
        self.in_layers = nn.ModuleList([_Linear(self.slab.parameter("W1"), self.slab.parameter("b1"))])
        self.out_layers = nn.ModuleList([_Linear(self.slab.parameter("W2"), self.slab.parameter("b2"))])
        self.device = device
        self._tb = None

    def params(self):
        """nn.Parameters in PARAM_NAMES order (views of the slab)."""
        return [self.emb_layer.weight, self.emb_layer.bias, self.in_layers[0].weight, self.in_layers[0].bias,
                self.out_layers[0].weight, self.out_layers[0].bias]

    @torch.no_grad()
    def init_like_reference(self):
        """Consume the CPU RNG exactly as the reference constructor does (nn.Linear default init,
        then init_weights' normal_ draws, diffmm.py:311-338) and copy the result in."""
        I, H, E = self.I, self.H, self.E
        emb = nn.Linear(E, E)
        lin_in = nn.Linear(I + E, H)
        lin_out = nn.Linear(H, I)
        nn.Dropout(1.0 - self.keep_prob)
        for lay in (lin_in, lin_out, emb):
            size = lay.weight.size()
            lay.weight.data.normal_(0.0, float(np.sqrt(2.0 / (size[0] + size[1]))))
            lay.bias.data.normal_(0.0, 0.001)
        self.slab.load("emb_W", emb.weight)
        self.slab.load("emb_b", emb.bias)
        self.slab.load("W1", lin_in.weight)
        self.slab.load("b1", lin_in.bias)
        self.slab.load("W2", lin_out.weight)
        self.slab.load("b2", lin_out.bias)

    # ------------------------------------------------------------------ time table
    def time_bias(self, T):
        """EB[t] = emb_layer(temb(t)) @ W1[:, I:]^T + b1 for t < T (recomputed after each update)."""
        if self._tb is None or self._tb[0].shape[0] != T:
            self._tb = (torch.empty((T, self.H), device=self.device), torch.empty((T, self.E), device=self.device),
                        torch.empty((T, self.E), device=self.device))
        EB, temb, emb = self._tb
        s = self.slab
        _lib.call("gmr_diff_time_bias", T, self.E, ptr(s.view("emb_W")), ptr(s.view("emb_b")), ptr(s.view("W1")),
                  self.ld_w1, self.I, ptr(s.view("b1")), self.H, ptr(EB), ptr(temb), ptr(emb), stream())
        return self._tb

    def W1x(self):
        return self.slab.view("W1")[:, :self.I]

    def refresh_w1t(self):
        """W1T = W1[:, :I]^T (I x H), the gather-friendly copy used by hidden_sparse; call after
        the weights change (once per graph rebuild / prediction pass)."""
        if getattr(self, "_w1t", None) is None:
            self._w1t = torch.empty((self.I, _r4(self.H)), device=self.device)[:, :self.H]
        _lib.call("gmr_transpose_f32", self.H, self.I, ptr(self.slab.view("W1")), self.ld_w1, ptr(self._w1t),
                  self._w1t.stride(0), stream())
        if PSAMPLE_FOLD:
            self.refresh_fold()
        return self._w1t

    def refresh_fold(self):
        """P = W1[:, :I] @ W2 (H x H) and v = W1[:, :I] @ b2 (H) for p_sample_fold; recomputed with W1T."""
        H = self.H
        if getattr(self, "_fold", None) is None:
            self._fold = (torch.empty((H, _r4(H)), device=self.device)[:, :H],
                          torch.empty((1, _r4(H)), device=self.device)[:, :H])
        P, v = self._fold
        K.gemm(self.W1x(), self.slab.view("W2"), P)                                  # (H x I) (I x H)
        K.gemm(self.slab.view("b2")[None, :], self.W1x(), v, trans_b=True)          # b2 W1[:, :I]^T
        return self._fold

    def p_sample_fold(self, users, user_ptr, user_items, EB, c1, c2, x, a, h):
        """p_sample(x0, steps = 0, sampling_noise = False) of binary histories (models/diffmm.py:408-426,
        models/diffrec.py:291-310), exact algebra of the same chain carried in the hidden pre-activation.

        The step-by-step chain is h_i = tanh(x_{i+1} W1x^T + EB[i]), x_i = c1_i (h_i W2^T + b2) + c2_i x_{i+1}
        (x_T = x0, W1x = W1[:, :I]).  With a_j = x_j W1x^T that is a_i = c1_i (h_i P^T + v) + c2_i a_{i+1}
        (P = W1x W2, v = W1x b2: refresh_fold), so the chain needs x only at the end: for i = T-1 .. 1 one
        B x H x H product with the posterior epilogue (in place over a) and h_{i-1} = tanh(a_i + EB[i-1]);
        the last step (t = 0) is x_0 = c1_0 (h_0 W2^T + b2) + c2_0 x_1 with c2_0 = 0 exactly (the posterior
        at t = 0 is the x0 prediction: alphas_cumprod_prev[0] = 1), i.e. ONE B x I x H product over the
        densified x0 that x holds on entry (0 * x0 = 0).  c1 / c2: the fp32 coefficient per t (len = T).
        Work for the DiffMM rebuild (T = 5, H = 1,000, I = 7,050): 4 B H^2 + B I H instead of 9 B I H."""
        T = len(c1)
        if c2[0] != 0.0:
            raise ValueError("p_sample_fold needs c2[0] == 0 (the posterior mean at t = 0 is the x0 prediction)")
        P, v = self._fold
        B, H = users.numel(), self.H
        _lib.call("gmr_diff_sparse_pre", B, H, ptr(users), ptr(user_ptr), ptr(user_items), ptr(self._w1t),
                  self._w1t.stride(0), ptr(EB[T - 1]), ptr(a), a.stride(0), ptr(h), h.stride(0), stream())
        for i in range(T - 1, 0, -1):
            K.gemm(h, P, a, trans_b=True, epi=K.EPI_POSTERIOR, bias=v[0], aux=a, slope=c1[i], beta=c2[i])
            _lib.call("gmr_tanh_bias_f32", B, H, ptr(a), a.stride(0), ptr(EB[i - 1]), ptr(h), h.stride(0), stream())
        return self.posterior_step(h, x, c1[0], 0.0)

    def hidden_sparse(self, users, user_ptr, user_items, h, eb_row):
        """h = tanh(x0 @ W1[:, :I]^T + eb_row) for binary x0 rows given as the users' item lists
        (the first p_sample step, whose input is the interaction history itself)."""
        _lib.call("gmr_diff_sparse_hidden", users.numel(), self.H, ptr(users), ptr(user_ptr), ptr(user_items),
                  ptr(self._w1t), self._w1t.stride(0), ptr(eb_row), ptr(h), h.stride(0), stream())
        return h

    # ------------------------------------------------------------------ forward pieces
    def hidden(self, x, h, EB, t_rows=None, t_const=None):
        """h = tanh(x @ W1[:, :I]^T + EB[t])."""
        if t_rows is not None:
            K.gemm(x, self.W1x(), h, trans_b=True, epi=K.EPI_BIAS_TANH, bias=EB, bias_row=t_rows, ld_bias=self.H)
        else:
            K.gemm(x, self.W1x(), h, trans_b=True, epi=K.EPI_BIAS_TANH, bias=EB[t_const], ld_bias=0)
        return h

    def output(self, h, out):
        """out = h @ W2^T + b2."""
        K.gemm(h, self.slab.view("W2"), out, trans_b=True, epi=K.EPI_BIAS, bias=self.slab.view("b2"))
        return out

    def posterior_step(self, h, x, c1, c2):
        """x <- c1 * (h @ W2^T + b2) + c2 * x (in place; GaussianDiffusion.p_mean_variance mean).  c2 == 0 (the
        last step, t = 0): the same values without reading x (GMR_EPI_SCALE_BIAS), so x need not hold anything."""
        if c2 == 0.0:
            K.gemm(h, self.slab.view("W2"), x, trans_b=True, epi=K.EPI_SCALE_BIAS, bias=self.slab.view("b2"),
                   slope=c1)
        else:
            K.gemm(h, self.slab.view("W2"), x, trans_b=True, epi=K.EPI_POSTERIOR, bias=self.slab.view("b2"), aux=x,
                   slope=c1, beta=c2)
        return x

    def slab_head_words(self):
        """Gradient words before the [W2 | b2] tail (the part reduced after the whole backward)."""
        return self.slab.offsets["W2"]

    # ------------------------------------------------------------------ backward
    def backward(self, x_in, h, dout, dpre, t_rows, T, S, early_reduce=False):
        """Parameter gradients (written into the slab's grad buffer) from dout = dL/d out.
        early_reduce (data parallel): the [W2 | b2] tail of the gradient slab is final after its two
        products, so its all-reduce starts there (handle in self.early_handle) and runs beside the
        dpre / dW1 products; the caller reduces the head [: W2) (slab_head_words())."""
        s = self.slab
        I = self.I
        K.gemm(dout, h, s.gview("W2"), trans_a=True)                      # dW2 = dout^T h
        K.colsum(dout, s.gview("b2"))                                     # db2
        if early_reduce:
            self.early_handle = dist.all_reduce_start(s.grad[self.slab_head_words():])
        K.gemm(dout, s.view("W2"), dpre, epi=K.EPI_DTANH, aux=h)          # dpre = (dout W2) * (1 - h^2)
        K.gemm(dpre, x_in, s.gview("W1")[:, :I], trans_a=True)             # dW1[:, :I] = dpre^T x_in
        K.colsum(dpre, S, group=t_rows, n_groups=T)                       # S[t] = sum_{b: t_b = t} dpre[b]
        EB, temb, emb = self._tb
        _lib.call("gmr_diff_time_bwd", T, self.E, self.H, ptr(S), ptr(temb), ptr(emb), ptr(s.view("W1")), self.ld_w1,
                  I, ptr(s.gview("W1")), ptr(s.gview("b1")), ptr(s.gview("emb_W")), ptr(s.gview("emb_b")), 0,
                  stream())
