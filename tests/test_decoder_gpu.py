"""GenRecV1's ModalDenoiseTransformer decoder (models/genrecv1.py:650-710: nn.TransformerDecoder on a length-1
target and a zero memory) through the C-ABI: the residual-branch dropout drawn inside the LayerNorm kernel
against mask + LayerNorm, and the layer loop issued from C++ (gmr_decoder_layers_fwd_f32) against the Python
loop, bit for bit.  (Round 4's one-launch fused stack and its tests were removed in round 6: it lost every A/B.)"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _den(I, dropout, L):
    from gmr.transformer import TransformerDenoiser
    torch.manual_seed(5)
    den = TransformerDenoiser(I, I, 10, DEV, nhead=8, num_layers=L, dim_feedforward=512, dropout=dropout)
    den.init_like_reference()
    return den


def _x(B, I, seed):
    rng = np.random.default_rng(seed)
    x = torch.zeros((B, (I + 3) // 4 * 4), dtype=torch.float32, device=DEV)[:, :I]
    x.copy_(torch.as_tensor((rng.random((B, I)) < 0.05).astype(np.float32)))
    return x


@pytest.mark.parametrize("B,row0,keep,skew", [(300, 0, 0.8, 0), (37, 1000, 0.5, 0), (2048, 5, 0.9, 0),
                                               (300, 3, 0.8, 77), (37, 0, 0.5, 255)])
def test_layernorm_drop_fwd_equals_mask_then_layernorm(B, row0, keep, skew):
    """gmr_layernorm_drop_fwd (the residual-branch dropout drawn inside the LayerNorm kernel) against
    gmr_keep_mask_u8 + gmr_layernorm_fwd with the same Philox key: keep bytes, y, s, mean and rstd bit for bit.
    skew != 0 starts the draw counter off a 256-unit block (the per-column path of the kernel's draws)."""
    from gmr import _lib
    from gmr.kernels import ptr, stream
    D = 512
    rng = np.random.default_rng(B)
    a = torch.as_tensor(rng.standard_normal((B, D)).astype(np.float32), device=DEV)
    b = torch.as_tensor(rng.standard_normal((B, D)).astype(np.float32), device=DEV)
    w = torch.as_tensor(rng.standard_normal(D).astype(np.float32), device=DEV)
    bs = torch.as_tensor(rng.standard_normal(D).astype(np.float32), device=DEV)
    res = []
    for fused in (False, True):
        m = torch.full((B, D), 7, dtype=torch.uint8, device=DEV)
        y, s = torch.empty((B, D), device=DEV), torch.empty((B, D), device=DEV)
        mean, rstd = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
        if fused:
            _lib.call("gmr_layernorm_drop_fwd", B, D, ptr(a), D, ptr(b), D, keep, 11, 1234, row0 * D + skew, ptr(m), D,
                      1.0 / keep, ptr(w), ptr(bs), 1e-5, 0, ptr(y), D, ptr(s), D, ptr(mean), ptr(rstd), stream())
        else:
            _lib.call("gmr_keep_mask_u8", B * D, keep, 11, 1234, row0 * D + skew, ptr(m), stream())
            _lib.call("gmr_layernorm_fwd", B, D, ptr(a), D, ptr(b), D, ptr(m), D, 1.0 / keep, ptr(w), ptr(bs), 1e-5, 0,
                      ptr(y), D, ptr(s), D, ptr(mean), ptr(rstd), stream())
        res.append([t.cpu() for t in (m, y, s, mean, rstd)])
    assert 0.3 < res[0][0].float().mean().item() / keep < 1.7
    for x0, x1 in zip(*res):
        assert torch.equal(x0, x1)


@pytest.mark.parametrize("train,B,L,row0", [(True, 300, 6, 0), (False, 300, 6, 0), (True, 37, 2, 1000),
                                            (True, 2048, 6, 5), (False, 2048, 6, 0)])
def test_native_layer_issue_bit_identical(train, B, L, row0, monkeypatch):
    """The decoder layers issued from C++ (gmr_decoder_layers_fwd_f32, csrc/decoder_host.hip) against the
    Python layer loop of transformer.forward: the same kernels with the same arguments, so the logits, every
    stored activation and mask, the parameter gradients of the backward that reads them, and an eval-mode
    forward reusing its tables (the p_sample steps) are equal bit for bit."""
    from gmr import transformer as tr
    I = 501
    x = _x(B, I, B + L + 1)
    t_rows = torch.as_tensor(np.random.default_rng(B).integers(0, 5, B).astype(np.int32)).to(DEV)
    runs = []
    for native in (False, True):
        monkeypatch.setattr(tr, "DEC_NATIVE", native)
        den = _den(I, 0.2, L)
        den.train(train)
        out = den.forward(x, t_rows=t_rows, T=5, seed=7, step=11, row0=row0)
        r = {"out": out.cpu().numpy().copy()}
        w = den._ws
        for k in ("h", "V", "SA", "s1", "h1", "m1", "s2", "h2", "F1", "F2", "s3", "m2", "m3"):
            # LayerNorm statistics (L, 3, Bmax): rows 0 / 1 = mean / rstd (row 2 is not written by the forward)
            r[k] = w[k][:, :2, :B].cpu().numpy().copy() if k[0] == "m" else w[k][:, :B].cpu().numpy().copy()
        if train:
            for k in ("SAin", "CA"):
                r[k] = w[k][:, :B].cpu().numpy().copy()
            for k in ("a", "c", "1", "2", "3", "f"):
                r["mask_" + k] = w["mask_" + k][:, :B].cpu().numpy().copy()
        den.slab.grad.zero_()
        dz = torch.ones_like(out) * 1e-3
        den.backward(dz)
        r["grad"] = den.slab.grad.cpu().numpy().copy()
        if not train:
            again = den.forward(x, t_rows=t_rows, T=5, seed=7, step=11, row0=row0, reuse_tables=True)
            r["reuse"] = again.cpu().numpy().copy()
        torch.cuda.synchronize()
        runs.append(r)
    for k in runs[0]:
        np.testing.assert_array_equal(runs[1][k].view(np.uint8), runs[0][k].view(np.uint8), err_msg=k)


@pytest.mark.parametrize("a", [1, 2, 3, 5, 150])
def test_draw_kernels_row_split_invariant(a):
    """Round 6: the per-element Bernoulli kernels take four draws per Philox call (two for flip_qsample), keyed
    by the GLOBAL unit index; a row split at any row (row0 = a, so the quads / pairs start unaligned) draws what
    the whole call drew: dropout masks and outputs (group 1 and the head group), flip_step samples, flip_qsample
    flips, bit for bit; the keep rates stay Bernoulli(p) (binomial bound)."""
    from gmr import _lib
    from gmr.kernels import ptr, stream
    torch.manual_seed(3)
    R, D, I, T = 301, 136, 1003, 10
    x = torch.randn(R, D, device="cuda")
    for group in (1, 17):
        y = torch.empty_like(x)
        m = torch.empty((R, D // group), dtype=torch.uint8, device="cuda")
        _lib.call("gmr_dropout_f32", R, D, group, ptr(x), D, 0.7, None, ptr(m), m.stride(0), 99, 5, 0, ptr(y), D,
                  stream())
        y2 = torch.empty_like(x)
        m2 = torch.empty_like(m)
        for lo, hi in ((0, a), (a, R)):
            _lib.call("gmr_dropout_f32", hi - lo, D, group, ptr(x[lo:]), D, 0.7, None, ptr(m2[lo:]), m2.stride(0), 99,
                      5, lo, ptr(y2[lo:]), D, stream())
        assert torch.equal(m, m2) and torch.equal(y, y2), group
        kr = m.float().mean().item()
        n = m.numel()
        assert abs(kr - 0.7) < 5 * (0.21 / n) ** 0.5, (group, kr)
    tab = torch.linspace(0.05, 0.6, 2 * T + 2, device="cuda")
    z = torch.randn(R, I, device="cuda")
    xs, xs2 = torch.empty_like(z), torch.empty_like(z)
    _lib.call("gmr_flip_step", R, I, ptr(z), I, ptr(tab), T, 3, 0, None, 0, 7, 2, 0, ptr(xs), I, None, 0, stream())
    for lo, hi in ((0, a), (a, R)):
        _lib.call("gmr_flip_step", hi - lo, I, ptr(z[lo:]), I, ptr(tab), T, 3, 0, None, 0, 7, 2, lo, ptr(xs2[lo:]), I,
                  None, 0, stream())
    assert torch.equal(xs, xs2)
    x0 = (torch.rand(R, I, device="cuda") < 0.1).float()
    t = torch.randint(0, T, (R,), dtype=torch.int32, device="cuda")
    xt, xt2 = torch.empty_like(x0), torch.empty_like(x0)
    _lib.call("gmr_flip_qsample", R, I, ptr(x0), I, ptr(t), 0, ptr(tab), T, 4.0, None, 0, 7, 3, 0, ptr(xt), I,
              stream())
    for lo, hi in ((0, a), (a, R)):
        _lib.call("gmr_flip_qsample", hi - lo, I, ptr(x0[lo:]), I, ptr(t[lo:]), 0, ptr(tab), T, 4.0, None, 0, 7, 3, lo,
                  ptr(xt2[lo:]), I, stream())
    assert torch.equal(xt, xt2)
    assert 0 < (xt != x0).float().mean().item() < 1
