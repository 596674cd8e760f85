"""The folded p_sample chain (Denoiser.p_sample_fold, GMR_PSAMPLE_FOLD=1, the product default for the DiffMM
graph rebuild and DiffRec's prediction) against the step-by-step chain of the reference
(models/diffmm.py:408-451, models/diffrec.py:291-310: h_i = tanh(x_{i+1} W1x^T + EB[i]),
x_i = c1_i (h_i W2^T + b2) + c2_i x_{i+1}) evaluated in fp64 on the host, and against our own
step-by-step chain (GMR_PSAMPLE_FOLD=0).

The fold is exact algebra (a_i = x_i W1x^T = c1_i (h_i P^T + v) + c2_i a_{i+1}, P = W1x W2, v = W1x b2;
the t = 0 posterior drops x_1 since c2_0 = 0), so both chains must sit at fp32 rounding distance from
the fp64 chain: the fold's error is held to <= 2x the step-by-step chain's error (plus a 1e-6 floor) and
<= 2e-5 relative to the output scale, at DiffMM's T = 5 and DiffRec's T = 100, on every GEMM path (split
-bf16 default and fp32 MFMA).  The top-1 of every row agrees with the fp64 chain's except where the
fp64 values of the two picks tie within 1e-5.  The baby-shape end-to-end checks against the reference
(tests/test_baby_gpu.py::test_p_sample_top1_all_users, tests/test_diffrec_baby_gpu.py) run the fold."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _chain64(x0, W1x, EB, W2, b2, c1, c2):
    x = x0.astype(np.float64)
    for i in reversed(range(len(c1))):
        h = np.tanh(x @ W1x.T + EB[i])
        x = c1[i] * (h @ W2.T + b2) + c2[i] * x
    return x


@pytest.mark.parametrize("T,H,sched", [(5, 256, "diffmm"), (100, 96, "diffrec")])
@pytest.mark.parametrize("x6", [True, False], ids=["x6", "f32"])
def test_p_sample_fold_vs_fp64_chain(T, H, sched, x6, monkeypatch):
    from gmr import kernels as K
    from gmr import denoise as dn
    from gmr.diffmm import diffmm_tables
    from gmr.diffrec import diffrec_tables
    if not x6:
        monkeypatch.setattr(K, "GEMM_TILE_FLAGS", 1 << 27)  # GMR_GEMM_F32: every product on the fp32-input MFMA
    torch.manual_seed(3)
    rng = np.random.default_rng(T + H)
    I, E, B = 1501, 10, 300
    den = dn.Denoiser(I, H, E, DEV)
    den.init_like_reference()
    tab = diffmm_tables(0.1, 1e-4, 0.02, T) if sched == "diffmm" else diffrec_tables("linear", 1e-4, 1e-4, 0.02, T)
    c1 = [float(np.float32(c)) for c in tab["c1"]]
    c2 = [float(np.float32(c)) for c in tab["c2"]]
    assert c2[0] == 0.0
    deg = rng.integers(1, 30, size=B)
    uptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    uit = np.concatenate([np.sort(rng.choice(I, size=d, replace=False)) for d in deg]).astype(np.int32)
    users = torch.arange(B, dtype=torch.int32, device=DEV)
    up, ui = torch.as_tensor(uptr).to(DEV), torch.as_tensor(uit).to(DEV)
    x0 = np.zeros((B, I), np.float32)
    for b in range(B):
        x0[b, uit[uptr[b]:uptr[b + 1]]] = 1.0
    EB, _, _ = den.time_bias(T)
    den.refresh_w1t()
    den.refresh_fold()
    Ip = (I + 3) // 4 * 4
    outs = {}
    for fold in (True, False):
        x = torch.zeros((B, Ip), device=DEV)[:, :I]
        x.copy_(torch.as_tensor(x0))
        h = torch.empty((B, H), device=DEV)
        if fold:
            a = torch.empty((B, H), device=DEV)
            den.p_sample_fold(users, up, ui, EB, c1, c2, x, a, h)
        else:
            for i in reversed(range(T)):
                if i == T - 1:
                    den.hidden_sparse(users, up, ui, h, EB[i])
                else:
                    den.hidden(x, h, EB, t_const=i)
                den.posterior_step(h, x, c1[i], c2[i])
        outs[fold] = x.cpu().numpy().astype(np.float64)
    s = den.slab
    W1x = s.view("W1")[:, :I].cpu().numpy().astype(np.float64)
    W2 = s.view("W2").cpu().numpy().astype(np.float64)
    b2 = s.view("b2").cpu().numpy().astype(np.float64)
    want = _chain64(x0, W1x, EB.cpu().numpy().astype(np.float64), W2, b2, np.float64(c1), np.float64(c2))
    scale = np.abs(want).max()
    e_fold = np.abs(outs[True] - want).max() / scale
    e_step = np.abs(outs[False] - want).max() / scale
    assert e_fold <= 2.0 * e_step + 1e-6 and e_fold <= 2e-5, (e_fold, e_step)
    top_f = outs[True].argmax(1)
    top_w = want.argmax(1)
    r = np.nonzero(top_f != top_w)[0]
    gap = want[r, top_w[r]] - want[r, top_f[r]]
    assert (gap <= 1e-5 * np.maximum(np.abs(want[r, top_w[r]]), 1.0)).all(), (r[:5], gap[:5])
