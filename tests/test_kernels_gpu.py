"""HIP kernels vs the CPU oracle / torch-fp32 references, through the C-ABI (GPU only)."""
import os

import numpy as np
import pytest
import torch

from oracle import eval_ref, graph_ref, model_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def K():
    from gmr import kernels, _lib
    _lib.load()
    return kernels


def _rng(s=0):
    return np.random.default_rng(s)


def _user_csr(U, I, rows, cols):
    key = np.unique(rows.astype(np.int64) * I + cols)
    u, i = key // I, key % I
    ptr = np.zeros(U + 1, np.int64)
    np.add.at(ptr, u + 1, 1)
    return np.cumsum(ptr).astype(np.int32), i.astype(np.int32)


def _dev(a, dt=None):
    t = torch.as_tensor(np.ascontiguousarray(a))
    if dt is not None:
        t = t.to(dt)
    return t.to(DEV)


@pytest.mark.parametrize("self_loops,eps", [(0, 1e-7), (1, 0.0)])
def test_bipartite_build_bit_exact(K, golden, self_loops, eps):
    g = golden("diffmm_tiny")
    U, I = int(g["U"]), int(g["I"])
    if self_loops:
        rows, cols = np.repeat(np.arange(U), 3), g["ui_k3_items"].reshape(-1)
        want = graph_ref.ui_adj_csr(U, I, rows, cols)
    else:
        rows, cols = g["train_rows"], g["train_cols"]
        want = graph_ref.norm_adj_csr(U, I, rows, cols)
    uptr, uitems = _user_csr(U, I, rows, cols)
    csr = K.bipartite_symnorm(U, I, _dev(uptr), _dev(uitems), self_loops, eps)
    torch.cuda.synchronize()
    assert np.array_equal(csr.rowptr.cpu().numpy(), want[0])
    assert np.array_equal(csr.col.cpu().numpy(), want[1])
    assert np.array_equal(csr.val.cpu().numpy().view(np.uint32), want[2].view(np.uint32))


@pytest.mark.parametrize("self_loops", [0, 1])
def test_bipartite_build_large_hubs(K, self_loops):
    # item rows above 256 users take the LDS-bitmap ordering path, shorter ones the rank path
    rng = _rng(1)
    U, I = 3000, 500
    rows = np.repeat(np.arange(U), 7)
    p = 1.0 / np.arange(1, I + 1) ** 1.2
    cols = rng.choice(I, size=rows.size, p=p / p.sum())
    if self_loops:
        want = graph_ref.ui_adj_csr(U, I, rows, cols)
    else:
        want = graph_ref.norm_adj_csr(U, I, rows, cols)
    uptr, uitems = _user_csr(U, I, rows, cols)
    assert np.bincount(uitems, minlength=I).max() > 256
    csr = K.bipartite_symnorm(U, I, _dev(uptr), _dev(uitems), self_loops, 0.0 if self_loops else 1e-7)
    assert np.array_equal(csr.rowptr.cpu().numpy(), want[0])
    assert np.array_equal(csr.col.cpu().numpy(), want[1])
    assert np.array_equal(csr.val.cpu().numpy().view(np.uint32), want[2].view(np.uint32))


def test_bipartite_build_many_items(K):
    """I above the LDS-privatised counting limit (8192 items): global-atomic path."""
    rng = _rng(6)
    U, I = 2000, 9000
    rows = np.repeat(np.arange(U), 4)
    p = 1.0 / np.arange(1, I + 1) ** 1.1
    cols = rng.choice(I, size=rows.size, p=p / p.sum())
    want = graph_ref.ui_adj_csr(U, I, rows, cols)
    uptr, uitems = _user_csr(U, I, rows, cols)
    csr = K.bipartite_symnorm(U, I, _dev(uptr), _dev(uitems), 1, 0.0)
    assert np.array_equal(csr.rowptr.cpu().numpy(), want[0])
    assert np.array_equal(csr.col.cpu().numpy(), want[1])
    assert np.array_equal(csr.val.cpu().numpy().view(np.uint32), want[2].view(np.uint32))


LANE32, PACKED32, CHUNK = (1 << 16) | 32, (1 << 17) | (1 << 16) | 32, 1 << 18
# segment, blocked, lane, packed lane, chunk plans
SPMM_SEGS = [64, 128, 512, 2048, LANE32, (1 << 16) | 64, (1 << 16) | 128, PACKED32, CHUNK]


@pytest.mark.parametrize("seg", SPMM_SEGS)
@pytest.mark.parametrize("nb", [1, 2, 4])
def test_spmm_vs_oracle(K, nb, seg):
    rng = _rng(2)
    U, I = 2500, 900
    deg = rng.integers(1, 20, size=U)
    deg[::97] = 0  # users without interactions -> empty rows
    rows = np.repeat(np.arange(U), deg)
    p = 1.0 / np.arange(1, I + 1) ** 1.1
    cols = rng.choice(I, size=rows.size, p=p / p.sum())  # hub items (rows > 1024 nnz) and never-seen items
    rp, col, val = graph_ref.norm_adj_csr(U, I, rows, cols)
    assert np.diff(rp).max() > 1024 and (np.diff(rp) == 0).any()
    N = U + I
    csr = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=seg)
    X = rng.standard_normal((N, 64 * nb)).astype(np.float32)
    Y0 = rng.standard_normal((N, 64 * nb)).astype(np.float32)
    Xd, Yd = _dev(X), _dev(Y0)
    blocks = [(Xd[:, 64 * b:64 * (b + 1)],) for b in range(nb)]
    K.CSR.spmm(csr, Yd, blocks, alpha=0.7, beta=0.3)
    A = graph_ref.csr_to_dense(rp, col, val).astype(np.float64)
    want = 0.7 * (A @ X.astype(np.float64)) + 0.3 * Y0
    np.testing.assert_allclose(Yd.cpu().numpy(), want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("seg", SPMM_SEGS)
def test_spmm_split_sources(K, seg):
    rng = _rng(3)
    U, I = 300, 200
    rows = np.repeat(np.arange(U), 6)
    cols = rng.integers(0, I, size=rows.size)
    rp, col, val = graph_ref.norm_adj_csr(U, I, rows, cols)
    csr = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=seg)
    uE = rng.standard_normal((U, 64)).astype(np.float32)
    F = rng.standard_normal((I, 128)).astype(np.float32)
    uEd, Fd = _dev(uE), _dev(F)
    out = torch.empty((U + I, 128), device=DEV)
    csr.spmm(out, [(uEd, Fd[:, :64]), (uEd, Fd[:, 64:])], split=U)
    A = graph_ref.csr_to_dense(rp, col, val).astype(np.float64)
    want0 = A @ np.concatenate([uE, F[:, :64]]).astype(np.float64)
    want1 = A @ np.concatenate([uE, F[:, 64:]]).astype(np.float64)
    np.testing.assert_allclose(out.cpu().numpy(), np.concatenate([want0, want1], 1), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("nb", [1, 2, 4])
def test_spmm_packed_bit_exact_vs_lane(K, nb):
    """The packed lane plan sums every row in the lane plan's order: bit-identical outputs, on a
    graph with hub rows, empty rows and rows of degree 31/32/33 around the packed bucket limit."""
    rng = _rng(7)
    U, I = 3000, 1200
    deg = rng.integers(0, 40, size=U)
    deg[:30] = 32
    deg[30:60] = 33
    deg[60:90] = 31
    rows = np.repeat(np.arange(U), deg)
    p = 1.0 / np.arange(1, I + 1) ** 1.1
    cols = rng.choice(I, size=rows.size, p=p / p.sum())
    rp, col, val = graph_ref.norm_adj_csr(U, I, rows, cols)
    N = U + I
    lane = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=LANE32)
    packed = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=PACKED32)
    assert packed.plan_header[2] & 1 and packed.plan_header[0] > 0  # packed, with hub rows
    X = _dev(rng.standard_normal((N, 64 * nb)).astype(np.float32))
    Y0 = rng.standard_normal((N, 64 * nb)).astype(np.float32)
    outs = []
    for g in (lane, packed):
        Yd = _dev(Y0)
        g.spmm(Yd, [(X[:, 64 * b:64 * (b + 1)],) for b in range(nb)], alpha=0.9, beta=0.25)
        outs.append(Yd.cpu().numpy())
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


@pytest.mark.parametrize("seg", [LANE32, PACKED32, CHUNK])
@pytest.mark.parametrize("nb", [1, 2, 4])
def test_spmm_panel_sources_bit_exact(K, nb, seg):
    """gmr_spmm_panel_f32: X as column panels gives the row-major product bit for bit."""
    rng = _rng(8)
    U, I = 2000, 700
    deg = rng.integers(0, 30, size=U)
    rows = np.repeat(np.arange(U), deg)
    p = 1.0 / np.arange(1, I + 1) ** 1.1
    cols = rng.choice(I, size=rows.size, p=p / p.sum())
    rp, col, val = graph_ref.norm_adj_csr(U, I, rows, cols)
    N = U + I
    g = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=seg)
    X = _dev(rng.standard_normal((N, 64 * nb)).astype(np.float32))
    Y0 = rng.standard_normal((N, 64 * nb)).astype(np.float32)
    Ya, Yb = _dev(Y0), _dev(Y0)
    g.spmm(Ya, [(X[:, 64 * b:64 * (b + 1)],) for b in range(nb)], alpha=1.25, beta=0.5)
    W = 32 if nb == 4 else 16
    Xp = X.reshape(N, 64 * nb // W, W).permute(1, 0, 2).contiguous()
    K.spmm_panel(g, Yb, Xp, nb, alpha=1.25, beta=0.5)
    assert torch.equal(Ya.view(torch.int32), Yb.view(torch.int32))
    with pytest.raises(ValueError):
        K.spmm_panel(g, Yb, Xp[:, :-1], nb)


@pytest.mark.parametrize("E,I", [(300, 1000), (64, 64), (4096, 6710), (1, 7)])
def test_score_f16_vs_torch(K, E, I):
    """gmr_score_f16 (fp16 MFMA scoring, config 5) against torch on the same fp16-rounded inputs:
    fp16 x fp16 products are exact in fp32, so only the summation order differs."""
    rng = _rng(10)
    A = torch.zeros((E, 68), device=DEV)[:, :64]  # padded rows: lda = 68
    A.copy_(_dev(0.1 * rng.standard_normal((E, 64)).astype(np.float32)))
    B = _dev(0.1 * rng.standard_normal((I, 64)).astype(np.float32))
    C = torch.full((E, I + 5), 7.0, device=DEV)
    K.score_f16(A, B, C[:, :I])
    want = A.half().float() @ B.half().float().T
    np.testing.assert_allclose(C[:, :I].cpu().numpy(), want.cpu().numpy(), rtol=1e-5, atol=1e-6)
    assert torch.all(C[:, I:] == 7.0)  # nothing written past the I columns
    with pytest.raises(ValueError):
        K.score_f16(A[:, :32], B[:, :32], C[:, :I])


@pytest.mark.parametrize("seg", [LANE32, PACKED32])
def test_spmm_multi_outputs_bit_exact(K, seg):
    """gmr_spmm_multi_f32: two independent 128-column products of one matrix in one launch, with
    split sources and per-block outputs, equal the two separate products (bit for bit on the
    rows of degree <= 32; the hub rows' partial sums split by 8- instead of 4-lane groups)."""
    rng = _rng(9)
    U, I = 2200, 800
    deg = rng.integers(0, 30, size=U)
    rows = np.repeat(np.arange(U), deg)
    p = 1.0 / np.arange(1, I + 1) ** 1.1
    cols = rng.choice(I, size=rows.size, p=p / p.sum())
    rp, col, val = graph_ref.norm_adj_csr(U, I, rows, cols)
    N = U + I
    g = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=seg)
    G = _dev(rng.standard_normal((N, 128)).astype(np.float32))
    E = _dev(rng.standard_normal((I, 64)).astype(np.float32))
    Q = _dev(rng.standard_normal((N, 128)).astype(np.float32))
    H1, K1 = torch.empty((N, 128), device=DEV), torch.empty((N, 128), device=DEV)
    g.spmm(H1, [(G[:, :64], E), (G[:, 64:], E)], split=U)
    g.spmm(K1, [(Q[:, :64],), (Q[:, 64:],)])
    H2, K2 = torch.empty((N, 128), device=DEV), torch.empty((N, 128), device=DEV)
    K.spmm_multi(g, [H2[:, :64], H2[:, 64:], K2[:, :64], K2[:, 64:]],
                 [(G[:, :64], E), (G[:, 64:], E), (Q[:, :64], Q[U:, :64]), (Q[:, 64:], Q[U:, 64:])], split=U)
    short = torch.as_tensor(np.diff(rp) <= 32, device=DEV)
    assert torch.equal(H1[short].view(torch.int32), H2[short].view(torch.int32))
    assert torch.equal(K1[short].view(torch.int32), K2[short].view(torch.int32))
    np.testing.assert_allclose(H2.cpu().numpy(), H1.cpu().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(K2.cpu().numpy(), K1.cpu().numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("seg", [128, LANE32, (1 << 16) | 128, PACKED32, CHUNK])
def test_spmm_empty_runs_and_repeat(K, seg):
    """Long runs of empty rows, a tiny and an empty matrix,
    and repeated products: bit-identical
    results across calls."""
    rng = _rng(4)
    for n, nnz_rows in ((700, 3), (700, 0), (4000, 600)):
        deg = np.zeros(n, dtype=np.int64)
        live = rng.choice(n, size=nnz_rows, replace=False)
        deg[live] = rng.integers(1, 400, size=nnz_rows)
        rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
        col = rng.integers(0, n, size=int(rp[-1])).astype(np.int32)
        val = rng.standard_normal(col.size).astype(np.float32)
        csr = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=seg)
        X = rng.standard_normal((n, 128)).astype(np.float32)
        Xd = _dev(X)
        Y0 = rng.standard_normal((n, 128)).astype(np.float32)
        blocks = [(Xd[:, :64],), (Xd[:, 64:],)]
        outs = []
        for _ in range(3):
            Yd = _dev(Y0)
            csr.spmm(Yd, blocks, alpha=1.5, beta=-0.5)
            outs.append(Yd.cpu().numpy())
        A = np.zeros((n, n))
        np.add.at(A, (np.repeat(np.arange(n), np.diff(rp)), col), val.astype(np.float64))  # duplicates add
        want = 1.5 * (A @ X.astype(np.float64)) - 0.5 * Y0
        np.testing.assert_allclose(outs[0], want, rtol=1e-5, atol=1e-4)
        for o in outs[1:]:
            assert np.array_equal(o.view(np.uint32), outs[0].view(np.uint32))


GEMM_CASES = [
    # (M, N, K, ta, tb)
    (2048, 1000, 7050, 0, 1), (2048, 7050, 1000, 0, 1), (2048, 1000, 7050, 0, 0), (7050, 1000, 2048, 1, 0),
    (97, 61, 33, 0, 0), (61, 97, 130, 1, 1), (130, 64, 4096, 0, 0), (4096, 64, 7050, 1, 0), (37, 5, 3, 1, 0),
]


@pytest.mark.parametrize("M,N,Kd,ta,tb", GEMM_CASES)
def test_gemm_vs_torch_fp32(K, M, N, Kd, ta, tb):
    torch.manual_seed(0)
    A = torch.randn(Kd, M) if ta else torch.randn(M, Kd)
    B = torch.randn(N, Kd) if tb else torch.randn(Kd, N)
    ref = (A.T if ta else A).double() @ (B.T if tb else B).double()
    C = torch.empty(M, N, device=DEV)
    K.gemm(A.to(DEV), B.to(DEV), C, trans_a=bool(ta), trans_b=bool(tb))
    err = (C.cpu().double() - ref).abs().max().item()
    scale = ((A.abs().T if ta else A.abs()).double() @ (B.abs().T if tb else B.abs()).double()).max().item()
    assert err <= 2e-6 * scale, (err, scale)


def test_gemm_unaligned_ld(K):
    torch.manual_seed(1)
    A = torch.randn(50, 71)[:, :69]  # lda = 71 (not a multiple of 4)
    B = torch.randn(69, 33)
    C = torch.empty(50, 33, device=DEV)
    K.gemm(A.to(DEV), B.to(DEV), C)
    np.testing.assert_allclose(C.cpu().numpy(), (A @ B).numpy(), rtol=1e-4, atol=1e-4)


def test_gemm_epilogues(K):
    torch.manual_seed(2)
    M, N, Kd, T = 200, 96, 150, 5
    A, B = torch.randn(M, Kd), torch.randn(N, Kd)
    acc = A.double() @ B.double().T
    eb = torch.randn(T, N)
    t = torch.randint(0, T, (M,), dtype=torch.int32)
    C = torch.empty(M, N, device=DEV)
    K.gemm(A.to(DEV), B.to(DEV), C, trans_b=True, epi=K.EPI_BIAS_TANH, bias=eb.to(DEV), bias_row=t.to(DEV), ld_bias=N)
    np.testing.assert_allclose(C.cpu().numpy(), torch.tanh(acc + eb[t.long()].double()).numpy(), rtol=1e-5, atol=1e-5)
    aux = torch.randn(M, N)
    b = torch.randn(N)
    K.gemm(A.to(DEV), B.to(DEV), C.copy_(aux.to(DEV)), trans_b=True, epi=K.EPI_POSTERIOR, bias=b.to(DEV), aux=C,
           slope=0.25, beta=0.75)
    np.testing.assert_allclose(C.cpu().numpy(), (0.25 * (acc + b.double()) + 0.75 * aux.double()).numpy(), rtol=1e-5,
                               atol=1e-5)
    K.gemm(A.to(DEV), B.to(DEV), C, trans_b=True, epi=K.EPI_DTANH, aux=aux.to(DEV))
    np.testing.assert_allclose(C.cpu().numpy(), (acc * (1 - aux.double() ** 2)).numpy(), rtol=1e-5, atol=1e-4)
    K.gemm(A.to(DEV), B.to(DEV), C, trans_b=True, epi=K.EPI_LEAKY, slope=0.2)
    np.testing.assert_allclose(C.cpu().numpy(), torch.nn.functional.leaky_relu(acc, 0.2).numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("k", [1, 10, 50])
def test_topk_rows_vs_oracle(K, k):
    rng = _rng(4)
    S = rng.standard_normal((300, 7050)).astype(np.float32)
    S[:, ::7] = np.float32(0.5)   # many exact ties
    S[5] = 1.0                     # all-equal row
    S[6, :100] = -1e10
    out = torch.empty((300, k), dtype=torch.int32, device=DEV)
    K.topk_rows(_dev(S), k, out)
    assert np.array_equal(out.cpu().numpy(), eval_ref.topk_rows(S, k))


@pytest.mark.parametrize("col0,n_cols", [(0, 7050), (0, 7051), (1, 7049), (3, 64)])
def test_argmax_rows_vector_and_tail_paths(K, col0, n_cols):
    """k = 1 (argmax_rows_kernel): the 16-byte-row path (four columns per load, round 6) and the scalar path
    (rows not 16-byte aligned), with ragged widths, exact ties (lowest index wins) and -1e10 blocks."""
    rng = _rng(43)
    S = rng.standard_normal((97, 7056)).astype(np.float32)
    S[:, ::3] = np.float32(2.5)
    S[4, :] = np.float32(-1e10)
    Sd = _dev(S)[:, col0:col0 + n_cols]
    out = torch.empty((97, 1), dtype=torch.int32, device=DEV)
    K.topk_rows(Sd, 1, out)
    assert np.array_equal(out.cpu().numpy(), eval_ref.topk_rows(S[:, col0:col0 + n_cols], 1))


def test_mask_and_topk_golden(K, golden):
    g = golden("diffmm_tiny")
    s = _dev(g["eval_scores_raw"])
    K.mask_scores(s, _dev(g["eval_mask_rows"], torch.int32), _dev(g["eval_mask_cols"], torch.int32))
    assert np.array_equal(s.cpu().numpy(), g["eval_scores_masked"])
    out = torch.empty((s.shape[0], 50), dtype=torch.int32, device=DEV)
    K.topk_rows(s, 50, out)
    assert np.array_equal(out.cpu().numpy(), eval_ref.topk_rows(g["eval_scores_masked"], 50))


def test_eval_metrics_vs_oracle(K, golden_meta):
    rng = _rng(5)
    n, Kk = 1000, 50
    topk = np.stack([rng.choice(400, size=Kk, replace=False) for _ in range(n)]).astype(np.int32)
    pos = [np.sort(rng.choice(400, size=int(rng.integers(1, 80)), replace=False)) for _ in range(n)]
    ptr = np.concatenate([[0], np.cumsum([len(p) for p in pos])]).astype(np.int64)
    from gmr import _lib
    parts = torch.empty(_lib.load().gmr_eval_metrics_partials(n), dtype=torch.float64, device=DEV)
    sums = torch.empty(32, dtype=torch.float64, device=DEV)
    ks = _dev(np.array([5, 10, 20, 50], np.int32))
    K.eval_metrics(_dev(topk), _dev(ptr), _dev(np.concatenate(pos).astype(np.int32)), ks, parts, sums)
    got = sums.cpu().numpy().reshape(4, 8)[:, :4] / n
    curves = eval_ref.metric_curves(eval_ref.hit_matrix(topk, pos), [len(p) for p in pos])
    for mi, m in enumerate(["recall", "ndcg", "precision", "map"]):
        np.testing.assert_allclose(got[mi], curves[m][[4, 9, 19, 49]], rtol=1e-12, atol=1e-14)


def test_adam_vs_torch(K):
    rng = _rng(6)
    p0 = rng.standard_normal(1000).astype(np.float32)
    gs = [[rng.standard_normal(1000).astype(np.float32)] for _ in range(4)]
    want = model_ref.adam_reference([p0], gs, lr=1e-3)[0]
    p, m, v = _dev(p0), torch.zeros(1000, device=DEV), torch.zeros(1000, device=DEV)
    for i, g in enumerate(gs):
        K.adam(p, _dev(g[0]), m, v, 1e-3, 0.9, 0.999, 1e-8, 0.0, i + 1)
    np.testing.assert_allclose(p.cpu().numpy(), want, rtol=3e-7, atol=1e-7)  # fp32 contraction: <= 1 ulp


@pytest.mark.parametrize("n", [1003, 4096, 3])
def test_adam_vector_path_bit_exact(K, n):
    """gmr_adam_f32's float4 kernel (16-byte aligned operands) against its scalar kernel (the same buffers
    offset by one element, so unaligned): p, m and v bit for bit over a few steps with weight decay; n not a
    multiple of four exercises the scalar tail."""
    rng = _rng(9)
    p0 = rng.standard_normal(n).astype(np.float32)
    gs = [rng.standard_normal(n).astype(np.float32) for _ in range(3)]
    out = []
    for off in (0, 1):  # the same n values at element offset 0 (aligned) and 1 (unaligned)
        sl = slice(off, off + n)
        p, m, v = (torch.zeros(n + 1, device=DEV) for _ in range(3))
        p[sl] = _dev(p0)
        for i, g in enumerate(gs):
            gd = torch.zeros(n + 1, device=DEV)
            gd[sl] = _dev(g)
            K.adam(p[sl], gd[sl], m[sl], v[sl], 1e-3, 0.9, 0.999, 1e-8, 0.01, i + 1)
        out.append([t[sl].cpu() for t in (p, m, v)])
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_normalize_rows_and_bwd(K):
    torch.manual_seed(3)
    x = torch.randn(333, 128)
    x[7] = 0.0
    xr = x.clone().requires_grad_(True)
    y = torch.nn.functional.leaky_relu(xr, 0.2)
    out = torch.nn.functional.normalize(y[:, :64])
    dy = torch.randn(333, 64)
    out.backward(dy)
    F = torch.nn.functional.leaky_relu(x, 0.2).to(DEV)
    yd = torch.empty(333, 64, device=DEV)
    nrm = torch.empty(333, device=DEV)
    K.normalize_rows(F[:, :64], yd, nrm)
    np.testing.assert_allclose(yd.cpu().numpy(), out.detach().numpy(), rtol=1e-6, atol=1e-7)
    dx = torch.empty(333, 64, device=DEV)
    K.normalize_rows_bwd(yd, nrm, dy.to(DEV), dx, slope=0.2)
    np.testing.assert_allclose(dx.cpu().numpy(), xr.grad[:, :64].numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,n", [(2048, 19445), (974, 7050), (37, 100), (300, 33)])
@pytest.mark.parametrize("pipe", ["x6", "f32"])
def test_contrast_fused_vs_fp64(K, B, n, pipe, monkeypatch):
    """K8 fused InfoNCE (gmr_contrast_fused_f32: contrastLoss fwd + bwd without the B x n logits)
    vs a float64 restatement of models/diffmm.py:251-258 on unit rows (|logit| <= 1/temp, no max
    subtraction, as the reference).  Loss rows rtol 1e-5; gradients rtol 2e-4 of their scale.  Both
    pipes: the split-bf16 MFMA passes (GMR_CL_X6, default) and the fp32-input MFMA ones."""
    monkeypatch.setenv("GMR_CL_X6", "1" if pipe == "x6" else "0")
    rng = _rng(11)
    off = 5
    N = off + n + 3
    C = rng.standard_normal((N, 128))
    C[:, :64] /= np.linalg.norm(C[:, :64], axis=1, keepdims=True)
    C[:, 64:] /= np.linalg.norm(C[:, 64:], axis=1, keepdims=True)
    C = C.astype(np.float32)
    nodes = rng.integers(0, n, B).astype(np.int32)
    temp, coef = 0.1, 0.01 / B
    Cd, nd = _dev(C), _dev(nodes)
    P = torch.empty((B, 64), device=DEV)
    K.gather_rows(Cd[:, :64], nd, P, off=off)
    loss = torch.empty(B, device=DEV)
    contrib = torch.empty((B, 128), device=DEV)
    dbuf = torch.full((N, 128), float("nan"), device=DEV)
    ws = K.contrast_workspace(B, n, DEV, "test_cl")
    K.contrast_fused(P, Cd[off:off + n, 64:], Cd, nd, off, 1.0 / temp, coef, loss, contrib, dbuf[off:off + n, 64:], ws)
    p = C[off + nodes, :64].astype(np.float64)
    T = C[off:off + n, 64:].astype(np.float64)
    E = np.exp(p @ T.T / temp)
    z = E.sum(1)
    p2 = T[nodes]
    k = coef / temp
    want_loss = np.log(z) - (p * p2).sum(1) / temp
    want_dp = k * (E @ T / z[:, None] - p2)
    want_dt = k * (E / z[:, None]).T @ p
    np.testing.assert_allclose(loss.cpu().numpy(), want_loss, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(contrib[:, :64].cpu().numpy(), want_dp, rtol=2e-4, atol=2e-4 * np.abs(want_dp).max())
    np.testing.assert_allclose(contrib[:, 64:].cpu().numpy(), -k * p, rtol=1e-6, atol=1e-12)
    got_dt = dbuf[off:off + n, 64:].cpu().numpy()
    np.testing.assert_allclose(got_dt, want_dt, rtol=2e-4, atol=2e-4 * np.abs(want_dt).max())
    assert np.isnan(dbuf[:off].cpu().numpy()).all() and np.isnan(dbuf[off:off + n, :64].cpu().numpy()).all()


@pytest.mark.parametrize("B,n", [(2048, 19445), (300, 7050), (37, 100)])
def test_contrast_two_fragments_bit_exact(K, B, n, monkeypatch):
    """GMR_CL_NF=2 (two 32-row fragments per wave, half the workgroups) keeps the chunking, so the
    loss, dP and dT are the one-fragment kernels' bit for bit (ragged B and n included)."""
    rng = _rng(12)
    C = rng.standard_normal((n, 128)).astype(np.float32)
    C /= np.linalg.norm(C, axis=1, keepdims=True)
    nodes = rng.integers(0, n, B).astype(np.int32)
    Cd, nd = _dev(C), _dev(nodes)
    P = torch.empty((B, 64), device=DEV)
    K.gather_rows(Cd[:, :64], nd, P, off=0)
    ws = K.contrast_workspace(B, n, DEV, "test_cl_nf")
    outs = []
    for nf in ("1", "2"):
        monkeypatch.setenv("GMR_CL_NF", nf)
        loss = torch.empty(B, device=DEV)
        contrib = torch.empty((B, 128), device=DEV)
        dt = torch.empty((n, 128), device=DEV)
        K.contrast_fused(P, Cd[:, 64:], Cd, nd, 0, 10.0, 0.01 / B, loss, contrib, dt[:, 64:], ws)
        outs.append((loss.cpu(), contrib.cpu(), dt[:, 64:].cpu()))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


@pytest.mark.parametrize("B,n", [(2048, 19445), (2048, 7050), (300, 7050), (37, 100), (300, 33), (64, 65)])
def test_contrast_pipelined_bit_exact(K, B, n, monkeypatch):
    """GMR_CL_PIPE (default): the split-bf16 InfoNCE passes with the next block's S product issued before
    this block's exp / split keep the staging, chunking and every sum of the unpipelined passes: loss,
    dP and dT bit for bit (chunks of one, two and many 32-row blocks, ragged last blocks)."""
    _contrast_env_bit_exact(K, B, n, monkeypatch, "GMR_CL_PIPE")


@pytest.mark.parametrize("B,n", [(2048, 19445), (2048, 7050), (300, 1000), (40, 97)])
def test_contrast_table_fixup_bit_exact(K, B, n, monkeypatch):
    """GMR_CL_FIXUP=1 (opt-in): the table pass sums its chunk partials itself (the last block of each
    128-row tile, in chunk order, counters left zero for the next call) instead of cl_table_reduce_kernel:
    dT bit for bit, and repeated calls (the counters reset) stay identical."""
    _contrast_env_bit_exact(K, B, n, monkeypatch, "GMR_CL_FIXUP", repeats=3)


@pytest.mark.parametrize("B,n", [(2048, 19445), (2048, 7050), (300, 1000), (37, 100), (64, 65)])
def test_contrast_rows_in_place_bit_exact(K, B, n, monkeypatch):
    """P = None (round 6): the passes read the batch rows CLN[off + nodes[i], :64] through the index instead of
    a gathered copy - loss, dP and dT bit for bit (ragged B and n, an offset table, repeated nodes); the
    unpipelined and fp32 forms refuse it."""
    monkeypatch.setenv("GMR_CL_X6", "1")
    monkeypatch.setenv("GMR_CL_PIPE", "1")
    rng = _rng(14)
    off = 7
    C = rng.standard_normal((off + n + 5, 128)).astype(np.float32)
    C /= np.linalg.norm(C, axis=1, keepdims=True)
    nodes = rng.integers(0, n, B).astype(np.int32)
    Cd, nd = _dev(C), _dev(nodes)
    P = torch.empty((B, 64), device=DEV)
    K.gather_rows(Cd[:, :64], nd, P, off=off)
    ws = K.contrast_workspace(B, n, DEV, "test_cl_inplace")
    outs = []
    for p in (P, None):
        loss = torch.empty(B, device=DEV)
        contrib = torch.empty((B, 128), device=DEV)
        dt = torch.empty((n, 128), device=DEV)
        K.contrast_fused(p, Cd[off:off + n, 64:], Cd, nd, off, 1.0 / 0.2, 0.01 / B, loss, contrib, dt[:, 64:], ws)
        outs.append((loss.cpu(), contrib.cpu(), dt[:, 64:].cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    for env in ("GMR_CL_PIPE", "GMR_CL_X6"):
        monkeypatch.setenv(env, "0")
        with pytest.raises(RuntimeError, match="pipelined"):
            K.contrast_fused(None, Cd[off:off + n, 64:], Cd, nd, off, 5.0, 0.01 / B, loss, contrib, dt[:, 64:], ws)
        monkeypatch.setenv(env, "1")


@pytest.mark.parametrize("B,n", [(2048, 19445), (2048, 7050), (300, 1000), (37, 100)])
def test_contrast_nbwd_pipelined_bit_exact(K, B, n, monkeypatch):
    """gmr_contrast_fused_nbwd_f32 (DiffMM's form: dT through the table view's normalize backward) on the pipelined
    passes against the unpipelined ones: loss, dP and dT bit for bit, with P given and P = NULL (rows read in
    place)."""
    from gmr import _lib
    from gmr.kernels import ptr, stream
    monkeypatch.setenv("GMR_CL_X6", "1")
    rng = _rng(15)
    off = 3
    C = rng.standard_normal((off + n + 2, 128)).astype(np.float32)
    C /= np.linalg.norm(C, axis=1, keepdims=True)
    nodes = rng.integers(0, n, B).astype(np.int32)
    Cd, nd = _dev(C), _dev(nodes)
    nrm = _dev(rng.uniform(0.5, 2.0, n + 8).astype(np.float32))
    P = torch.empty((B, 64), device=DEV)
    K.gather_rows(Cd[:, :64], nd, P, off=off)
    ws = K.contrast_workspace(B, n, DEV, "test_cl_nbwd")
    T = Cd[off:off + n, 64:]
    outs = []
    for pipe, p in (("0", P), ("1", P), ("1", None)):
        monkeypatch.setenv("GMR_CL_PIPE", pipe)
        loss = torch.empty(B, device=DEV)
        contrib = torch.empty((B, 128), device=DEV)
        dt = torch.full((n, 128), float("nan"), device=DEV)
        _lib.call("gmr_contrast_fused_nbwd_f32", B, n, ptr(p), 64 if p is not None else 128, ptr(T), 128, ptr(Cd),
                  ptr(nd), off, 5.0, 0.01 / B, ptr(loss), ptr(contrib), 128, ptr(dt[:, 64:]), 128, ptr(T), 128,
                  ptr(nrm), ptr(ws), ws.numel(), stream())
        outs.append((loss.cpu(), contrib.cpu(), dt[:, 64:].cpu()))
    assert torch.isfinite(outs[0][2]).all()
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


def _contrast_env_bit_exact(K, B, n, monkeypatch, env, repeats=1, value="1"):
    monkeypatch.setenv("GMR_CL_X6", "1")
    rng = _rng(13)
    C = rng.standard_normal((n, 128)).astype(np.float32)
    C /= np.linalg.norm(C, axis=1, keepdims=True)
    nodes = rng.integers(0, n, B).astype(np.int32)
    Cd, nd = _dev(C), _dev(nodes)
    P = torch.empty((B, 64), device=DEV)
    K.gather_rows(Cd[:, :64], nd, P, off=0)
    ws = K.contrast_workspace(B, n, DEV, "test_cl_" + env)
    outs = []
    for pipe in ["0"] + [value] * repeats:
        monkeypatch.setenv(env, pipe)
        loss = torch.empty(B, device=DEV)
        contrib = torch.empty((B, 128), device=DEV)
        dt = torch.empty((n, 128), device=DEV)
        K.contrast_fused(P, Cd[:, 64:], Cd, nd, 0, 1.0 / 0.2, 0.01 / B, loss, contrib, dt[:, 64:], ws)
        outs.append((loss.cpu(), contrib.cpu(), dt[:, 64:].cpu()))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


@pytest.mark.parametrize("nb", [1, 2, 4])
def test_spmm_chunk_rows_spanning_groups(K, nb):
    """Chunk plan: rows of degree 1..128 packed into 128-entry tasks, many of them crossing the
    8- / 16-entry lane-group boundaries (degrees 1, 2, 7, 9, 15, 17, 33, 64, 100, 127, 128, 129),
    hub rows of thousands and empty rows; against fp64 and bit-identical across repeats."""
    rng = _rng(11)
    n = 5000
    degs = np.array([1, 2, 7, 9, 15, 17, 33, 64, 100, 127, 128, 129, 0, 3000])
    deg = rng.choice(degs, size=n, p=[.2, .2, .1, .1, .05, .05, .05, .05, .05, .04, .04, .03, .03, .01])
    rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    col = rng.integers(0, n, size=int(rp[-1])).astype(np.int32)
    val = rng.standard_normal(col.size).astype(np.float32)
    g = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=CHUNK)
    hdr = g.plan_header
    assert hdr[0] == int((deg > 128).sum()) and hdr[2] == int((deg == 0).sum())
    assert hdr[3] == int(deg[(deg > 0) & (deg <= 128)].sum())
    X = rng.standard_normal((n, 64 * nb)).astype(np.float32)
    Y0 = rng.standard_normal((n, 64 * nb)).astype(np.float32)
    Xd = _dev(X)
    outs = []
    for _ in range(2):
        Yd = _dev(Y0)
        g.spmm(Yd, [(Xd[:, 64 * b:64 * (b + 1)],) for b in range(nb)], alpha=0.8, beta=0.4)
        outs.append(Yd.cpu().numpy())
    A = np.zeros((n, n))
    np.add.at(A, (np.repeat(np.arange(n), deg), col), val.astype(np.float64))
    want = 0.8 * (A @ X.astype(np.float64)) + 0.4 * Y0
    np.testing.assert_allclose(outs[0], want, rtol=1e-5, atol=1e-4)
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


@pytest.mark.parametrize("seg", [LANE32, PACKED32])
@pytest.mark.parametrize("nb", [1, 2, 4])
def test_spmm_split_hub_rows(K, nb, seg):
    """Lane plans cut hub rows longer than 8,192 entries into 1,024-entry segments whose partials a
    fixup pass adds in segment order (the rebuilt UI graph of a collapsed p_sample: one item row
    holding most users); shorter hubs stay whole.  Against fp64, bit-identical across repeats and
    between the launch entry points."""
    rng = _rng(12)
    U, I = 20000, 300
    top = rng.integers(0, I, U)
    r = rng.random(U)
    top[r < 0.6] = 5                                   # item 5: ~12k users (split)
    top[(r >= 0.6) & (r < 0.8)] = 17                   # item 17: ~4k users (a whole-row hub)
    rp, col, val = graph_ref.ui_adj_csr(U, I, np.arange(U), top)
    assert np.diff(rp).max() > 8192 and np.sort(np.diff(rp))[-2] > 2048
    N = U + I
    g = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=seg)
    assert g.flags & K.SPMM_HUB_FIXUP and g.plan_header[2] >> 1 >= 1
    X = rng.standard_normal((N, 64 * nb)).astype(np.float32)
    Y0 = rng.standard_normal((N, 64 * nb)).astype(np.float32)
    Xd = _dev(X)
    blocks = [(Xd[:, 64 * b:64 * (b + 1)],) for b in range(nb)]
    outs = []
    for _ in range(2):
        Yd = _dev(Y0)
        g.spmm(Yd, blocks, alpha=0.6, beta=0.5)
        outs.append(Yd.cpu().numpy())
    A = graph_ref.csr_to_dense(rp, col, val).astype(np.float64)
    want = 0.6 * (A @ X.astype(np.float64)) + 0.5 * Y0
    np.testing.assert_allclose(outs[0], want, rtol=1e-5, atol=1e-5)
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    Ym = [_dev(Y0[:, 64 * b:64 * (b + 1)].copy()) for b in range(nb)]
    K.spmm_multi(g, Ym, blocks, alpha=0.6, beta=0.5)
    got = np.concatenate([y.cpu().numpy() for y in Ym], 1)
    assert np.array_equal(got.view(np.uint32), outs[0].view(np.uint32))


def test_spmm_jobs_bit_exact(K):
    """gmr_spmm_jobs_f32: products of three matrices (a packed norm_adj-like plan, a UI graph whose
    hub rows are split into fixup segments, a small lane plan) in one launch, with split sources,
    1- and 2-block jobs and alpha/beta, equal the separate CSR.spmm calls bit for bit; two 4-block
    jobs likewise; mixing 4-block with narrower jobs is refused."""
    rng = _rng(21)
    U, I = 14000, 300
    deg = rng.integers(0, 30, size=U)
    rows = np.repeat(np.arange(U), deg)
    p = 1.0 / np.arange(1, I + 1) ** 1.1
    cols = rng.choice(I, size=rows.size, p=p / p.sum())
    g1 = K.CSR(*(_dev(a) for a in graph_ref.norm_adj_csr(U, I, rows, cols)), seg_nnz=PACKED32)
    top = rng.integers(0, I, U)
    top[rng.random(U) < 0.7] = 5
    g2 = K.CSR(*(_dev(a) for a in graph_ref.ui_adj_csr(U, I, np.arange(U), top)), seg_nnz=LANE32)
    assert g2.flags & K.SPMM_HUB_FIXUP
    Us, Is = 500, 90
    d3 = rng.integers(0, 6, size=Us)
    g3 = K.CSR(*(_dev(a) for a in graph_ref.norm_adj_csr(Us, Is, np.repeat(np.arange(Us), d3),
                                                          rng.integers(0, Is, size=d3.sum()))), seg_nnz=LANE32)
    N, N3 = U + I, Us + Is
    X = _dev(rng.standard_normal((N, 256)).astype(np.float32))
    E = _dev(rng.standard_normal((I, 64)).astype(np.float32))
    X3 = _dev(rng.standard_normal((N3, 64)).astype(np.float32))
    Y0 = rng.standard_normal((N, 256)).astype(np.float32)
    Y3 = rng.standard_normal((N3, 64)).astype(np.float32)
    jobs_in = [(g1, 2, [(X[:, :64], E), (X[:, 64:128], E)], U),
               (g2, 2, [(X[:, 128:192],), (X[:, 192:],)], None),
               (g3, 1, [(X3,)], None)]
    want = []
    for g, nb, blocks, split in jobs_in:
        y = _dev((Y3 if g is g3 else Y0)[:, :64 * nb].copy())
        g.spmm(y, blocks, split=split, alpha=0.7, beta=0.3)
        want.append(y.cpu().numpy())
    outs = [_dev((Y3 if g is g3 else Y0)[:, :64 * nb].copy()) for g, nb, _, _ in jobs_in]
    K.spmm_jobs([(g, o, blocks, split, None) for (g, nb, blocks, split), o in zip(jobs_in, outs)], alpha=0.7, beta=0.3)
    for w, o in zip(want, outs):
        assert np.array_equal(o.cpu().numpy().view(np.uint32), w.view(np.uint32))
    # two 4-block jobs
    w4 = []
    for g in (g1, g2):
        y = torch.empty((N, 256), device=DEV)
        g.spmm(y, [(X[:, 64 * b:64 * (b + 1)],) for b in range(4)])
        w4.append(y)
    o4 = [torch.empty((N, 256), device=DEV) for _ in range(2)]
    K.spmm_jobs([(g, o, [(X[:, 64 * b:64 * (b + 1)],) for b in range(4)], None, None) for g, o in zip((g1, g2), o4)])
    for w, o in zip(w4, o4):
        assert torch.equal(w.view(torch.int32), o.view(torch.int32))
    with pytest.raises(Exception, match="lane width"):
        K.spmm_jobs([(g1, o4[0], [(X[:, 64 * b:64 * (b + 1)],) for b in range(4)], None, None),
                     (g3, _dev(Y3.copy()), [(X3,)], None, None)])


@pytest.mark.parametrize("tile", [64, 128, 256, 256128, 128256, 12864])
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_gemm_glds_bit_exact_vs_register_staging(K, tile, ta, tb):
    """global_load_lds operand staging (GMR_GEMM_GLDS, swizzled k-contiguous LDS images) gives the
    register-staged kernel's sums bit for bit: ragged M/N edges, a partial last k tile, split-K
    slabs and the posterior epilogue; against torch fp32 as well."""
    GLDS, REG = 1 << 22, 1 << 23
    rng = _rng(31)
    for M, N, Kd, split in ((300, 200, 1000, 1), (517, 260, 70, 1), (64, 1000, 2048, 4), (1000, 64, 7050, 8)):
        A = _dev(rng.standard_normal((Kd, M) if ta else (M, Kd)).astype(np.float32))
        B = _dev(rng.standard_normal((N, Kd) if tb else (Kd, N)).astype(np.float32))
        bias = _dev(rng.standard_normal(N).astype(np.float32))
        outs = []
        for flag in (GLDS, REG):
            C = _dev(np.full((M, N), 0.5, dtype=np.float32))
            K.gemm(A, B, C, trans_a=bool(ta), trans_b=bool(tb), epi=K.EPI_POSTERIOR, bias=bias, aux=C, slope=0.9,
                   beta=0.1, tile=tile | flag, split_k=split)
            outs.append(C)
        assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32)), (M, N, Kd, split)
        ref = (A.t() if ta else A) @ (B.t() if tb else B)
        want = 0.9 * (ref + bias) + 0.1 * 0.5
        torch.testing.assert_close(outs[0], want, rtol=2e-4, atol=2e-3)


X6, F32 = 1 << 26, 1 << 27  # GMR_GEMM_X6 / GMR_GEMM_F32 tile flags (include/gmr.h)


# split-bf16 accuracy bar: per shape, the split kernel's max normalised error
# |C - C64| / (|A| |B|) is at most 1.25x the fp32-input MFMA kernel's on the same inputs (plus one
# 2^-24 floor for the tiny-K shapes whose errors are at the fp32 rounding of a single sum) and at
# most 6e-7 absolute.  A two-term (bf16 x 3) split would sit near 2^-16 ~ 1.5e-5 at K = 1,000 and
# 7,050 and fails both; the round-2 study measured 3.7e-7 (split) vs 4.2e-7 (fp32 MFMA).
X6_RATIO, X6_FLOOR, X6_ABS = 1.25, 2.0 ** -24, 6e-7


@pytest.mark.parametrize("tile", [0, 64, 128, 256128, 128256])
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_gemm_x6_fp32_accuracy(K, tile, ta, tb):
    """Split-bf16 products (GMR_GEMM_X6: x = hi + mid + lo exactly, six bf16 MFMA products) carry fp32
    accuracy: against an fp64 product the normalised error is within 1.25x the fp32-MFMA kernel's on
    the same inputs and below 6e-7, on ragged M / N edges, K = 1,000 and 7,050 (the denoiser
    products), K not a multiple of 32 or of 4 (padded rows), split-K slabs and values spanning
    2^-20 .. 2^20.  TN / NN / TT calls run as NT on k-contiguous copies of their operands."""
    rng = _rng(37)
    for M, N, Kd, split in ((300, 200, 1000, 1), (517, 260, 70, 1), (19, 33, 7, 1), (1000, 700, 7050, 4),
                            (640, 384, 1001, 2), (512, 1000, 7050, 1)):
        a = rng.standard_normal((M, Kd)) * np.exp2(rng.integers(-20, 21, size=(M, 1)))
        b = rng.standard_normal((N, Kd))
        pad = lambda x: np.pad(x, ((0, 0), (0, (-x.shape[1]) % 4))).astype(np.float32)  # noqa: E731  16-byte rows
        A = _dev(pad(a.T) if ta else pad(a))[:, :(M if ta else Kd)]
        B = _dev(pad(b) if tb else pad(b.T))[:, :(Kd if tb else N)]
        a64, b64 = torch.as_tensor(a, device=DEV), torch.as_tensor(b, device=DEV)
        a64, b64 = a64.float().double(), b64.float().double()
        ref = a64 @ b64.t()
        scale = a64.abs() @ b64.abs().t()
        err = {}
        for flag in (X6, F32):
            C = torch.empty(M, N, device=DEV)
            K.gemm(A, B, C, trans_a=bool(ta), trans_b=bool(tb), tile=tile | flag if tile else flag, split_k=split)
            err[flag] = ((C.double() - ref).abs() / scale).max().item()
        assert err[X6] <= X6_RATIO * err[F32] + X6_FLOOR, (M, N, Kd, split, err)
        assert err[X6] <= X6_ABS, (M, N, Kd, split, err)
    if tile and (tile != 64 or (ta, tb) == (0, 1)):
        # an explicit >= 128^2 tile with GMR_GEMM_X6 takes the split kernel in every layout, a 64^2 one
        # for plain NT calls (the other layouts keep the fp32 kernel: their operand copies cost more)
        assert _lib_kind(ta, tb, 1000, 700, 7050, tile | X6) == 6
    if tile == 64 and (ta, tb) != (0, 1):
        assert _lib_kind(ta, tb, 1000, 700, 7050, tile | X6) == 32


@pytest.mark.parametrize("tile", [128, 256128, 128256])
@pytest.mark.parametrize("ta,tb", [(0, 0), (1, 0)])
def test_gemm_x6_inplace_operands_bit_exact(K, tile, ta, tb):
    """TN / NN split-bf16 calls (default: their m- / n-contiguous operands copied k-contiguous; with
    GMR_X6_INPLACE = 1 / 2 read in place by gemm_x6.hip's MnTile, test_gemm_x6_inplace_subprocess) equal, bit
    for bit, the NT call on k-contiguous copies of the same operands (same plane images, same MFMA order), on
    ragged edges (M, N not multiples of 4; padded and unpadded leading dimensions), a partial last k tile and
    split-K slabs, with the posterior epilogue."""
    rng = _rng(39)
    for M, N, Kd, split, padded in ((517, 261, 1000, 1, True), (130, 1001, 2052, 4, False),
                                    (1000, 64, 7052, 2, True)):
        a = rng.standard_normal((M, Kd)).astype(np.float32)
        b = rng.standard_normal((N, Kd)).astype(np.float32)
        pad = lambda x: np.pad(x, ((0, 0), (0, (-x.shape[1]) % 4 if padded else 0)))  # noqa: E731  16-byte rows
        A = _dev(pad(a.T))[:, :M] if ta else _dev(a)
        B = _dev(pad(b.T))[:, :N]
        bias = _dev(rng.standard_normal(N).astype(np.float32))
        aux = _dev(rng.standard_normal((M, N)).astype(np.float32))
        outs = []
        for AA, BB, t_a, t_b in ((A, B, bool(ta), False), (_dev(a), _dev(b), False, True)):
            C = aux.clone()
            K.gemm(AA, BB, C, trans_a=t_a, trans_b=t_b, epi=K.EPI_POSTERIOR, bias=bias, aux=C, slope=0.5,
                   beta=0.25, tile=tile | X6, split_k=split)
            outs.append(C)
        assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32)), (M, N, Kd, split)
        want = 0.5 * (torch.as_tensor(a, dtype=torch.float64) @ torch.as_tensor(b, dtype=torch.float64).t()
                      + bias.double().cpu()) + 0.25 * aux.double().cpu()
        torch.testing.assert_close(outs[0].double().cpu(), want, rtol=1e-4, atol=2e-3)  # fp32 sums, K <= 7,052


@pytest.mark.timeout(180)
@pytest.mark.parametrize("mode", ["1", "2"])
def test_gemm_x6_inplace_subprocess(mode):
    """GMR_X6_INPLACE (read once per process) = 1: B read in place, the m-contiguous A of TN calls copied;
    = 2: both in place.  The bit-exact cases above (NN and TN), in a child process with that setting."""
    import subprocess
    import sys
    code = ("import sys; sys.path[:0] = ['tests', 'generative-multimodal-recommendation_amd']\n"
            "import test_kernels_gpu as t\nfrom gmr import kernels as K, _lib\n_lib.load()\n"
            "for tile in (128, 256128, 128256):\n    for ta in (0, 1):\n"
            "        t.test_gemm_x6_inplace_operands_bit_exact(K, tile, ta, 0)\n"
            "print('OK')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GMR_X6_INPLACE=mode)
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-2000:] + r.stderr[-2000:]


def _lib_kind(ta, tb, M, N, Kd, tile):
    from gmr import _lib
    return int(_lib.load().gmr_gemm_kernel_kind(ta, tb, M, N, Kd, tile, 0, 1))


def test_gemm_x6_epilogues(K):
    """The split-bf16 kernel runs the denoiser epilogues: BIAS_TANH with a per-row bias table index
    (the time-embedding collapse) and the in-place p_sample POSTERIOR, at the fp32-MFMA kernel's
    accuracy (same ratio bar as test_gemm_x6_fp32_accuracy; both epilogues are 1-Lipschitz in the
    product, the normaliser adds the fp32 rounding of the epilogue's own terms)."""
    rng = _rng(38)
    M, N, Kd, T = 600, 520, 1000, 5
    A = _dev(rng.standard_normal((M, Kd)).astype(np.float32))
    B = _dev(rng.standard_normal((N, Kd)).astype(np.float32))
    acc = A.double() @ B.double().t()
    scale = A.double().abs() @ B.double().abs().t()
    eb = _dev(rng.standard_normal((T, N)).astype(np.float32))
    t = _dev(rng.integers(0, T, size=M), torch.int32)
    want = torch.tanh(acc + eb.double()[t.long()])
    for tile in (128, 64):
        err = {}
        for flag in (X6, F32):
            C = torch.empty(M, N, device=DEV)
            K.gemm(A, B, C, trans_b=True, epi=K.EPI_BIAS_TANH, bias=eb, bias_row=t, ld_bias=N, tile=tile | flag)
            err[flag] = ((C.double() - want).abs() / (scale + 1.0)).max().item()
        assert err[X6] <= X6_RATIO * err[F32] + X6_FLOOR and err[X6] <= X6_ABS, (tile, err)
    aux = _dev(rng.standard_normal((M, N)).astype(np.float32))
    bias = _dev(rng.standard_normal(N).astype(np.float32))
    want = 0.25 * (acc + bias.double()) + 0.75 * aux.double()
    for flag in (X6, F32):
        C = aux.clone()
        K.gemm(A, B, C, trans_b=True, epi=K.EPI_POSTERIOR, bias=bias, aux=C, slope=0.25, beta=0.75,
               tile=(256128 if flag == X6 else 128) | flag)
        err[flag] = ((C.double() - want).abs() / (0.25 * scale + aux.double().abs() + 1.0)).max().item()
    assert err[X6] <= X6_RATIO * err[F32] + X6_FLOOR and err[X6] <= X6_ABS, err


def test_split3_planes_exact(K):
    """gmr_split3_planes: hi + mid + lo == x exactly (fp32), pad columns zero."""
    rng = _rng(40)
    x = (rng.standard_normal((37, 70)) * np.exp2(rng.integers(-30, 31, size=(37, 1)))).astype(np.float32)
    p = K.Planes(40, 70, DEV).load(_dev(x))
    assert torch.equal(p.to_float()[:37].cpu(), torch.as_tensor(x))
    assert (p.t[:, :, 70:] == 0).all() and (p.t[:, 37:] == 0).all()


def test_gemm_x6_edge_values(K):
    """Split of edge values: |x| near FLT_MAX (where rounding hi to bf16 would overflow)
    splits by truncation and stays finite and accurate; inf / NaN operands give non-finite results
    exactly where the fp32-MFMA kernel does (an inf operand may come out NaN rather than inf: its
    cross terms inf * 0 meet the other operand's zero mid / lo terms)."""
    M, N, Kd = 64, 64, 256
    rng = _rng(39)
    a = rng.standard_normal((M, Kd)).astype(np.float32)
    b = (rng.standard_normal((N, Kd)) * 1e-30).astype(np.float32)
    a[3, :] = np.float32(3.3999e38) * np.sign(a[3, :])   # above bf16's max: RN would give inf
    a[5, 7] = np.float32(np.finfo(np.float32).max)
    A, B = _dev(a), _dev(b)
    ref = torch.as_tensor(a.astype(np.float64) @ b.astype(np.float64).T, device=DEV)
    scale = torch.as_tensor(np.abs(a).astype(np.float64) @ np.abs(b).astype(np.float64).T, device=DEV)
    C = torch.empty(M, N, device=DEV)
    K.gemm(A, B, C, trans_b=True, tile=128 | X6)
    assert torch.isfinite(C).all()
    assert (((C.double() - ref).abs()) / scale).max().item() <= X6_ABS
    a2 = a.copy()
    a2[0, 0], a2[1, 1], a2[2, 2] = np.inf, -np.inf, np.nan
    b2 = np.abs(b) + 1e-31
    outs = []
    for flag in (X6, F32):
        C = torch.empty(M, N, device=DEV)
        K.gemm(_dev(a2), _dev(b2.astype(np.float32)), C, trans_b=True, tile=128 | flag)
        outs.append(C)
    assert torch.equal(torch.isfinite(outs[0]), torch.isfinite(outs[1]))
    fin = torch.isfinite(outs[1])
    sc2 = torch.as_tensor(np.abs(np.nan_to_num(a2, posinf=0, neginf=0)).astype(np.float64) @ b2.astype(np.float64).T,
                          device=DEV)
    assert ((outs[0] - outs[1]).double().abs()[fin] / sc2[fin]).max().item() <= 2 * X6_ABS


@pytest.mark.parametrize("nb", [1, 2, 4])
def test_spmm_row_classes_bit_exact(K, nb):
    """Lane plans with row classes (item rows scheduled before user rows,
    gmr_spmm_plan_build_split) give the one-class plan's sums bit for bit, with split sources and
    a hub row above the segment-split threshold."""
    rng = _rng(23)
    U, I = 12000, 400
    deg = rng.integers(0, 25, size=U)
    rows = np.repeat(np.arange(U), deg)
    p = 1.0 / np.arange(1, I + 1) ** 1.2
    cols = rng.choice(I, size=rows.size, p=p / p.sum())
    rp, col, val = graph_ref.norm_adj_csr(U, I, rows, cols)
    N = U + I
    saved = K.SPMM_CLASSES
    K.SPMM_CLASSES = True
    try:
        g0 = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=LANE32, class_split=0)
        g1 = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=LANE32, class_split=U)
    finally:
        K.SPMM_CLASSES = saved
    X = _dev(rng.standard_normal((N, 64 * nb)).astype(np.float32))
    E = _dev(rng.standard_normal((I, 64 * nb)).astype(np.float32))
    outs = []
    for g in (g0, g1):
        y = torch.empty((N, 64 * nb), device=DEV)
        g.spmm(y, [(X[:, 64 * b:64 * (b + 1)], E[:, 64 * b:64 * (b + 1)]) for b in range(nb)], split=U)
        outs.append(y)
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))


def _side_graph(self_loops, U=3000, I=500, seed=41):
    """Bipartite graph with Zipf hub items (rows far above the 64-entry task size), empty user and
    item rows, and optional self loops (a rebuilt UI graph)."""
    rng = _rng(seed)
    deg = rng.integers(0, 12, size=U)
    deg[::97] = 0
    rows = np.repeat(np.arange(U), deg)
    p = 1.0 / np.arange(1, I + 1) ** 1.1
    p[-20:] = 0.0  # items nobody picks: empty item rows
    cols = rng.choice(I, size=rows.size, p=p / p.sum())
    if self_loops:
        return graph_ref.ui_adj_csr(U, I, rows, cols)
    return graph_ref.norm_adj_csr(U, I, rows, cols)


@pytest.mark.parametrize("classes", [True, False])
@pytest.mark.parametrize("nb", [1, 2, 4])
@pytest.mark.parametrize("self_loops", [0, 1])
def test_spmm_side_vs_fp64_and_lane(K, nb, self_loops, classes):
    """Side-split plan (csrc/spmm_side.hip), degree-class (GMR_SIDE_CLASSES, the default) and task form:
    every row within fp32 tolerance of an fp64 product with split sources, alpha / beta; rows of degree
    <= T (16) bit-identical to the lane plan (both sum a short row's entries in CSR order from zero); hub
    rows (pieces added in order by the last arriving piece) identical across repeated launches (the
    counters re-arm) and with a second scratch."""
    rp, col, val = _side_graph(self_loops)
    U, I = 3000, 500
    N = U + I
    gs = K.CSR(_dev(rp), _dev(col), _dev(val), class_split=U, side=True)
    gs.build_side_plan(U, classes=classes)
    assert gs.side_classes == classes
    gl = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=LANE32)
    assert gs.side is not None and gl.side is None
    deg = np.diff(rp)
    assert deg.max() > 4 * 64 and (self_loops or (deg == 0).sum() > 20)
    rng = _rng(5)
    X = rng.standard_normal((N, 64 * nb)).astype(np.float32)
    E = rng.standard_normal((I, 64 * nb)).astype(np.float32)
    Y0 = rng.standard_normal((N, 64 * nb)).astype(np.float32)
    Xd, Ed = _dev(X), _dev(E)
    blocks = [(Xd[:, 64 * b:64 * (b + 1)], Ed[:, 64 * b:64 * (b + 1)]) for b in range(nb)]
    outs = []
    for g in (gs, gl, gs, gs):
        y = _dev(Y0)
        g.spmm(y, blocks, split=U, alpha=0.7, beta=0.3)
        outs.append(y)
    ys, yl = outs[0], outs[1]
    src = np.concatenate([X[:U], E]).astype(np.float64)
    a = np.zeros((N, N))
    a[np.repeat(np.arange(N), deg), col] = val
    want = 0.7 * (a @ src) + 0.3 * Y0
    scale = 0.7 * (np.abs(a) @ np.abs(src)) + 0.3 * np.abs(Y0) + 1e-6
    err = np.abs(ys.cpu().numpy() - want) / scale
    assert err.max() <= 1e-6, err.max()
    T = gs.side_hdr[3]  # the plan's short-row bound (H_T): longer rows are hub rows (wave blocks)
    short = torch.as_tensor(deg <= T, device=DEV)
    assert torch.equal(ys[short].view(torch.int32), yl[short].view(torch.int32))
    for y in outs[2:]:
        assert torch.equal(y.view(torch.int32), ys.view(torch.int32))
    # a second scratch (two products of one matrix on concurrent streams) gives the same bits
    y2 = _dev(Y0)
    gs.spmm(y2, blocks, split=U, alpha=0.7, beta=0.3, partial=torch.zeros_like(gs.partial))
    assert torch.equal(y2.view(torch.int32), ys.view(torch.int32))


@pytest.mark.parametrize("classes", [True, False])
def test_spmm_side_all_hub_rows_split_blocks(K, classes):
    """Every row a hub row: users of degree 17-40 (one wave block each)
    and item rows of degree ~400-550, split into 2-3 wave blocks of 8 TW = 256 entries whose partial sums
    meet through the relaxed agent-scope counter hand-off (csrc/spmm_side.hip, hub publish / last-block
    sum); d = 64 and d = 128.  The degree-class plan then holds no class rows (H_NSR = 0: the job
    loader's clamped loads land in the plan's zero pad).  Checked: fp64 within 1e-6, and bit-identical
    across four launches and with a second scratch (the counters re-arm, the block order is fixed)."""
    rng = _rng(47)
    U, I = 2000, 120
    N = U + I
    deg = rng.integers(17, 41, size=U)
    rows = np.repeat(np.arange(U), deg)
    cols = np.concatenate([rng.choice(I, size=d, replace=False) for d in deg])
    rp, col, val = graph_ref.norm_adj_csr(U, I, rows, cols)
    d_all = np.diff(rp)
    assert d_all.min() > 16 and d_all[U:].min() > 256  # every item row spans >= 2 wave blocks
    gs = K.CSR(_dev(rp), _dev(col), _dev(val), class_split=U, side=True)
    gs.build_side_plan(U, classes=classes)
    assert gs.side_hdr[24] == 0  # H_NSR: no short rows in the plan
    a = np.zeros((N, N))
    a[np.repeat(np.arange(N), d_all), col] = val
    for nb in (1, 2):
        X = rng.standard_normal((N, 64 * nb)).astype(np.float32)
        Xd = _dev(X)
        blocks = [(Xd[:, 64 * b:64 * (b + 1)],) for b in range(nb)]
        outs = []
        for _ in range(4):
            y = torch.empty((N, 64 * nb), device=DEV)
            gs.spmm(y, blocks)
            outs.append(y)
        want = a @ X.astype(np.float64)
        scale = np.abs(a) @ np.abs(X.astype(np.float64)) + 1e-6
        err = np.abs(outs[0].cpu().numpy() - want) / scale
        assert err.max() <= 1e-6, err.max()
        for y in outs[1:]:
            assert torch.equal(y.view(torch.int32), outs[0].view(torch.int32))
        y2 = torch.empty((N, 64 * nb), device=DEV)
        gs.spmm(y2, blocks, partial=torch.zeros_like(gs.partial))
        assert torch.equal(y2.view(torch.int32), outs[0].view(torch.int32))


@pytest.mark.parametrize("nb", [1, 2, 4])
def test_spmm_side_jobs_one_launch_bit_exact(K, nb):
    """gmr_spmm_side_jobs_f32 (round 5): up to four side-plan products of different graphs (a norm_adj-like
    graph, a rebuilt-UI-like graph with self loops, a second norm_adj) with split sources in ONE launch equal
    their separate launches bit for bit (own plans and hub scratches, the same XCD map), with beta too."""
    U, I = 3000, 500
    N = U + I
    graphs = []
    for seed, loops in ((41, 0), (42, 1), (43, 0)):
        rp, col, val = _side_graph(loops, seed=seed)
        g = K.CSR(_dev(rp), _dev(col), _dev(val), class_split=U, side=True)
        graphs.append(g)
    rng = _rng(9)
    X = _dev(rng.standard_normal((N, 64 * nb)).astype(np.float32))
    E = _dev(rng.standard_normal((I, 64 * nb)).astype(np.float32))
    Y0 = _dev(rng.standard_normal((N, 64 * nb)).astype(np.float32))
    blocks = [(X[:, 64 * b:64 * (b + 1)], E[:, 64 * b:64 * (b + 1)]) for b in range(nb)]
    for beta in (0.0, 0.5):
        sep = []
        for g in graphs:
            y = Y0.clone()
            g.spmm(y, blocks, split=U, alpha=0.9, beta=beta)
            sep.append(y)
        outs = [Y0.clone() for _ in graphs]
        assert K.SIDE_JOBS
        K.spmm_jobs([(g, o, blocks, U, None) for g, o in zip(graphs, outs)], alpha=0.9, beta=beta)
        for a, b in zip(sep, outs):
            assert torch.equal(a.view(torch.int32), b.view(torch.int32))


def test_spmm_side_multi_outputs_and_jobs(K):
    """spmm_multi / spmm_jobs on side plans: per-block outputs equal the one-output product, and a
    jobs launch mixing a side-plan matrix with a lane-plan one equals the separate calls."""
    rp, col, val = _side_graph(0, seed=43)
    U, I = 3000, 500
    N = U + I
    gs = K.CSR(_dev(rp), _dev(col), _dev(val), class_split=U, side=True)
    gl = K.CSR(_dev(rp), _dev(col), _dev(val), seg_nnz=LANE32)
    rng = _rng(6)
    X = _dev(rng.standard_normal((N, 256)).astype(np.float32))
    y_one = torch.empty((N, 256), device=DEV)
    gs.spmm(y_one, [(X[:, 64 * b:64 * (b + 1)],) for b in range(4)])
    outs = [torch.empty((N, 64), device=DEV) for _ in range(4)]
    K.spmm_multi(gs, outs, [(X[:, 64 * b:64 * (b + 1)],) for b in range(4)])
    for b in range(4):
        assert torch.equal(outs[b].view(torch.int32), y_one[:, 64 * b:64 * (b + 1)].view(torch.int32))
    ya, yb = torch.empty((N, 128), device=DEV), torch.empty((N, 128), device=DEV)
    K.spmm_jobs([(gs, ya, [(X[:, :64],), (X[:, 64:128],)], None, None),
                 (gl, yb, [(X[:, :64],), (X[:, 64:128],)], None, None)])
    ra, rb = torch.empty_like(ya), torch.empty_like(yb)
    gs.spmm(ra, [(X[:, :64],), (X[:, 64:128],)])
    gl.spmm(rb, [(X[:, :64],), (X[:, 64:128],)])
    assert torch.equal(ya.view(torch.int32), ra.view(torch.int32))
    assert torch.equal(yb.view(torch.int32), rb.view(torch.int32))



@pytest.mark.parametrize("tile", [0, 1 << 27, 1 << 26])
@pytest.mark.parametrize("M,N,Kd", [(300, 7050, 1000), (64, 130, 70), (2048, 1000, 1000)])
def test_gemm_scale_bias_equals_posterior_c2_zero(K, M, N, Kd, tile):
    """GMR_EPI_SCALE_BIAS (round 6; the last p_sample step) = GMR_EPI_POSTERIOR with c2 = 0 bit for bit, on the
    default plan, the fp32-input kernel and the split-bf16 kernel (split-K plans included), without reading aux:
    the SCALE_BIAS output buffer starts as NaN."""
    torch.manual_seed(7)
    A = torch.randn(M, Kd, device=DEV)
    B = torch.randn(N, Kd, device=DEV)
    bias = torch.randn(N, device=DEV)
    aux = (torch.rand(M, N, device=DEV) < 0.3).float()
    C1 = aux.clone()
    K.gemm(A, B, C1, trans_b=True, epi=K.EPI_POSTERIOR, bias=bias, aux=C1, slope=0.37, beta=0.0, tile=tile)
    C2 = torch.full((M, N), float("nan"), device=DEV)
    K.gemm(A, B, C2, trans_b=True, epi=K.EPI_SCALE_BIAS, bias=bias, slope=0.37, tile=tile)
    torch.cuda.synchronize()
    assert torch.isfinite(C2).all()
    assert torch.equal(C1, C2)
