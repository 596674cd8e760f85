"""Fused eval kernel (gmr_score_topk_f32 / gmr_score_topk_x6): scores = U[users] . I^T -> train positives set to -1e10 ->
top-k (score desc, ties -> lowest index), the reference's common/trainer.py:379-386 with
models/diffmm.py:276-277, without the E x I score matrix.

Exactness is checked on integer-valued embeddings (every dot product is exact in fp32, so the
expected top-k is known exactly and ties are everywhere: the tie-breaking and the select-among-equal
path of the candidate compaction are exercised); real-valued embeddings are checked against the
unfused GEMM + mask + radix top-k path with an fp64 tolerance for near ties."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, params=[False, True], ids=["fp32", "x6"])
def scoring(request, monkeypatch):
    """Every test on both score forms: fp32 MFMA (gmr_score_topk_f32, the default) and, for d = 64, the
    split-bf16 MFMA from item planes (gmr_score_topk_x6, GMR_EVAL_X6=1)."""
    from gmr import kernels as K
    monkeypatch.setattr(K, "EVAL_X6", request.param)
    return request.param


def _mask(rng, n_rows, n_items, max_len, full_row=None):
    rows = []
    for r in range(n_rows):
        m = int(rng.integers(0, max_len + 1))
        if full_row is not None and r == full_row:
            m = n_items - 10  # only 10 unmasked items: masked -1e10 entries reach the top-k
        rows.append(np.sort(rng.choice(n_items, size=min(m, n_items), replace=False)).astype(np.int32))
    ptr = np.concatenate([[0], np.cumsum([len(x) for x in rows])]).astype(np.int64)
    cols = np.concatenate(rows) if rows else np.zeros(0, np.int32)
    return rows, ptr, cols


def _expected(scores, rows, k, fill=-1e10):
    s = scores.astype(np.float64).copy()
    out = np.empty((s.shape[0], k), np.int64)
    for r in range(s.shape[0]):
        s[r, rows[r]] = fill
        order = np.lexsort((np.arange(s.shape[1]), -s[r]))  # score desc, then index asc
        out[r] = order[:k]
    return out, s


def _run(U, I, users, ptr, cols, k, want_val=False, fill=-1e10):
    from gmr import kernels as K
    n = len(users) if users is not None else U.shape[0]
    out = torch.full((n, k), -7, dtype=torch.int32, device=DEV)
    val = torch.zeros((n, k), dtype=torch.float32, device=DEV) if want_val else None
    ut = torch.as_tensor(users, dtype=torch.int32, device=DEV) if users is not None else None
    K.score_topk(torch.as_tensor(U, device=DEV), torch.as_tensor(I, device=DEV), ut,
                 torch.as_tensor(ptr, device=DEV), torch.as_tensor(cols, device=DEV), k, out, val, fill=fill)
    torch.cuda.synchronize()
    return out.cpu().numpy(), (val.cpu().numpy() if want_val else None)


@pytest.mark.parametrize("D,n_items,k,n_rows", [(64, 1000, 50, 301), (64, 7050, 50, 70), (128, 999, 20, 33),
                                                (64, 37, 20, 17), (64, 64, 64, 16), (64, 3000, 1, 50),
                                                (128, 130, 64, 5)])
def test_integer_embeddings_exact(D, n_items, k, n_rows):
    rng = np.random.default_rng(D + n_items + k)
    n_users = 400
    U = rng.integers(-3, 4, size=(n_users, D)).astype(np.float32)  # small ints: exact fp32 dots, many ties
    I = rng.integers(-3, 4, size=(n_items, D)).astype(np.float32)
    users = rng.integers(0, n_users, size=n_rows).astype(np.int32)
    users[: min(3, n_rows)] = users[0]  # duplicate users in one launch
    rows, ptr, cols = _mask(rng, n_rows, n_items, min(40, n_items - k), full_row=1 if n_items > 20 else None)
    want, s = _expected(U[users].astype(np.int64) @ I.T.astype(np.int64), rows, k)
    got, val = _run(U, I, users, ptr, cols, k, want_val=True)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(val, np.take_along_axis(s, want, 1).astype(np.float32))


@pytest.mark.parametrize("D,n_items,k", [(64, 1000, 50), (128, 300, 64), (64, 7050, 50)])
def test_minus_inf_fill_with_rows_short_of_k(D, n_items, k):
    """fill = -inf (torch's usual masking value): masked items score -inf and must still reach
    the top-k of a row that has fewer than k unmasked items (row 1: n_items - 10 masked), ties among them
    to the lowest index, with every returned index valid and the value -inf."""
    rng = np.random.default_rng(D + n_items)
    n_rows = 37
    U = rng.integers(-3, 4, size=(n_rows, D)).astype(np.float32)
    I = rng.integers(-3, 4, size=(n_items, D)).astype(np.float32)
    rows, ptr, cols = _mask(rng, n_rows, n_items, min(40, n_items - k), full_row=1)
    rows[3] = np.arange(n_items, dtype=np.int32)  # a row with every item masked
    ptr = np.concatenate([[0], np.cumsum([len(x) for x in rows])]).astype(np.int64)
    cols = np.concatenate(rows).astype(np.int32)
    want, s = _expected(U.astype(np.int64) @ I.T.astype(np.int64), rows, k, fill=-np.inf)
    got, val = _run(U, I, None, ptr, cols, k, want_val=True, fill=float("-inf"))
    assert got.min() >= 0 and got.max() < n_items
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(val, np.take_along_axis(s, want, 1).astype(np.float32))
    assert np.isneginf(val[1, 10:]).all() and np.isneginf(val[3]).all()


def test_users_none_and_empty_masks():
    rng = np.random.default_rng(5)
    U = rng.integers(-2, 3, size=(45, 64)).astype(np.float32)
    I = rng.integers(-2, 3, size=(500, 64)).astype(np.float32)
    ptr = np.zeros(46, np.int64)
    cols = np.zeros(1, np.int32)
    want, _ = _expected(U.astype(np.int64) @ I.T.astype(np.int64), [np.zeros(0, np.int64)] * 45, 50)
    got, _ = _run(U, I, None, ptr, cols, 50)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("D,n_items,k", [(64, 5000, 50), (128, 3001, 64), (64, 700, 1)])
def test_all_scores_tied(D, n_items, k):
    """Zero embeddings: every item scores 0, so every tile fills the candidate buffer with ties and
    the compaction must keep the lowest indices (masked items excluded)."""
    rng = np.random.default_rng(D + k)
    n_rows = 40
    U = np.zeros((n_rows, D), np.float32)
    I = np.zeros((n_items, D), np.float32)
    rows, ptr, cols = _mask(rng, n_rows, n_items, 60)
    want, _ = _expected(np.zeros((n_rows, n_items)), rows, k)
    got, val = _run(U, I, None, ptr, cols, k, want_val=True)
    np.testing.assert_array_equal(got, want)
    assert (val == 0).all()


@pytest.mark.parametrize("D,sign", [(64, 1), (64, -1), (128, 1)])
def test_monotone_scores(D, sign):
    """Scores strictly increasing (sign 1: every tile beats the running top-k, the most compactions)
    or decreasing (sign -1: the threshold rejects everything after the first tiles) with item index."""
    rng = np.random.default_rng(D)
    n_rows, n_items, k = 24, 6000, 50
    U = np.zeros((n_rows, D), np.float32)
    U[:, 0] = sign * (1 + np.arange(n_rows))  # integer-valued: exact fp32 dots
    I = np.zeros((n_items, D), np.float32)
    I[:, 0] = np.arange(n_items)
    rows, ptr, cols = _mask(rng, n_rows, n_items, 30)
    want, s = _expected(U.astype(np.int64) @ I.T.astype(np.int64), rows, k)
    got, val = _run(U, I, None, ptr, cols, k, want_val=True)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(val, np.take_along_axis(s, want, 1).astype(np.float32))


def test_zero_rows_is_a_no_op():
    from gmr import kernels as K
    out = torch.full((1, 20), -7, dtype=torch.int32, device=DEV)
    K.score_topk(torch.zeros((4, 64), device=DEV), torch.zeros((100, 64), device=DEV),
                 torch.zeros(0, dtype=torch.int32, device=DEV), torch.zeros(1, dtype=torch.int64, device=DEV),
                 torch.zeros(1, dtype=torch.int32, device=DEV), 20, out)
    torch.cuda.synchronize()
    assert (out.cpu() == -7).all()


def test_float_embeddings_vs_unfused_path():
    """Real-valued embeddings: the fused result equals the unfused GEMM + mask + radix top-k wherever
    the fp64 scores are not within 1e-6 (relative) of a tie, and every differing row holds a pair within 16
    ulp of the row's |u|.|i| (an fp32-rounding tie) among its swapped items AND among its fp64 top-(k + 1)
    (no row without such a tie may differ; replaces round 4's fixed >= 99.8 % bar)."""
    from gmr import kernels as K
    rng = np.random.default_rng(11)
    n_users, n_items, k, n_rows = 2000, 7050, 50, 1500
    U = (rng.standard_normal((n_users, 64)) * 0.1).astype(np.float32)
    I = (rng.standard_normal((n_items, 64)) * 0.1).astype(np.float32)
    users = rng.integers(0, n_users, size=n_rows).astype(np.int32)
    rows, ptr, cols = _mask(rng, n_rows, n_items, 30)
    got, _ = _run(U, I, users, ptr, cols, k)
    # unfused path on the same device tensors
    ut = torch.as_tensor(users, device=DEV)
    ub = torch.empty((n_rows, 64), device=DEV)
    K.gather_rows(torch.as_tensor(U, device=DEV), ut, ub)
    sc = torch.empty((n_rows, n_items), device=DEV)
    K.gemm(ub, torch.as_tensor(I, device=DEV), sc, trans_b=True)
    mr = torch.as_tensor(np.repeat(np.arange(n_rows), np.diff(ptr)).astype(np.int32), device=DEV)
    K.mask_scores(sc, mr, torch.as_tensor(cols, device=DEV))
    ref = torch.empty((n_rows, k), dtype=torch.int32, device=DEV)
    K.topk_rows(sc, k, ref)
    ref = ref.cpu().numpy()
    s64 = U[users].astype(np.float64) @ I.T.astype(np.float64)
    for r in range(n_rows):
        s64[r, rows[r]] = -1e10
    same = (got == ref).all(axis=1)
    # fp32 rounding scale of a 64-term dot product: both kernels' scores lie within a few ulps of
    # |u|.|i|; two items closer than that in fp64 are a tie either fp32 kernel may break either way
    mag = np.abs(U[users]).astype(np.float64) @ np.abs(I.T).astype(np.float64)
    for r in np.nonzero(~same)[0]:  # any difference must be a near tie in fp64 (1e-6 relative)
        a, b = s64[r, got[r]], s64[r, ref[r]]
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-9, err_msg=f"row {r}")
        assert np.abs(np.sort(a) - np.sort(b)).max() <= 1e-6 * np.abs(a).max()
        # and the tie is at fp32 rounding scale: some swapped pair differs by <= 16 ulp of the row's |u|.|i|
        d = np.setxor1d(got[r], ref[r]) if set(got[r]) != set(ref[r]) else got[r][got[r] != ref[r]]
        gap = np.abs(s64[r, d][:, None] - s64[r, d][None, :]) + np.eye(len(d)) * 1e30
        assert gap.min() <= 16 * 2.0 ** -24 * mag[r].max(), (r, gap.min(), mag[r].max())
    n_diff = int((~same).sum())
    # the rows where a difference is possible at all: some pair among the row's fp64 top-(k + 1) lies within
    # the 16-ulp fp32 rounding window (a tie either fp32 kernel may break either way); a differing row must be
    # one of them (a principled bound in place of a fixed percentage: no row without such a tie may differ)
    top = np.argsort(-s64, axis=1, kind="stable")[:, :k + 1]
    ts = np.take_along_axis(s64, top, 1)
    eligible = (np.abs(np.diff(ts, axis=1)) <= 16 * 2.0 ** -24 * mag.max(axis=1, keepdims=True)).any(axis=1)
    print(f"fused vs unfused: {n_diff} of {n_rows} rows differ; {int(eligible.sum())} rows hold an fp32-scale tie")
    assert eligible[~same].all(), np.nonzero(~same & ~eligible)[0]
    assert n_diff <= int(eligible.sum())
    # and every row is sorted by fp64 score up to the same tolerance
    g64 = np.take_along_axis(s64, got.astype(np.int64), 1)
    assert (np.diff(g64, axis=1) <= 1e-6 * np.abs(g64[:, :1])).all()


def test_bad_arguments_raise():
    from gmr import kernels as K
    U = torch.zeros((4, 64), device=DEV)
    I = torch.zeros((10, 64), device=DEV)
    out = torch.zeros((4, 20), dtype=torch.int32, device=DEV)
    ptr = torch.zeros(5, dtype=torch.int64, device=DEV)
    cols = torch.zeros(1, dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError):
        K.score_topk(U, I, None, ptr, cols, 20, out)  # k > n_items
    with pytest.raises(RuntimeError):
        K.score_topk(torch.zeros((4, 32), device=DEV), torch.zeros((10, 32), device=DEV), None, ptr, cols, 5, out)
