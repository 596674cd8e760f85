"""CSR restatements of the two normalised adjacency builders (TEST ORACLE ONLY).

Both builders produce the N x N (N = U + I) symmetric bipartite matrix
D^-1/2 A D^-1/2 in CSR with columns ascending inside each row, values computed
in float64 and rounded once to float32 (scipy computes the products in float64
and torch.FloatTensor rounds them, so this is bit-exact with the reference).
"""
import numpy as np


def _csr_from_pairs(n, r, c, v):
    order = np.lexsort((c, r))
    r, c, v = r[order], c[order], v[order]
    rowptr = np.zeros(n + 1, np.int64)
    np.add.at(rowptr, r + 1, 1)
    return np.cumsum(rowptr).astype(np.int32), c.astype(np.int32), v


def norm_adj_csr(n_users, n_items, rows, cols):
    """DiffMM.get_norm_adj_mat — reference models/diffmm.py:88-107.

    A = [[0, R], [R^T, 0]] with binary entries (duplicate interactions collapse,
    :92-96), deg = row count of A>0 plus 1e-7 (:97-98), L = D^-1/2 A D^-1/2 (:99-101).
    """
    n = n_users + n_items
    key = np.unique(rows.astype(np.int64) * n_items + cols.astype(np.int64))
    u, i = key // n_items, key % n_items
    r = np.concatenate([u, i + n_users])
    c = np.concatenate([i + n_users, u])
    deg = np.bincount(r, minlength=n).astype(np.float64) + 1e-7
    dis = np.power(deg, -0.5)
    v = (dis[r] * dis[c]).astype(np.float32)
    return _csr_from_pairs(n, r, c, v)


def ui_adj_csr(n_users, n_items, users, items):
    """DiffMMTrainer.buildUIMatrix + normalizeAdj — reference common/trainer.py:464-485.

    Bipartite edges from (user, item) pairs (binarised, :476), plus self loops on
    all N nodes (:478), deg = row sum of (A + I) (:465), values deg_r^-1/2 deg_c^-1/2.
    """
    n = n_users + n_items
    key = np.unique(np.asarray(users, np.int64) * n_items + np.asarray(items, np.int64))
    u, i = key // n_items, key % n_items
    loops = np.arange(n, dtype=np.int64)
    r = np.concatenate([u, i + n_users, loops])
    c = np.concatenate([i + n_users, u, loops])
    deg = np.bincount(r, minlength=n).astype(np.float64)
    dis = np.power(deg, -0.5)
    dis[np.isinf(dis)] = 0.0
    v = (dis[c] * dis[r]).astype(np.float32)
    return _csr_from_pairs(n, r, c, v)


def csr_to_dense(rowptr, col, val, n_cols=None):
    n = len(rowptr) - 1
    m = np.zeros((n, n if n_cols is None else n_cols), np.float32)
    for r in range(n):
        s, e = rowptr[r], rowptr[r + 1]
        m[r, col[s:e]] = val[s:e]
    return m


def coo_to_csr(n, idx, val):
    """Sorted CSR of a reference COO (indices 2 x nnz)."""
    return _csr_from_pairs(n, idx[0].astype(np.int64), idx[1].astype(np.int64), val)
