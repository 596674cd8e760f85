"""Dump a baby/sports-shaped norm_adj (or rebuilt UI graph) CSR for scripts/micro/side_spmm.hip.

python scripts/micro/dump_graph.py baby norm_adj out.bin
File: int64 n_rows, split, nnz; int32 rowptr[n_rows+1], col[nnz]; float32 val[nnz].
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))
sys.path.insert(0, ROOT)

from gmr.synthetic import SHAPES, make_interactions  # noqa: E402


def csr(shape, kind):
    U, I, n, _, _ = SHAPES[shape]
    u, i, lb = make_interactions(U, I, n, seed=0)
    tr = lb == 0
    u, i = u[tr], i[tr]
    N = U + I
    if kind == "norm_adj":
        key = np.unique(u.astype(np.int64) * I + i)
        uu, ii = key // I, key % I
        r = np.concatenate([uu, ii + U])
        c = np.concatenate([ii + U, uu])
        deg = np.bincount(r, minlength=N).astype(np.float64) + 1e-7
    elif kind == "uniform":  # the same user degrees, items uniform (no popularity hubs)
        rng = np.random.default_rng(1)
        ii = rng.integers(0, I, len(i))
        key = np.unique(u.astype(np.int64) * I + ii)
        uu, ii = key // I, key % I
        r = np.concatenate([uu, ii + U])
        c = np.concatenate([ii + U, uu])
        deg = np.bincount(r, minlength=N).astype(np.float64) + 1e-7
    else:  # ui_top1: one random item per user + self loops
        rng = np.random.default_rng(0)
        it = rng.integers(0, I, U)
        loops = np.arange(N)
        r = np.concatenate([np.arange(U), it + U, loops])
        c = np.concatenate([it + U, np.arange(U), loops])
        deg = np.bincount(r, minlength=N).astype(np.float64)
    dis = deg ** -0.5
    v = (dis[r] * dis[c]).astype(np.float32)
    o = np.lexsort((c, r))
    r, c, v = r[o], c[o], v[o]
    rp = np.zeros(N + 1, np.int64)
    np.add.at(rp, r + 1, 1)
    return U, np.cumsum(rp).astype(np.int32), c.astype(np.int32), v


def main():
    shape, kind, out = sys.argv[1], sys.argv[2], sys.argv[3]
    U, rp, c, v = csr(shape, kind)
    with open(out, "wb") as f:
        np.array([len(rp) - 1, U, len(c)], np.int64).tofile(f)
        rp.tofile(f)
        c.tofile(f)
        v.tofile(f)
    deg = np.diff(rp)
    print(f"{shape} {kind}: n={len(rp) - 1} split={U} nnz={len(c)} max_deg user={deg[:U].max()} item={deg[U:].max()}")


if __name__ == "__main__":
    main()
