"""Device K-means for the GenRecV1 interest clusters — common/interest_cluster.py:60-79 of the
reference (sklearn StandardScaler + KMeans(n_clusters=k).fit(...).labels_).

StandardScaler (population std, zero std -> 1), greedy k-means++ seeding (sklearn's default: 2 + ln k
candidates per center, Philox draws, the one of the lowest potential kept), then Lloyd iterations until no
label changes (or max_iter): the point-centroid
dot products and the centroid sums (one-hot^T X) are MFMA GEMMs, the argmin / update steps are
small kernels (gengraph.hip).  Init-time only; the reference's own clustering is unseeded, so
parity is on the partition (tests: planted clusters recovered up to a label permutation).
"""
import math

import torch

from . import _lib
from . import kernels as K
from .kernels import ptr, stream


def kmeans_labels(X, k, seed=0, max_iter=300):
    """X: n x d fp32 device tensor; returns int32 labels (n,) on the device."""
    n, d = X.shape
    dev = X.device
    if not (1 <= k <= 64):
        raise ValueError("k must be 1..64 (the debias kernel keeps per-row cluster counts in 64 slots)")
    ld = (d + 3) // 4 * 4
    Y = torch.empty((n, ld), dtype=torch.float32, device=dev)[:, :d]
    mean = torch.empty(d, dtype=torch.float32, device=dev)
    scale = torch.empty(d, dtype=torch.float32, device=dev)
    xsq = torch.empty(n, dtype=torch.float32, device=dev)
    _lib.call("gmr_kmeans_standardize", n, d, ptr(X), K._ld(X), ptr(mean), ptr(scale), ptr(Y), ld, ptr(xsq), stream())
    C = torch.zeros((k, ld), dtype=torch.float32, device=dev)[:, :d]
    csq = torch.zeros(k, dtype=torch.float32, device=dev)
    pick = torch.zeros(1, dtype=torch.int32, device=dev)
    mind = torch.empty(n, dtype=torch.float32, device=dev)
    dots = torch.empty((n, 4), dtype=torch.float32, device=dev)[:, :1]
    # greedy k-means++ seeding (sklearn KMeans' default: the first center uniform, then per center L = 2 +
    # floor(ln k) candidates drawn with probability mind / sum, the one of the lowest potential kept)
    L = 2 + int(math.log(k))
    cand = torch.zeros(L, dtype=torch.int32, device=dev)
    Cc = torch.zeros((L, ld), dtype=torch.float32, device=dev)[:, :d]
    ccsq = torch.zeros(L, dtype=torch.float32, device=dev)
    dots_c = torch.empty((n, (L + 3) // 4 * 4), dtype=torch.float32, device=dev)[:, :L]
    _lib.call("gmr_kmeans_pp_pick", n, None, seed, 0, ptr(pick), stream())
    _lib.call("gmr_kmeans_take_center", d, ptr(Y), ld, ptr(pick), ptr(C), ld, 0, ptr(xsq), ptr(csq), stream())
    K.gemm(Y, C[0:1], dots, trans_b=True)
    _lib.call("gmr_kmeans_min_dist", n, ptr(xsq), ptr(dots), K._ld(dots), ptr(csq), 0, ptr(mind), 1, stream())
    for j in range(1, k):
        for t in range(L):
            _lib.call("gmr_kmeans_pp_pick", n, ptr(mind), seed, 1024 + 16 * j + t, ptr(cand[t:t + 1]), stream())
            _lib.call("gmr_kmeans_take_center", d, ptr(Y), ld, ptr(cand[t:t + 1]), ptr(Cc), ld, t, ptr(xsq), ptr(ccsq),
                      stream())
        K.gemm(Y, Cc, dots_c, trans_b=True)
        _lib.call("gmr_kmeans_pp_greedy", n, L, ptr(xsq), ptr(dots_c), K._ld(dots_c), ptr(ccsq), ptr(mind), ptr(Cc), ld,
                  d, ptr(C), ld, j, ptr(csq), stream())
    # Lloyd
    kp = (k + 3) // 4 * 4
    D2 = torch.empty((n, kp), dtype=torch.float32, device=dev)[:, :k]
    labels = torch.full((n,), -1, dtype=torch.int32, device=dev)
    np4 = (n + 3) // 4 * 4
    OH = torch.empty((k, np4), dtype=torch.float32, device=dev)[:, :n]
    sums = torch.empty((k, ld), dtype=torch.float32, device=dev)[:, :d]
    changed = torch.zeros(1, dtype=torch.int32, device=dev)
    parts = torch.empty(int(_lib.load().gmr_kmeans_parts(n)), dtype=torch.float64, device=dev)
    for it in range(max_iter):
        K.gemm(Y, C, D2, trans_b=True)
        K.zero_(changed)
        _lib.call("gmr_kmeans_assign", n, k, ptr(D2), K._ld(D2), ptr(csq), ptr(xsq), ptr(labels), ptr(OH), np4,
                  ptr(changed), ptr(parts), stream())
        K.gemm(OH, Y, sums)
        _lib.call("gmr_kmeans_centroids", k, d, ptr(sums), ld, ptr(OH), np4, n, ptr(C), ld, ptr(csq), stream())
        if int(changed.item()) == 0:
            break
    return labels
