"""Full-rank top-K selection and ranking metrics (TEST ORACLE ONLY).

Top-K order is defined as: score descending, ties -> lowest item index.  The
reference calls torch.topk (common/trainer.py:386), whose tie order on CPU is
implementation-defined; parity with it is checked per tie group as sets.
Metric formulas restate utils/metrics.py:12-105 (float64), the 4-decimal
rounding of utils/topk_evaluator.py:120 is applied by ``round4``.
"""
import numpy as np


def topk_rows(scores, k):
    """Per-row top-k indices, score desc / index asc."""
    s = np.asarray(scores, np.float32)
    n, m = s.shape
    out = np.empty((n, k), np.int64)
    idx = np.arange(m)
    for r in range(n):
        order = np.lexsort((idx, -s[r].astype(np.float64)))
        out[r] = order[:k]
    return out


def mask_scores(scores, mask_rows, mask_cols, fill=-1e10):
    """scores[mask] = -1e10 — common/trainer.py:383-384."""
    s = np.array(scores, np.float32, copy=True)
    s[np.asarray(mask_rows), np.asarray(mask_cols)] = np.float32(fill)
    return s


def hit_matrix(topk, pos_lists):
    """bool_rec_matrix — utils/topk_evaluator.py:109-112."""
    return np.asarray([[int(i) in set(np.asarray(m).tolist()) for i in row] for m, row in zip(pos_lists, topk)],
                      dtype=bool).reshape(len(pos_lists), -1)


def metric_curves(hits, pos_len):
    """recall_/ndcg_/precision_/map_ — utils/metrics.py:12-105. Returns dict metric -> array over k=1..K."""
    hits = np.asarray(hits, bool)
    pos_len = np.asarray(pos_len, np.int64)
    n, K = hits.shape
    ranks = np.arange(1, K + 1, dtype=np.float64)
    cum = np.cumsum(hits, axis=1)
    recall = (cum / pos_len[:, None]).mean(0)
    precision = (cum / ranks).mean(0)
    disc = 1.0 / np.log2(ranks + 1)
    dcg = np.cumsum(np.where(hits, disc, 0.0), axis=1)
    ilen = np.minimum(pos_len, K)
    idcg_full = np.cumsum(disc)
    idcg = np.where(ranks[None, :] <= ilen[:, None], idcg_full[None, :], idcg_full[ilen - 1][:, None])
    ndcg = (dcg / idcg).mean(0)
    sum_pre = np.cumsum((cum / ranks) * hits, axis=1)
    denom = np.minimum(np.broadcast_to(ranks, hits.shape), ilen[:, None].astype(np.float64))
    mapk = (sum_pre / denom).mean(0)
    return {"recall": recall, "ndcg": ndcg, "precision": precision, "map": mapk}


def metric_dict(curves, ks=(5, 10, 20, 50), metrics=("recall", "ndcg", "precision", "map"), rounded=True):
    out = {}
    for m in metrics:
        for k in ks:
            v = float(curves[m][k - 1])
            out[f"{m}@{k}"] = round(v, 4) if rounded else v
    return out
