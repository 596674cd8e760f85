"""Top-K evaluator — mirrors utils/topk_evaluator.py + utils/metrics.py of the reference.

Recall/NDCG/Precision/MAP@k for the full eval split are computed on the device
(gmr_eval_metrics: per-user hit test against sorted positives + fp64 sums), then averaged and
rounded to 4 decimals (topk_evaluator.py:114-120).  The test-only extras (topk_evaluator.py:122-270)
run on the device too: Pop/Niche are the same sums against each user's popular / niche positives
over the users holding any (gmr_eval_metrics_sel), Cold/Warm the sums over the user groups, and
Coverage/Gini/Tail% come from per-item recommendation counts (gmr_topk_item_counts); the host
only turns those few numbers into the rounded dict.  The group tables (per-user popular and niche
positives, cold/warm rows) are built once per eval split.  `evaluate` keeps the reference's host
path (and its top-K CSV dump, :93-106) for callers holding batch lists.
"""
import os
from collections import Counter

import numpy as np
import pandas as pd
import torch

from . import _lib
from . import kernels as K
from .utils import get_local_time

_NAMES = {m.lower(): m for m in ["Recall", "Recall2", "Precision", "NDCG", "MAP"]}
_DEVICE_METRICS = ["recall", "ndcg", "precision", "map"]


def _trapz(y, x):
    f = getattr(np, "trapezoid", None) or getattr(np, "trapz")
    return f(y, x=x)


def cal_gini(d_counter):
    cum = np.cumsum(sorted(np.append(d_counter, 0)))
    s = cum[-1]
    x = np.arange(len(cum)) / (len(cum) - 1)
    B = _trapz(cum / s, x)
    A = 0.5 - B
    return A / (A + B)


def metric_curves(hits, pos_len):
    """Host metric curves over k = 1..K (utils/metrics.py:12-105), used for subgroup metrics."""
    hits = np.asarray(hits, bool)
    pos_len = np.asarray(pos_len, np.int64)
    n, Kk = hits.shape
    ranks = np.arange(1, Kk + 1, dtype=np.float64)
    cum = np.cumsum(hits, 1)
    disc = 1.0 / np.log2(ranks + 1)
    ilen = np.minimum(pos_len, Kk)
    idcg_full = np.cumsum(disc)
    idcg = np.where(ranks[None] <= ilen[:, None], idcg_full[None], idcg_full[ilen - 1][:, None])
    prec = cum / ranks
    return {"recall": (cum / pos_len[:, None]).mean(0),
            "recall2": cum.sum(0) / pos_len.sum(),
            "ndcg": (np.cumsum(np.where(hits, disc, 0.0), 1) / idcg).mean(0),
            "precision": prec.mean(0),
            "map": (np.cumsum(prec * hits, 1) / np.minimum(ranks[None], ilen[:, None])).mean(0)}


class TopKEvaluator:
    def __init__(self, config):
        self.config = config
        self.metrics = config["metrics"]
        self.topk = config["topk"]
        self.save_recom_result = config["save_recommended_topk"]
        self.pop_items = config["pop_items"] if "pop_items" in config else None
        self.warm_users = config["warm_users"] if "warm_users" in config else None
        self.pop_mask = None
        self._check_args()
        self._dev = {}

    def _check_args(self):
        if isinstance(self.metrics, str):
            self.metrics = [self.metrics]
        for m in self.metrics:
            if m.lower() not in _NAMES:
                raise ValueError(f"There is no user grouped topk metric named {m}!")
        self.metrics = [m.lower() for m in self.metrics]
        if isinstance(self.topk, int):
            self.topk = [self.topk]
        if any(k <= 0 for k in self.topk):
            raise ValueError("topk must be a positive integer or a list of positive integers")

    # ------------------------------------------------------------------ device path
    def device_sums(self, topk_dev, eval_data):
        """fp64 sums of recall/ndcg/precision/map at self.topk over all eval users (device)."""
        d = eval_data.to_device()
        dev = topk_dev.device
        n = topk_dev.shape[0]
        key = (n, dev)
        if key not in self._dev:
            self._dev[key] = (torch.empty(int(_lib.load().gmr_eval_metrics_partials(n)), dtype=torch.float64,
                                          device=dev),
                              torch.empty(32, dtype=torch.float64, device=dev),
                              torch.as_tensor(np.asarray(sorted(self.topk), np.int32)).to(dev))
        parts, sums, ks = self._dev[key]
        K.eval_metrics(topk_dev, d["pos_ptr"], d["pos_items"], ks, parts, sums)
        return sums

    def evaluate_device(self, topk_dev, eval_data, is_test=False, idx=0, sums=None, n_users=None):
        n = n_users if n_users is not None else topk_dev.shape[0]
        if sums is None:
            sums = self.device_sums(topk_dev, eval_data)
        s = sums.cpu().numpy().reshape(4, 8)
        ks = sorted(self.topk)
        out = {}
        for m in self.metrics:
            for k in self.topk:
                if m in _DEVICE_METRICS:
                    v = s[_DEVICE_METRICS.index(m), ks.index(k)] / n
                else:  # recall2 needs the global positive count
                    v = None
                out[f"{m}@{k}"] = round(float(v), 4) if v is not None else None
        if is_test:
            out.update(self.extras_device(topk_dev, eval_data, n))
            if self.save_recom_result:
                self._dump(topk_dev[:n].cpu().numpy(), eval_data, idx)
        if any(v is None for v in out.values()):  # recall2 (global positive count): host path
            host = self.evaluate([topk_dev[:n]], eval_data, is_test=False, idx=idx)
            for k2, v in host.items():
                if out.get(k2) is None:
                    out[k2] = v
        return out

    # ------------------------------------------------------------------ test-time extras on the device
    def _groups(self, eval_data, dev):
        """Per eval split, once: sorted popular / niche positives per user and the user rows of the
        Pop / Niche / Cold / Warm groups (topk_evaluator.py:122-200)."""
        key = (id(eval_data), dev)
        cache = getattr(self, "_grp", None)
        if cache is not None and cache[0] == key:
            return cache[1]
        n = len(eval_data.eval_u_np)
        lens = np.asarray(eval_data.get_eval_len_list(), np.int64)
        items = np.concatenate([np.sort(x) for x in eval_data.get_eval_items()]) if n else np.zeros(0, np.int64)
        rows = np.repeat(np.arange(n), lens)
        g = {}
        t = lambda a, dt=np.int32: torch.as_tensor(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
        if self.pop_items is not None:
            pop = np.isin(items, np.fromiter(self.pop_items, np.int64, len(self.pop_items)))
            for name, msk in (("Pop", pop), ("Niche", ~pop)):
                cnt = np.bincount(rows[msk], minlength=n)
                ptr = np.concatenate([[0], np.cumsum(cnt)])
                sel = np.nonzero(cnt > 0)[0]
                if len(sel):
                    g[name] = (t(sel), t(ptr, np.int64), t(items[msk]), len(sel))
        if self.warm_users is not None:
            warm = np.isin(eval_data.eval_u_np, np.fromiter(self.warm_users, np.int64, len(self.warm_users)))
            d = eval_data.to_device()
            for name, msk in (("Cold", ~warm), ("Warm", warm)):
                sel = np.nonzero(msk)[0]
                if len(sel):
                    g[name] = (t(sel), d["pos_ptr"], d["pos_items"], len(sel))
        self._grp = (key, g)
        return g

    def extras_device(self, topk_dev, eval_data, n):
        dev = topk_dev.device
        ks = sorted(self.topk)
        kt = torch.as_tensor(np.asarray(ks, np.int32)).to(dev)
        out = {}
        for name, (sel, ptr_, items_, m) in self._groups(eval_data, dev).items():
            parts = torch.empty(int(_lib.load().gmr_eval_metrics_partials(m)), dtype=torch.float64, device=dev)
            sums = torch.empty(32, dtype=torch.float64, device=dev)
            _lib.call("gmr_eval_metrics_sel", m, K.ptr(sel), K.ptr(topk_dev), K._ld(topk_dev), topk_dev.shape[1],
                      K.ptr(ptr_), K.ptr(items_), len(ks), K.ptr(kt), K.ptr(parts), K.ptr(sums), K.stream())
            s = sums.cpu().numpy().reshape(4, 8) / m
            for mname in self.metrics:
                if mname in _DEVICE_METRICS:
                    for k in self.topk:
                        out[f"{name}_{_NAMES.get(mname, mname)}@{k}"] = round(float(s[_DEVICE_METRICS.index(mname),
                                                                                       ks.index(k)]), 4)
        item_num = eval_data.dataset.item_num
        counts = torch.empty((len(ks), item_num), dtype=torch.int32, device=dev)
        _lib.call("gmr_topk_item_counts", n, K.ptr(topk_dev), K._ld(topk_dev), len(ks), K.ptr(kt), item_num,
                  K.ptr(counts), K.stream())
        cnts = counts.cpu().numpy().astype(np.int64)
        if self.pop_items is not None and self.pop_mask is None:
            self.pop_mask = np.zeros(item_num, bool)
            self.pop_mask[[i for i in self.pop_items if i < item_num]] = True
        for j, k in enumerate(ks):
            out.update(self._diversity(cnts[j], k, n, item_num))
        return out

    def _diversity(self, cnt, k, n_users, item_num):
        """Coverage / Gini / Gini2 / Coverage2 / Tail% at k from the per-item counts (topk_evaluator.py:222-270)."""
        out = {f"Coverage@{k}": round(np.count_nonzero(cnt) / item_num, 4)}
        srt = np.sort(cnt)
        tot = srt.sum()
        if tot > 0:
            nn = item_num
            out[f"Gini@{k}"] = round(float((2 * np.sum(np.arange(1, nn + 1) * srt)) / (nn * tot) - (nn + 1) / nn), 4)
        else:
            out[f"Gini@{k}"] = 0.0
        nz = cnt[cnt > 0]
        if len(nz):
            out[f"Gini2@{k}"] = round(float(cal_gini(nz)), 4)
            out[f"Coverage2@{k}"] = round(len(nz) / item_num, 4)
        else:
            out[f"Gini2@{k}"] = 0.0
            out[f"Coverage2@{k}"] = 0.0
        if self.pop_mask is not None:
            out[f"Tail%@{k}"] = round(float(cnt[~self.pop_mask].sum() / (n_users * k)), 4)
        return out

    # ------------------------------------------------------------------ reference-style host path
    def evaluate(self, batch_matrix_list, eval_data, is_test=False, idx=0):
        pos_items = eval_data.get_eval_items()
        pos_len = np.asarray(eval_data.get_eval_len_list())
        topk_index = torch.cat([b.long() for b in batch_matrix_list], 0).cpu().numpy()
        if self.save_recom_result and is_test:
            self._dump(topk_index, eval_data, idx)
        assert len(pos_len) == len(topk_index)
        hits = self._hits(topk_index, pos_items)
        out = {}
        curves = metric_curves(hits, pos_len)
        for m in self.metrics:
            for k in self.topk:
                out[f"{m}@{k}"] = round(float(curves[m][k - 1]), 4)
        if is_test:
            out.update(self._extras(topk_index, pos_items, pos_len, hits, eval_data))
        return out

    @staticmethod
    def _hits(topk_index, pos_items):
        n, Kk = topk_index.shape
        lens = np.array([len(p) for p in pos_items])
        rows = np.repeat(np.arange(n), lens)
        flat = np.concatenate(pos_items) if len(pos_items) else np.zeros(0, np.int64)
        width = int(max(topk_index.max(initial=0), flat.max(initial=0))) + 1
        keys = np.unique(rows.astype(np.int64) * width + flat)
        q = np.repeat(np.arange(n), Kk).astype(np.int64) * width + topk_index.reshape(-1)
        return np.isin(q, keys).reshape(n, Kk)

    def _dump(self, topk_index, eval_data, idx):
        from . import dist
        if dist.rank() != 0:  # every rank holds the gathered top-k: one writer
            return
        k = max(self.topk)
        d = os.path.abspath(self.config["recommend_topk"] or "recommend_topk/")
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "{}-{}-idx{}-top{}-{}.csv".format(self.config["model"], self.config["dataset"], idx, k,
                                                                   get_local_time()))
        df = pd.DataFrame(topk_index)
        df.insert(0, "id", np.asarray(eval_data.get_eval_users()))
        df.columns = ["id"] + ["top_" + str(i) for i in range(k)]
        df.astype(int).to_csv(path, sep="\t", index=False)

    def _group(self, out, prefix, curves):
        for m in self.metrics:
            for k in self.topk:
                out[f"{prefix}_{_NAMES.get(m, m)}@{k}"] = round(float(curves[m][k - 1]), 4)

    def _extras(self, topk_index, pos_items, pos_len, hits, eval_data):
        out = {}
        if self.pop_items is not None:
            pop = self.pop_items
            groups = {"Pop": [], "Niche": []}
            for gt, rec in zip(pos_items, topk_index):
                gp = [i for i in gt if i in pop]
                gn = [i for i in gt if i not in pop]
                if gp:
                    sp = set(gp)
                    groups["Pop"].append((len(gp), [r in sp for r in rec]))
                if gn:
                    sn = set(gn)
                    groups["Niche"].append((len(gn), [r in sn for r in rec]))
            for name, lst in groups.items():
                if lst:
                    self._group(out, name, metric_curves(np.array([h for _, h in lst]), np.array([n for n, _ in lst])))
        if self.warm_users is not None:
            users = np.asarray(eval_data.get_eval_users())
            warm = np.array([u in self.warm_users for u in users])
            for name, msk in (("Cold", ~warm), ("Warm", warm)):
                if msk.any():
                    self._group(out, name, metric_curves(hits[msk], pos_len[msk]))
        item_num = eval_data.dataset.item_num
        if self.pop_items is not None and self.pop_mask is None:
            self.pop_mask = np.zeros(item_num, bool)
            self.pop_mask[[i for i in self.pop_items if i < item_num]] = True
        for k in self.topk:
            rec = topk_index[:, :k].reshape(-1)
            cnt = np.bincount(rec, minlength=item_num)
            out[f"Coverage@{k}"] = round(np.count_nonzero(cnt) / item_num, 4)
            srt = np.sort(cnt)
            tot = srt.sum()
            if tot > 0:
                n = item_num
                out[f"Gini@{k}"] = round(float((2 * np.sum(np.arange(1, n + 1) * srt)) / (n * tot) - (n + 1) / n), 4)
            else:
                out[f"Gini@{k}"] = 0.0
            counts = list(Counter(rec.tolist()).values())
            if counts:
                out[f"Gini2@{k}"] = round(float(cal_gini(counts)), 4)
                out[f"Coverage2@{k}"] = round(len(counts) / item_num, 4)
            else:
                out[f"Gini2@{k}"] = 0.0
                out[f"Coverage2@{k}"] = 0.0
            if self.pop_mask is not None:
                out[f"Tail%@{k}"] = round(float((~self.pop_mask[rec]).sum() / len(rec)), 4)
        return out
