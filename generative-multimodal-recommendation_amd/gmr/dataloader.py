"""Device-resident data loaders — mirror utils/dataloader.py of the reference.

TrainDataLoader keeps the train split on the GPU and draws each epoch with the on-device
sampler (gmr_sample_epoch: shuffled interactions + rejection-sampled negatives, reference
dataloader.py:218-275).  Iterating it yields (3, B) LongTensors [users, pos, neg] exactly like
the reference; the fused trainers use `epoch()` which returns int32 views plus the per-batch
sorted scatter plans the deterministic gradient kernels need.

EvalDataLoader reproduces the evaluation order and masks of the reference
(dataloader.py:330-416): users in order of first appearance in the split, train-positive mask
as (2, nnz) with batch-local row ids, eval positives per user.
"""
import math

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib
from .kernels import ptr, stream


def user_csr(n_users, users, items):
    """Unique, ascending items per user (the binary-adjacency view of the interactions)."""
    key = np.unique(np.asarray(users, np.int64) * (int(np.max(items)) + 1 if len(items) else 1) + np.asarray(items))
    n_it = int(np.max(items)) + 1 if len(items) else 1
    u, i = key // n_it, key % n_it
    rowptr = np.zeros(n_users + 1, np.int64)
    np.add.at(rowptr, u + 1, 1)
    return np.cumsum(rowptr).astype(np.int32), i.astype(np.int32)


def _pow2(n):
    return 1 << max(1, math.ceil(math.log2(max(n, 2))))


class TrainDataLoader:
    def __init__(self, config, dataset, batch_size=1, shuffle=False):
        self.config = config
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.step = self.batch_size
        self.shuffle = shuffle
        self.device = config["device"]
        df = dataset.df
        self.u_np = df[dataset.uid_field].values.astype(np.int32)
        self.i_np = df[dataset.iid_field].values.astype(np.int32)
        self.n_inter = len(self.u_np)
        self.n_users, self.n_items = dataset.get_user_num(), dataset.get_item_num()
        self.all_items_np = np.unique(self.i_np).astype(np.int32)
        self.uptr_np, self.uitems_np = user_csr(self.n_users, self.u_np, self.i_np)
        self.seed = int((config["seed"][0] if isinstance(config["seed"], (list, tuple)) else config["seed"]) or 0)
        self._epoch = 0
        self._dev = None
        self.pr = 0

    # --- device state -------------------------------------------------------------
    def sub_batch_offsets(self, world):
        """Interaction offsets of the (batch, rank) sub-batches: batch b = rows [b*B, min((b+1)*B, n))
        of the epoch draw, split in contiguous shards over `world` data-parallel ranks (the first
        rows % world ranks hold one more row).  Returns nb * world + 1 monotone offsets."""
        nb = (self.n_inter + self.batch_size - 1) // self.batch_size
        offs = [0]
        for b in range(nb):
            lo, hi = b * self.batch_size, min((b + 1) * self.batch_size, self.n_inter)
            q, rem = divmod(hi - lo, world)
            for r in range(world):
                offs.append(offs[-1] + q + (1 if r < rem else 0))
        return np.asarray(offs, np.int64)

    def to_device(self):
        from . import dist
        W = 1 if dist.local_batches() else dist.world()  # sub-batches per batch (whole batches: 1)
        if self._dev is not None and self._dev["world"] != W:
            self._dev = None
        if self._dev is None:
            d = self.device
            t = lambda a: torch.as_tensor(a).to(d)  # noqa: E731
            nb = (self.n_inter + self.batch_size - 1) // self.batch_size
            offs = self.sub_batch_offsets(W)
            sb = -(-self.batch_size // W)  # rows of the largest sub-batch
            self._dev = {
                "world": W,
                "inter_user": t(self.u_np), "inter_item": t(self.i_np),
                "user_ptr": t(self.uptr_np), "user_items": t(self.uitems_np),
                "all_items": t(self.all_items_np),
                "batch_offsets": t(offs), "offsets_np": offs, "n_batches": nb,
                "sample": torch.empty((3, self.n_inter), dtype=torch.int32, device=d),
                "plan_bpr": torch.empty((nb * W, _pow2(3 * sb)), dtype=torch.int64, device=d),
                "plan_cl": torch.empty((nb * W, _pow2(2 * sb)), dtype=torch.int64, device=d),
                "key_add_bpr": t(np.array([0, self.n_users, self.n_users], np.int32)),
                "key_add_cl": t(np.array([0, self.n_users], np.int32)),
                "n_fallback": torch.zeros(1, dtype=torch.int32, device=d),
            }
        return self._dev

    def pretrain_setup(self):
        self._epoch = 0

    def inter_matrix(self, form="coo", value_field=None):
        data = np.ones(self.n_inter) if value_field is None else self.dataset.df[value_field].values
        m = sp.coo_matrix((data, (self.u_np, self.i_np)), shape=(self.n_users, self.n_items))
        return m if form == "coo" else m.tocsr()

    def epoch(self, with_plans=True):
        """Draw one epoch on the device: returns dict with 'sample' (3, n_inter) int32 and plans."""
        d = self.to_device()
        s = d["sample"]
        _lib.call("gmr_zero", ptr(d["n_fallback"]), 4, stream())
        _lib.call("gmr_sample_epoch", self.n_inter, ptr(d["inter_user"]), ptr(d["inter_item"]), ptr(d["user_ptr"]),
                  ptr(d["user_items"]), ptr(d["all_items"]), len(self.all_items_np), self.seed, self._epoch,
                  ptr(s[0]), ptr(s[1]), ptr(s[2]), ptr(d["n_fallback"]), stream())
        self._epoch += 1
        if with_plans:
            nb = d["n_batches"] * d["world"]  # one plan per (batch, rank) sub-batch
            _lib.call("gmr_sort_batch_keys", nb, ptr(s), ptr(d["batch_offsets"]), ptr(d["key_add_bpr"]), 3,
                      self.n_inter, ptr(d["plan_bpr"]), d["plan_bpr"].shape[1], d["plan_bpr"].shape[1], stream())
            _lib.call("gmr_sort_batch_keys", nb, ptr(s), ptr(d["batch_offsets"]), ptr(d["key_add_cl"]), 2,
                      self.n_inter, ptr(d["plan_cl"]), d["plan_cl"].shape[1], d["plan_cl"].shape[1], stream())
        return d

    def fallbacks(self):
        """Rows of the last epoch draw whose negative is not a true negative (device read; 0 unless
        a user holds nearly every item, see gmr_sample_epoch)."""
        return int(self.to_device()["n_fallback"].item())

    def batches(self, d, rank=None):
        """Per global optimiser step g of the epoch draw: (g, rank_rows, users, pos, neg, plan_bpr,
        plan_cl) of this rank's rows — its sub-batch of batch g (the whole batch at world size 1), or
        under GMR_DP_MODE=local its own whole batch g * world + rank.  rank_rows lists the rows of
        every rank in the step (dist.dp_scales normalises by their sum); a rank's part may be empty."""
        from . import dist
        W = d["world"]
        r = dist.rank() if rank is None else rank
        nb, B = d["n_batches"], self.batch_size
        s, offs = d["sample"], d["offsets_np"]
        if W == 1 and dist.local_batches():
            Wd = dist.world()
            for g in range(-(-nb // Wd)):
                sizes = [max(0, min(self.n_inter, (g * Wd + q + 1) * B) - min(self.n_inter, (g * Wd + q) * B))
                         for q in range(Wd)]
                b = g * Wd + r
                if b < nb:
                    lo, hi = int(offs[b]), int(offs[b + 1])
                    yield g, sizes, s[0, lo:hi], s[1, lo:hi], s[2, lo:hi], d["plan_bpr"][b], d["plan_cl"][b]
                else:
                    e = s[:, :0]
                    yield g, sizes, e[0], e[1], e[2], d["plan_bpr"][0], d["plan_cl"][0]
            return
        for b in range(nb):
            lo, hi = int(offs[b * W + r]), int(offs[b * W + r + 1])
            rows = min((b + 1) * B, self.n_inter) - b * B
            yield (b, dist.shard_sizes(rows, W), s[0, lo:hi], s[1, lo:hi], s[2, lo:hi], d["plan_bpr"][b * W + r],
                   d["plan_cl"][b * W + r])

    def step_rows(self, d, g, rank=None):
        """(users, pos, row0) of global optimiser step g: every row of the step (the global batch g,
        or under GMR_DP_MODE=local the world whole batches of step g, which sit back to back in the
        epoch draw) and the offset of this rank's rows inside it.  In-batch terms (GenRecV1's B x B
        InfoNCE, models/genrecv1.py:407-414) take their keys from all of them."""
        from . import dist
        W, r = d["world"], dist.rank() if rank is None else rank
        s, offs = d["sample"], d["offsets_np"]
        if W == 1 and dist.local_batches():
            Wd = dist.world()
            nb = d["n_batches"]
            glo, ghi = int(offs[min(nb, g * Wd)]), int(offs[min(nb, (g + 1) * Wd)])
            own = int(offs[min(nb, g * Wd + r)])
        else:
            glo, ghi = int(offs[g * W]), int(offs[(g + 1) * W])
            own = int(offs[g * W + r])
        return s[0, glo:ghi], s[1, glo:ghi], own - glo

    # --- reference-style iteration -------------------------------------------------------
    def __len__(self):
        return math.ceil(self.n_inter / self.step)

    def __iter__(self):
        d = self.epoch(with_plans=False)
        s, B = d["sample"], self.batch_size
        for lo in range(0, self.n_inter, B):
            yield s[:, lo:lo + B].long()


class EvalDataLoader:
    def __init__(self, config, dataset, additional_dataset=None, batch_size=1, shuffle=False):
        if additional_dataset is None:
            raise ValueError("Training datasets is nan")
        self.config = config
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.step = self.batch_size
        self.device = config["device"]
        uid, iid = dataset.uid_field, dataset.iid_field
        # users in order of first appearance (pandas unique, dataloader.py:345)
        ev_u = dataset.df[uid].values.astype(np.int64)
        self.eval_u_np = ev_u[np.sort(np.unique(ev_u, return_index=True)[1])]
        n_users = dataset.get_user_num()
        rank = np.full(n_users, -1, np.int64)
        rank[self.eval_u_np] = np.arange(len(self.eval_u_np))
        # train positives of each eval user, in train-df order (groupby keeps row order)
        tr_u = additional_dataset.df[uid].values.astype(np.int64)
        tr_i = additional_dataset.df[iid].values.astype(np.int64)
        sel = rank[tr_u] >= 0
        r, it = rank[tr_u[sel]], tr_i[sel]
        order = np.argsort(r, kind="stable")
        self.mask_rows_np, self.mask_cols_np = r[order], it[order]
        self.train_pos_len = np.bincount(self.mask_rows_np, minlength=len(self.eval_u_np))
        # eval positives per user, in split-df order
        er = rank[ev_u]
        eo = np.argsort(er, kind="stable")
        e_items = dataset.df[iid].values.astype(np.int64)[eo]
        self.eval_len_list = np.bincount(er, minlength=len(self.eval_u_np))
        self.eval_ptr_np = np.concatenate([[0], np.cumsum(self.eval_len_list)]).astype(np.int64)
        self.eval_items_per_u = np.split(e_items, self.eval_ptr_np[1:-1])
        self.eval_items_flat = e_items
        self.pr = 0
        self.inter_pr = 0
        self._dev = None

    def to_device(self):
        if self._dev is None:
            d = self.device
            # sorted positives per user for the device hit test
            sorted_items = np.concatenate([np.sort(x) for x in self.eval_items_per_u]) if len(
                self.eval_items_per_u) else np.zeros(0, np.int64)
            mptr = np.concatenate([[0], np.cumsum(self.train_pos_len)]).astype(np.int64)
            by_row = np.lexsort((self.mask_cols_np, self.mask_rows_np))  # the fused eval kernel's mask order
            self._dev = {
                "mask_ptr_dev": torch.as_tensor(mptr).to(d),
                "mask_cols_sorted": torch.as_tensor(self.mask_cols_np[by_row].astype(np.int32)).to(d),
                "eval_u32": torch.as_tensor(self.eval_u_np.astype(np.int32)).to(d),
                "eval_u": torch.as_tensor(self.eval_u_np).to(d),
                "mask_rows": torch.as_tensor(self.mask_rows_np.astype(np.int32)).to(d),
                "mask_cols": torch.as_tensor(self.mask_cols_np.astype(np.int32)).to(d),
                "mask_ptr": mptr,
                "pos_ptr": torch.as_tensor(self.eval_ptr_np).to(d),
                "pos_items": torch.as_tensor(sorted_items.astype(np.int32)).to(d),
            }
        return self._dev

    @property
    def pr_end(self):
        return len(self.eval_u_np)

    def __len__(self):
        return math.ceil(self.pr_end / self.step)

    def __iter__(self):
        d = self.to_device()
        mptr = d["mask_ptr"]
        for lo in range(0, self.pr_end, self.step):
            hi = min(lo + self.step, self.pr_end)
            users = d["eval_u"][lo:hi]
            m0, m1 = int(mptr[lo]), int(mptr[hi])
            mask = torch.stack([(d["mask_rows"][m0:m1] - lo).long(), d["mask_cols"][m0:m1].long()])
            yield [users, mask]

    def get_eval_items(self):
        return self.eval_items_per_u

    def get_eval_len_list(self):
        return self.eval_len_list

    def get_eval_users(self):
        return torch.as_tensor(self.eval_u_np)
