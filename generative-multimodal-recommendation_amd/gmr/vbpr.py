"""VBPR on MI355X — drop-in for models/vbpr.py of the reference (GeneralRecommender API).

Layout in HBM: one (U + I) x 128 table `UI` in the parameter slab — user rows are u_embedding
(U x 2d), item rows are [i_embedding | item_linear(raw)] (the reference's concatenated
item_embeddings, vbpr.py:68-74), so the BPR gathers and the sorted gradient scatter work on a
single table with items at row offset U.  The item_linear output columns are work space: the
forward GEMM rewrites them every step and their gradient is zeroed after it has produced the
item_linear gradients, so Adam never moves them.
  forward      F = raw @ W^T + b          (fp32 MFMA GEMM, BIAS epilogue, into UI[U:, 64:])
  loss         BPR + reg_weight * EmbLoss  (gmr_vbpr_loss_fwd_bwd: rows, fp64 reduce, contribs)
  backward     sorted scatter into the slab gradient; dW = dF^T raw, db = colsum(dF)
  predict      gather user rows, scores = U_b @ item_table^T (GEMM, K = 128)
"""
import torch
import torch.nn as nn

from . import _lib
from . import dist
from . import kernels as K
from .abstract_recommender import GeneralRecommender
from .kernels import ptr, stream
from .slab import Slab


def _r4(n):
    return (n + 3) // 4 * 4


class _Linear(nn.Module):
    def __init__(self, weight, bias):
        super().__init__()
        self.weight = weight
        self.bias = bias


class _VBPRLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, users, pos, neg, *params):
        loss = model.rec_step(users, pos, neg)
        ctx.model = model
        return loss.clone()

    @staticmethod
    def backward(ctx, g):
        return (None, None, None, None, *[gv * g for gv in ctx.model.grad_views()])


class VBPR(GeneralRecommender):
    def __init__(self, config, dataloader):
        super().__init__(config, dataloader)
        d = int(config["embedding_size"])
        if d != 64:
            raise NotImplementedError("embedding_size = 64 (VBPR.yaml)")
        self.u_embedding_size = self.i_embedding_size = d
        self.reg_weight = float(config["reg_weight"])
        U, I, dev = self.n_users, self.n_items, self.device
        self.D = 2 * d
        # item_raw_features = cat(t_feat, v_feat) (vbpr.py:34-39), rows padded to 16 bytes
        feats = [f for f in (self.t_feat, self.v_feat) if f is not None]
        Kr = sum(f.shape[1] for f in feats)
        self.raw_dim = Kr
        raw = torch.zeros((I, _r4(Kr)), device=dev)
        c = 0
        for f in feats:
            raw[:, c:c + f.shape[1]].copy_(f)
            c += f.shape[1]
        self.raw = raw[:, :Kr]
        # parameters in the reference's RNG order (vbpr.py:31-45, common/init.py)
        g_u = nn.init.xavier_uniform_(torch.empty(U, 2 * d))
        g_i = nn.init.xavier_uniform_(torch.empty(I, d))
        lin = nn.Linear(Kr, d)
        nn.init.xavier_normal_(lin.weight.data)
        nn.init.constant_(lin.bias.data, 0)
        self.slab = Slab([("UI", (U + I, 2 * d), None), ("W", (d, Kr), _r4(Kr)), ("b", (d,), None)], dev)
        ui, gui = self.slab.view("UI"), self.slab.gview("UI")
        ui[:U].copy_(g_u)
        ui[U:, :d].copy_(g_i)
        ui[U:, d:].zero_()
        self.slab.load("W", lin.weight.data)
        self.slab.load("b", lin.bias.data)
        self.u_embedding = nn.Parameter(ui[:U])
        self.u_embedding.grad = gui[:U]
        self.i_embedding = nn.Parameter(ui[U:, :d])
        self.i_embedding.grad = gui[U:, :d]
        self.item_linear = _Linear(self.slab.parameter("W"), self.slab.parameter("b"))
        self._w = None

    def optim_slabs(self):
        return [self.slab]

    def grad_views(self):
        g, U, d = self.slab.gview("UI"), self.n_users, self.u_embedding_size
        return [g[:U], g[U:, :d], self.slab.gview("W"), self.slab.gview("b")]

    def _work(self, B):
        if self._w is not None and self._w["B"] >= B:
            return self._w
        dev = self.device
        self._w = {"B": B, "x": torch.empty(B, device=dev), "sq": torch.empty(3 * B, dtype=torch.float64, device=dev),
                   "coef": torch.empty(4, device=dev), "loss": torch.empty(4, device=dev),
                   "contrib": torch.empty((3 * B, self.D), device=dev)}
        return self._w

    def _item_features(self):
        """UI[U:, 64:] = item_linear(item_raw_features) (vbpr.py:69)."""
        F = self.slab.view("UI")[self.n_users:, self.i_embedding_size:]
        K.gemm(self.raw, self.slab.view("W"), F, trans_b=True, epi=K.EPI_BIAS, bias=self.slab.view("b"))
        return F

    def _plan(self, users, pos, neg):
        B = users.numel()
        keys = torch.stack([users, pos, neg]).contiguous()
        offs = torch.tensor([0, B], dtype=torch.int64, device=self.device)
        ka = torch.tensor([0, self.n_users, self.n_users], dtype=torch.int32, device=self.device)
        n2 = 1 << max(1, (3 * B - 1).bit_length())
        plan = torch.empty((1, n2), dtype=torch.int64, device=self.device)
        _lib.call("gmr_sort_batch_keys", 1, ptr(keys), ptr(offs), ptr(ka), 3, B, ptr(plan), n2, n2, stream())
        return plan[0]

    def rec_step(self, users, pos, neg, plan_bpr=None, plan_cl=None, norm_rows=None, reg_share=1.0):
        """calculate_loss (vbpr.py:76-97) and all parameter gradients (into the slab gradient)."""
        if dist.is_dist():
            raise NotImplementedError("VBPR (the CPU-plumbing config) runs on one device")
        B = users.numel()
        if norm_rows not in (None, B):
            raise ValueError("VBPR normalises by its own batch")
        if plan_bpr is None:
            plan_bpr = self._plan(users, pos, neg)
        w = self._work(B)
        U, d = self.n_users, self.i_embedding_size
        s = self.slab
        ui = s.view("UI")
        self._item_features()
        _lib.call("gmr_vbpr_loss_fwd_bwd", B, self.D, ptr(ui), ui.stride(0), ptr(users), ptr(pos), ptr(neg), U,
                  self.reg_weight, ptr(w["x"]), ptr(w["sq"]), ptr(w["coef"]), ptr(w["loss"]), ptr(w["contrib"]),
                  self.D, stream())
        s.zero_grad()
        gui = s.gview("UI")
        _lib.call("gmr_scatter_sorted_f32", plan_bpr.numel(), self.D, ptr(plan_bpr), ptr(w["contrib"]), self.D,
                  ptr(gui), gui.stride(0), stream())
        dF = gui[U:, d:]
        K.gemm(dF, self.raw, s.gview("W"), trans_a=True)                      # dW = dF^T raw
        K.colsum(dF, s.gview("b"))                                             # db
        _lib.call("gmr_fill2d_f32", dF.shape[0], dF.shape[1], ptr(dF), dF.stride(0), 0.0, stream())
        return w["loss"][0]

    def calculate_loss(self, interaction):
        users, pos, neg = (interaction[i].to(torch.int32).contiguous() for i in range(3))
        params = [self.u_embedding, self.i_embedding, self.item_linear.weight, self.item_linear.bias]
        for p in params:
            p.grad = None
        return _VBPRLoss.apply(self, users, pos, neg, *params)

    # ------------------------------------------------------------------ prediction
    @torch.no_grad()
    def forward_embeddings(self):
        self._item_features()
        ui = self.slab.view("UI")
        return ui[:self.n_users], ui[self.n_users:]

    @torch.no_grad()
    def topk_from_embeddings(self, usr, itm, users_i32, mask_rows, mask_cols, k, out_idx, scores_buf, out_val=None):
        E = users_i32.numel()
        ub = scores_buf.new_empty((E, self.D))
        K.gather_rows(usr, users_i32, ub)
        sc = scores_buf[:E, :self.n_items]
        K.gemm(ub, itm, sc, trans_b=True)
        K.mask_scores(sc, mask_rows, mask_cols)
        K.topk_rows(sc, k, out_idx, out_val)
        return out_idx

    @torch.no_grad()
    def full_sort_predict(self, interaction):
        users = interaction[0].to(torch.int32).contiguous()
        usr, itm = self.forward_embeddings()
        E = users.numel()
        ub = torch.empty((E, self.D), device=self.device)
        K.gather_rows(usr, users, ub)
        scores = torch.empty((E, self.n_items), device=self.device)
        K.gemm(ub, itm, scores, trans_b=True)
        return scores
