"""GenRecV1 on MI355X — drop-in for models/genrecv1.py of the reference (GeneralRecommender API).

Rows G1-G5 of SURVEY.md §8a:
  * rec model (:16-427): user/item ID tables, modality projections (Linear+BN+LeakyReLU+Dropout),
    gates (Linear+BN+Sigmoid), user_item_GCN on norm_adj and the rebuilt (edge-dropped) UI graph,
    item_item_GCN on the kNN II graphs then R (U x I), gate_attention_fusion; calculate_loss =
    BPR(log-sigmoid) + reg + 4 InfoNCE terms on B x B logits.  One fused forward and a
    hand-derived backward: CSR SpMM (spmm.hip), fp32 MFMA GEMMs (gemm.hip), BN / fusion / content
    row kernels (genrec.hip), transposed CSRs for the non-symmetric graphs (gengraph.hip), the
    deterministic sorted scatter for the gathered rows;
  * FlipInterestDiffusion (:460-648) + ModalDenoiseTransformer (:650-710): gendiff.hip +
    transformer.py.

Layout in HBM (N = U + I, d = 64): one rec slab [E0 = user_embedding; item_id_embedding (N x 64) |
every other rec parameter under its reference name], the denoiser slab, N x 64 activation tables.
BatchNorm running statistics are kept per module and updated in the reference's call order.
"""
import copy
import ctypes
import os
import numpy as np
import torch
import torch.nn as nn

from . import _lib
from . import dist
from . import kernels as K
from .abstract_recommender import GeneralRecommender
from .kernels import ptr, stream
from .kmeans import kmeans_labels
from .slab import Slab
from .transformer import TransformerDenoiser

# GMR_NCE_FUSED (default 1): the four in-batch InfoNCE terms of the rec step through the fused contrast kernel
# (gmr_contrast_fused_f32 + gmr_nce_pairs / _combine); 0: logits GEMM + row softmax + two gradient GEMMs per term
NCE_FUSED = os.environ.get("GMR_NCE_FUSED", "1") != "0"

BN_NAMES = ["image_residual_project_1", "image_modal_project_1", "text_residual_project_1",
            "text_modal_project_1", "caculate_common_1", "gate_image_modal_1", "gate_text_modal_1",
            "gate_audio_modal_1"]
# BN call order of one forward (models/genrecv1.py:225-353) -> saved-statistics slot
_BN_CALLS = ["image_residual_project_1", "image_modal_project_1", "gate_image_modal_1",
             "text_residual_project_1", "text_modal_project_1", "gate_text_modal_1",
             "caculate_common_1", "caculate_common_1", "gate_image_modal_1", "gate_text_modal_1"]
ACT_NONE, ACT_LEAKY, ACT_SIGMOID, ACT_TANH = 0, 1, 2, 3
POST_NONE, POST_RES, POST_MUL, POST_ROWDOT = 0, 1, 2, 3


class _RecLoss(torch.autograd.Function):
    """calculate_loss as an autograd node (external trainers call loss.backward())."""

    @staticmethod
    def forward(ctx, model, users, pos, neg, *params):
        loss = model.rec_step(users, pos, neg)
        ctx.model = model
        return loss.clone()

    @staticmethod
    def backward(ctx, g):
        m = ctx.model
        return (None, None, None, None, *[m.grad_view(n) * g for n in m.param_names()])


def _rec_init_twin(U, I, d, DV, DT):
    """The reference constructor's RNG order (models/genrecv1.py:60-97, :155-222) on CPU torch
    modules, to draw identical initial values under the caller's seed."""
    out = {}
    out["origin_weight"] = torch.ones(1)
    out["generation_weight"] = torch.ones(1)
    for n in ("img_weight", "txt_weight", "aud_weight"):
        out[n] = torch.ones(1)
    for n in ("img_weight", "txt_weight", "aud_weight"):
        nn.init.normal_(out[n], mean=1.0, std=0.1)
    ue, ie = nn.Embedding(U, d), nn.Embedding(I, d)
    nn.init.xavier_uniform_(ue.weight)
    nn.init.xavier_uniform_(ie.weight)
    out["user_embedding_weight"], out["item_id_embedding_weight"] = ue.weight.data, ie.weight.data
    out["fusion_weight"] = torch.ones(3)
    out["res_scale"] = torch.ones(1)

    def proj(din):
        return nn.Sequential(nn.Linear(din, d), nn.BatchNorm1d(d), nn.LeakyReLU(0.2), nn.Dropout(0.1))

    mods = {}
    for mod, din in (("image", DV), ("text", DT)):
        if din is None:
            continue
        mods[mod + "_residual_project"] = proj(din)
        mods[mod + "_modal_project"] = proj(d)
        nn.init.xavier_uniform_(mods[mod + "_residual_project"][0].weight)
        nn.init.xavier_uniform_(mods[mod + "_modal_project"][0].weight)
    cc = nn.Sequential(nn.Linear(d, d), nn.BatchNorm1d(d), nn.Tanh(), nn.Linear(d, 1, bias=False))
    nn.init.xavier_uniform_(cc[0].weight)
    nn.init.xavier_uniform_(cc[3].weight)
    mods["caculate_common"] = cc
    for g in ("gate_image_modal", "gate_text_modal", "gate_audio_modal"):
        s = nn.Sequential(nn.Linear(d, d), nn.BatchNorm1d(d), nn.Sigmoid())
        nn.init.xavier_uniform_(s[0].weight)
        mods[g] = s
    for name, m in mods.items():
        for pn, p in m.named_parameters():
            out[f"{name}_{pn.replace('.', '_')}"] = p.data
    return out


class GenRecV1(GeneralRecommender):
    rec_step_takes_batch = True  # data parallel: the Trainer passes the global step's rows (in-batch InfoNCE)

    def __init__(self, config, dataloader):
        super().__init__(config, dataloader)
        c = config
        self.config = config
        self.latdim = int(c["embedding_size"])
        if self.latdim != 64:
            raise NotImplementedError("the gfx950 kernels are built for embedding_size = 64")
        self.n_layers = int(c["n_layers"])
        if self.n_layers != 1:
            raise NotImplementedError("n_layers = 1 (GenRecV1.yaml) is the configured hot path")
        self.keep_rate = float(c["keep_rate"])
        self.sparse_temp = float(c["sparse_temp"])
        self.temp = float(c["temperature"])
        self.scoring_dtype = str(c["scoring_dtype"] if "scoring_dtype" in c else "fp32")
        if self.scoring_dtype not in ("fp32", "fp16"):
            raise ValueError(f"scoring_dtype {self.scoring_dtype!r}: fp32 or fp16")
        self.ssl_reg1, self.ssl_reg2 = float(c["ssl_reg1"]), float(c["ssl_reg2"])
        self.gen_topk, self.rebuild_k = int(c["gen_topk"]), int(c["rebuild_k"])
        self.d_emb_size, self.nhead, self.num_layers = int(c["d_emb_size"]), int(c["nhead"]), int(c["num_layers"])
        self.steps = int(c["steps"])
        self.flip_temp = float(c["flip_temp"])
        self.bayesian_samplinge_schedule = bool(c["bayesian_samplinge_schedule"])
        self.sampling_steps = int(c["sampling_steps"])
        self.reg_weight = float(c["reg_weight"])
        self.audio_modality = bool(c["audio_modality"])
        if self.audio_modality:
            raise NotImplementedError("audio_modality: the reference cannot run it (self.a_feat unset, genrecv1.py:46; "
                                      "self.softmax undefined, :314) — see DESIGN.md")
        if self.v_feat is None or self.t_feat is None:
            raise NotImplementedError("GenRecV1's forward uses both the image and the text branch (:266-306)")
        if not self.bayesian_samplinge_schedule:
            raise NotImplementedError("bayesian_samplinge_schedule = True (GenRecV1.yaml) is the configured path")
        self.seed = int((c["seed"][0] if isinstance(c["seed"], (list, tuple)) else c["seed"]) or 0)
        U, I, d = self.n_users, self.n_items, 64
        self.N = U + I
        self.DV, self.DT = self.v_feat.shape[1], self.t_feat.shape[1]
        dev = self.device
        init = _rec_init_twin(U, I, d, self.DV, self.DT)
        specs = [("E0", (self.N, d), None)]
        for n, v in init.items():
            if n in ("user_embedding_weight", "item_id_embedding_weight"):
                continue
            specs.append((n, tuple(v.shape), None))
        self._pnames = [s[0] for s in specs[1:]]
        self.rec_slab = Slab(specs, dev)
        e0 = self.rec_slab.view("E0")
        e0[:U].copy_(init["user_embedding_weight"])
        e0[U:].copy_(init["item_id_embedding_weight"])
        for n in self._pnames:
            self.rec_slab.load(n, init[n])
        self.user_embedding_weight = nn.Parameter(e0[:U])
        self.user_embedding_weight.grad = self.rec_slab.gview("E0")[:U]
        self.item_id_embedding_weight = nn.Parameter(e0[U:])
        self.item_id_embedding_weight.grad = self.rec_slab.gview("E0")[U:]
        for n in self._pnames:
            setattr(self, n, self.rec_slab.parameter(n))
        self.bn_state = {n: (torch.zeros(d, device=dev), torch.ones(d, device=dev)) for n in BN_NAMES}
        # graphs: norm_adj (:54, :133-152), R (:55, :128-131) and R^T for the backward
        tl = dataloader
        self.user_ptr = torch.as_tensor(tl.uptr_np).to(dev)
        self.user_items = torch.as_tensor(tl.uitems_np).to(dev)
        self.norm_adj = K.bipartite_symnorm(U, I, self.user_ptr, self.user_items, self_loops=False, deg_eps=1e-7,
                                          seg_nnz=K.SPMM_NORM_ADJ)
        self.R = K.user_item_csr(U, I, self.user_ptr, self.user_items)
        self.RT = K.csr_transpose(self.R)
        self.image_UI_matrix = None
        self.image_UI_matrix_T = None
        self.image_II_matrix = None
        self.text_II_matrix = None
        self._ii_T = None
        # generator (:99-115): the denoiser is constructed after the rec modules (same RNG stream)
        self.denoise_in_dims = self.denoise_out_dims = I
        self.denoise_model_image = TransformerDenoiser(I, I, self.d_emb_size, dev, nhead=self.nhead,
                                                       num_layers=self.num_layers)
        self.denoise_model_image.init_like_reference()
        self.diffusion_model = FlipDiffusion(self)
        self._w = None
        self._step = 0
        self.training_mode = True

    # ================================================================= API pieces
    def param_names(self):
        return ["user_embedding_weight", "item_id_embedding_weight"] + self._pnames

    def grad_view(self, name):
        s, U = self.rec_slab, self.n_users
        if name == "user_embedding_weight":
            return s.gview("E0")[:U]
        if name == "item_id_embedding_weight":
            return s.gview("E0")[U:]
        return s.gview(name)

    def P(self, name):
        return self.rec_slab.view(name)

    def G(self, name):
        return self.rec_slab.gview(name)

    def optim_slabs(self):
        return [self.rec_slab]

    def train(self, mode=True):
        super().train(mode)
        self.training_mode = mode
        self.denoise_model_image.train(mode)
        return self

    def getItemEmbeds(self):
        return self.item_id_embedding_weight

    def getUserEmbeds(self):
        return self.user_embedding_weight

    # ================================================================= graphs built by the trainer
    def build_item_item_graphs(self, knn_k):
        """GenRecV1Trainer._build_item_item_matrix (common/trainer.py:673-687) on the device."""
        self.image_II_matrix = K.knn_graph(self.v_feat, knn_k)
        self.text_II_matrix = K.knn_graph(self.t_feat, knn_k)
        self._ii_T = (K.csr_transpose(self.image_II_matrix), K.csr_transpose(self.text_II_matrix))

    def set_image_ui_matrix(self, csr, transpose=None):
        """The rebuilt, edge-dropped UI graph and its transpose (backward of A2 = ui @ E)."""
        self.image_UI_matrix = csr
        self.image_UI_matrix_T = transpose if transpose is not None else K.csr_transpose(csr)

    def set_item_item_graphs(self, img, txt):
        self.image_II_matrix, self.text_II_matrix = img, txt
        self._ii_T = (K.csr_transpose(img), K.csr_transpose(txt))

    # ================================================================= buffers
    def _work(self, B):
        if self._w is not None and self._w["B"] >= B:
            return self._w
        N, I, U, dev = self.N, self.n_items, self.n_users, self.device
        f = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)  # noqa: E731
        Bp = (B + 3) // 4 * 4
        w = {"B": B, "A1": f(N, 64), "A2": f(N, 64), "C": f(N, 64),
             "Zr": f(2, I, 64), "Xr": f(2, I, 64), "Zm": f(2, I, 64), "F": f(2, I, 64), "Zg": f(2, I, 64),
             "Gt": f(2, I, 64), "Pm": f(2, I, 64), "MOD": f(2, N, 64), "Zc": f(2, N, 64), "a": f(2, N),
             "Zp": f(2, N, 64), "PG": f(2, N, 64), "SIDE": f(N, 64), "alpha": f(N),
             "stats": f(len(_BN_CALLS), 2, 64), "masks": torch.ones((4, I, 64), dtype=torch.uint8, device=dev),
             "parts": torch.empty(max(int(_lib.load().gmr_bn_parts_doubles(N)), 4096), dtype=torch.float64,
                                  device=dev),
             "sums": f(128), "sqws": torch.empty(1024, dtype=torch.float64, device=dev),
             # loss
             "loss_bpr": f(B), "contrib": f(3 * B, 64), "contrib_s": f(2 * B, 64), "contrib_g": f(2 * B, 64),
             "g": f(4, B, 64),
             "nv": f(4, B, 64), "nrm": f(4, B), "raw": f(4, B, 64), "L": f(B, Bp), "rows": f(4, B), "loss": f(4),
             # backward
             "dC": f(N, 64), "dS": f(N, 64), "dM": f(2, N, 64), "da": f(2, N), "dPG": f(2, N, 64),
             "dZ": f(N, 64), "dZ2": f(2, N, 64), "T1": f(N, 64), "T2": f(N, 64), "dP": f(I, 64), "dF": f(I, 64), "dX": f(I, 64),
             "dZi": f(I, 64)}
        self._w = w
        return w

    # ================================================================= forward
    def _bn(self, w, call, z, rows, act, train, y=None, keep=None, post=POST_NONE, aux=None, rs=None, out2=None,
            rowdot=None):
        name = _BN_CALLS[call]
        rm, rv = self.bn_state[name]
        st = w["stats"][call]
        pre = name[:-2]
        _lib.call("gmr_bn_fwd_f32", rows, ptr(z), K._ld(z), int(train), 1e-5, 0.1, ptr(rm), ptr(rv), ptr(w["parts"]),
                  ptr(st[0]), ptr(st[1]), ptr(self.P(pre + "_1_weight")), ptr(self.P(pre + "_1_bias")), act, 0.2,
                  ptr(keep), 64 if keep is not None else 0, 1.0 / 0.9, ptr(y), K._ld(y) if y is not None else 0, post,
                  ptr(aux), K._ld(aux) if (aux is not None and aux.dim() == 2) else 0, ptr(rs), ptr(out2),
                  K._ld(out2) if out2 is not None else 0, ptr(rowdot), stream())

    def _linear(self, x, name, out, beta=0.0):
        K.gemm(x, self.P(name + "_weight"), out, trans_b=True, epi=K.EPI_BIAS, bias=self.P(name + "_bias"), beta=beta)

    def _modal_feature(self, w, m, train, masks=None):
        """getImageFeats / getTextFeats (:225-239) -> w['F'][m] (and the saved BN inputs)."""
        mod = ("image", "text")[m]
        X = self.v_feat if m == 0 else self.t_feat
        I = self.n_items
        c0 = 3 * m
        mk = w["masks"]
        if train:
            for j, site in enumerate(("residual", "modal")):
                given = masks.get(f"{mod}_{site}_project_3") if masks else None
                if given is not None:
                    mk[2 * m + j].copy_(torch.as_tensor(given, dtype=torch.uint8))
                else:
                    _lib.call("gmr_keep_mask_u8", I * 64, 0.9, self.seed, self._mask_step(m, j), 0, ptr(mk[2 * m + j]),
                              stream())
        self._linear(X, f"{mod}_residual_project_0", w["Zr"][m])
        self._bn(w, c0, w["Zr"][m], I, ACT_LEAKY, train, y=w["Xr"][m], keep=mk[2 * m] if train else None)
        self._linear(w["Xr"][m], f"{mod}_modal_project_0", w["Zm"][m])
        self._bn(w, c0 + 1, w["Zm"][m], I, ACT_LEAKY, train, keep=mk[2 * m + 1] if train else None, post=POST_RES,
                 aux=w["Xr"][m], rs=self.P("res_scale"), out2=w["F"][m])
        return w["F"][m]

    def _mask_step(self, m, j):
        return (self._step * 8 + 2 * m + j) * 2 + (0 if self.training_mode else 1)

    def _content(self, w):
        """user_item_GCN on norm_adj and the rebuilt UI graph, softmax-weighted (:255-264, :332-336)."""
        E = self.rec_slab.view("E0")
        self.norm_adj.spmm(w["A1"], [(E,)])
        self.image_UI_matrix.spmm(w["A2"], [(E,)])
        _lib.call("gmr_gr_content_fwd", self.N, ptr(E), ptr(w["A1"]), ptr(w["A2"]), ptr(self.P("origin_weight")),
                  ptr(self.P("generation_weight")), ptr(w["C"]), stream())
        return w["C"]

    def _forward(self, w, train, masks=None):
        """GenRecV1.forward (:330-353): content -> C, side -> SIDE (train mode: BN batch statistics,
        running-stat updates, dropout)."""
        U, I, N = self.n_users, self.n_items, self.N
        iE = self.rec_slab.view("E0")[U:]
        self._content(w)
        for m, (gate, ii) in enumerate((("gate_image_modal", self.image_II_matrix),
                                        ("gate_text_modal", self.text_II_matrix))):
            F = self._modal_feature(w, m, train, masks)
            self._linear(F, gate + "_0", w["Zg"][m])
            self._bn(w, 3 * m + 2, w["Zg"][m], I, ACT_SIGMOID, train, y=w["Gt"][m], post=POST_MUL, aux=iE,
                     out2=w["Pm"][m])
            MOD = w["MOD"][m]
            ii.spmm(MOD[U:], [(w["Pm"][m],)])                 # item_item_GCN (n_layers = 1)
            self.R.spmm(MOD[:U], [(MOD[U:],)])                 # users <- R @ items
        wc2 = self.P("caculate_common_3_weight").view(64)
        # caculate_common's Linear on both modality tables in one product (the same weight: 2N stacked rows)
        self._linear(w["MOD"].view(2 * N, 64), "caculate_common_0", w["Zc"].view(2 * N, 64))
        for m in range(2):
            self._bn(w, 6 + m, w["Zc"][m], N, ACT_TANH, train, post=POST_ROWDOT, aux=wc2, rowdot=w["a"][m])
        for m, gate in enumerate(("gate_image_modal", "gate_text_modal")):
            self._linear(w["C"], gate + "_0", w["Zp"][m])
            self._bn(w, 8 + m, w["Zp"][m], N, ACT_SIGMOID, train, y=w["PG"][m])
        _lib.call("gmr_gr_fusion_fwd", N, ptr(w["MOD"][0]), ptr(w["MOD"][1]), ptr(w["a"][0]), ptr(w["a"][1]),
                  ptr(w["PG"][0]), ptr(w["PG"][1]), ptr(w["SIDE"]), ptr(w["alpha"]), stream())
        return w["C"], w["SIDE"]

    # ================================================================= fused rec step
    def _nce(self, w, i1, i2, coef, rows, row0=0, B=None, Bg=None):
        """InfoNCE(nv[i1], nv[i2]) (:407-414): loss rows + gradients into g[i1], g[i2].  Queries are
        rows [row0, row0 + B) of the step, keys all Bg rows (one process: row0 = 0, B = Bg)."""
        Bg = w["B"] if Bg is None else Bg
        B = Bg if B is None else B
        v1, v2 = w["nv"][i1][row0:row0 + B], w["nv"][i2][:Bg]
        L = w["L"][:B, :Bg]
        inv_t = 1.0 / self.temp
        K.gemm(v1, v2, L, trans_b=True, alpha=inv_t)
        _lib.call("gmr_nce_rows_off_f32", B, Bg, ptr(L), L.stride(0), row0, coef, ptr(rows), stream())
        K.gemm(L, v2, w["g"][i1][row0:row0 + B], alpha=inv_t, beta=1.0)
        K.gemm(L, v1, w["g"][i2][:Bg], trans_a=True, alpha=inv_t, beta=1.0)

    def _nce_fused(self, w, terms, nr, loss, row0, B, Bg):
        """The four in-batch InfoNCE terms through the fused contrast kernel (gmr_contrast_fused_f32: no B x Bg
        logit block, no GEMM launches): pair rows, one contrast call per term, then every nv row's
        gradient in one combine pass (w['g'] overwritten)."""
        nv, g = w["nv"], w["g"]
        tab = nv.stride(0) // 64
        if "nce_cln" not in w:
            Bm = w["B"]
            f = lambda *sh: torch.empty(sh, dtype=torch.float32, device=self.device)  # noqa: E731
            w["nce_cln"], w["nce_ctr"], w["nce_dt"] = f(4, Bm, 128), f(4, Bm, 128), f(4, Bm, 64)
            w["nce_nodes"] = torch.arange(Bm, dtype=torch.int32, device=self.device)
            self._nce_i1 = (ctypes.c_int32 * 4)(*[t[0] for t in terms])
            self._nce_i2 = (ctypes.c_int32 * 4)(*[t[1] for t in terms])
        cln, ctr, dt = w["nce_cln"], w["nce_ctr"], w["nce_dt"]
        i1p, i2p = ctypes.cast(self._nce_i1, ctypes.c_void_p), ctypes.cast(self._nce_i2, ctypes.c_void_p)
        _lib.call("gmr_nce_pairs_f32", 4, B, Bg, row0, i1p, i2p, ptr(nv), tab, ptr(cln), cln.stride(0) // 128, stream())
        ws = K.contrast_workspace(B, Bg, self.device, "gr_nce")
        for k, (i1, i2, reg) in enumerate(terms):
            rows = w["rows"][k][:B]
            K.contrast_fused(nv[i1][row0:row0 + B], nv[i2][:Bg], cln[k], w["nce_nodes"][:B], 0, 1.0 / self.temp,
                             reg / nr, rows, ctr[k][:B], dt[k][:Bg], ws)
            _lib.call("gmr_sum_f32", B, ptr(rows), reg / nr, ptr(loss), 1, stream())
        _lib.call("gmr_nce_combine_f32", 4, B, Bg, row0, i1p, i2p, ptr(ctr), ctr.stride(0) // 128, ptr(dt),
                  dt.stride(0) // 64, ptr(g), tab, stream())

    def rec_step(self, users, pos, neg, plan_bpr=None, plan_cl=None, norm_rows=None, reg_share=1.0, masks=None,
                 gbatch=None):
        """calculate_loss (:355-405) and all rec-parameter gradients (into rec_slab.grad).

        gbatch = (step users, step pos, row0) under data parallelism: the four in-batch InfoNCE terms
        (:389-397) take this rank's rows [row0, row0 + B) of the global step as queries against the
        step's keys, so the sum over ranks is the reference's global-batch loss; each rank scatters
        its key-side gradients for every step row and the rec-slab all-reduce adds them up."""
        if self.image_UI_matrix is None:
            return torch.zeros((), device=self.device)  # the reference returns 0 before the first rebuild (:363-364)
        B = users.numel()
        nr = float(norm_rows or B)
        gu, gp, row0 = (users, pos, 0) if gbatch is None else gbatch
        Bg = gu.numel()
        if not 0 <= row0 <= Bg - B:
            raise ValueError(f"rank rows [{row0}, {row0 + B}) outside the step's {Bg} rows")
        w = self._work(max(B, Bg))
        U, I, N = self.n_users, self.n_items, self.N
        s = self.rec_slab
        E0 = s.view("E0")
        if plan_bpr is None:
            plan_bpr, plan_cl = self._plans(users, pos, neg)
        C, SIDE = self._forward(w, True, masks)
        # ---- losses
        contrib, cs = w["contrib"][:3 * B], w["contrib_s"][:2 * Bg]
        _lib.call("gmr_bpr_logsigmoid_f32", B, U, ptr(C), ptr(users), ptr(pos), ptr(neg), ptr(w["loss_bpr"]),
                  ptr(contrib), 1.0 / nr, stream())
        loss = w["loss"][:1]
        _lib.call("gmr_sum_f32", B, ptr(w["loss_bpr"]), 1.0 / nr, ptr(loss), 0, stream())
        _lib.call("gmr_sqnorm_f32", N * 64, ptr(E0), self.reg_weight * reg_share, ptr(loss), 1, ptr(w["sqws"]),
                  stream())
        # gathered views of the step's rows: 0 = C[users], 1 = C[U+pos], 2 = SIDE[users], 3 = SIDE[U+pos]
        for j, (src, idx, off) in enumerate(((C, gu, 0), (C, gp, U), (SIDE, gu, 0), (SIDE, gp, U))):
            K.gather_rows(src, idx, w["raw"][j][:Bg], off=off)
            K.normalize_rows(w["raw"][j][:Bg], w["nv"][j][:Bg], w["nrm"][j][:Bg])
        terms = ((3, 1, self.ssl_reg1), (2, 0, self.ssl_reg1), (0, 1, self.ssl_reg2), (0, 3, self.ssl_reg2))
        if NCE_FUSED:
            self._nce_fused(w, terms, nr, loss, row0, B, Bg)
        else:
            K.zero_(w["g"])
            for k, (i1, i2, reg) in enumerate(terms):
                rows = w["rows"][k][:B]
                self._nce(w, i1, i2, reg / nr, rows, row0, B, Bg)
                _lib.call("gmr_sum_f32", B, ptr(rows), reg / nr, ptr(loss), 1, stream())
        dC, dS = w["dC"], w["dS"]
        K.zero_(dC)
        K.zero_(dS)
        K.normalize_rows_bwd(w["nv"][2][:Bg], w["nrm"][2][:Bg], w["g"][2][:Bg], cs[:Bg])
        K.normalize_rows_bwd(w["nv"][3][:Bg], w["nrm"][3][:Bg], w["g"][3][:Bg], cs[Bg:])
        if gbatch is None:  # the views' rows are the BPR rows: one scatter per table
            K.normalize_rows_bwd(w["nv"][0][:B], w["nrm"][0][:B], w["g"][0][:B], contrib[:B], accumulate=True)
            K.normalize_rows_bwd(w["nv"][1][:B], w["nrm"][1][:B], w["g"][1][:B], contrib[B:2 * B], accumulate=True)
            plan_g = plan_cl
        else:  # the step's rows: their own plan (keys users | U + pos, as plan_cl)
            cg = w["contrib_g"][:2 * Bg]
            K.normalize_rows_bwd(w["nv"][0][:Bg], w["nrm"][0][:Bg], w["g"][0][:Bg], cg[:Bg])
            K.normalize_rows_bwd(w["nv"][1][:Bg], w["nrm"][1][:Bg], w["g"][1][:Bg], cg[Bg:])
            plan_g = self._plan2(gu, gp)
            _lib.call("gmr_scatter_sorted_f32", plan_g.numel(), 64, ptr(plan_g), ptr(cg), 64, ptr(dC), 64, stream())
        _lib.call("gmr_scatter_sorted_f32", plan_bpr.numel(), 64, ptr(plan_bpr), ptr(contrib), 64, ptr(dC), 64, stream())
        _lib.call("gmr_scatter_sorted_f32", plan_g.numel(), 64, ptr(plan_g), ptr(cs), 64, ptr(dS), 64, stream())
        self._backward(w, reg_share)
        self._step += 1
        return loss[0]

    def _plan2(self, users, pos):
        """Sorted scatter plan of the keys [users | U + pos] (plan_cl's layout) for any row set."""
        B = users.numel()
        dev = self.device
        keys = torch.stack([users, pos]).to(torch.int32).contiguous()
        # the constant operands are built once (per B): torch.tensor(..., device) is a blocking copy
        cache = self.__dict__.setdefault("_plan2_const", {})
        if B not in cache:
            cache[B] = (torch.tensor([0, B], dtype=torch.int64, device=dev),
                        torch.tensor([0, self.n_users], dtype=torch.int32, device=dev))
        offs, ka = cache[B]
        pc = torch.empty((1, 1 << max(1, (2 * B - 1).bit_length())), dtype=torch.int64, device=dev)
        _lib.call("gmr_sort_batch_keys", 1, ptr(keys), ptr(offs), ptr(ka), 2, B, ptr(pc), pc.shape[1], pc.shape[1],
                  stream())
        return pc[0]

    def _bn_bwd(self, w, call, z, rows, act, dy=None, mul=None, keep=None, da=None, dz=None, acc_dz=False):
        name = _BN_CALLS[call]
        pre = name[:-2]
        st = w["stats"][call]
        dv = self.G("caculate_common_3_weight").view(64) if da is not None else None
        _lib.call("gmr_bn_bwd_f32", rows, ptr(z), K._ld(z), ptr(st[0]), ptr(st[1]), ptr(self.P(pre + "_1_weight")),
                  ptr(self.P(pre + "_1_bias")), act, 0.2, ptr(keep), 64 if keep is not None else 0, 1.0 / 0.9,
                  ptr(dy), K._ld(dy) if dy is not None else 0, ptr(mul), K._ld(mul) if mul is not None else 0,
                  ptr(da), ptr(self.P("caculate_common_3_weight").view(64)) if da is not None else None,
                  ptr(w["parts"]), ptr(w["sums"]), ptr(self.G(pre + "_1_weight")), ptr(self.G(pre + "_1_bias")),
                  ptr(dv), 1, ptr(dz), K._ld(dz), int(acc_dz), stream())
        return dz

    def _linear_bwd(self, dz, x, name, dx=None, dx_beta=0.0):
        """y = x W^T + b: dW += dz^T x, db += colsum(dz), dx (+)= dz W."""
        K.gemm(dz, x, self.G(name + "_weight"), trans_a=True, beta=1.0)
        K.colsum(dz, self.G(name + "_bias"), accumulate=True)
        if dx is not None:
            K.gemm(dz, self.P(name + "_weight"), dx, beta=dx_beta)

    def _backward(self, w, reg_share):
        U, I, N = self.n_users, self.n_items, self.N
        s = self.rec_slab
        s.zero_grad()
        E0 = s.view("E0")
        gE = s.gview("E0")
        iE = E0[U:]
        dC, dS, dM, dZ = w["dC"], w["dS"], w["dM"], w["dZ"]
        _lib.call("gmr_gr_fusion_bwd", N, ptr(w["MOD"][0]), ptr(w["MOD"][1]), ptr(w["alpha"]), ptr(w["PG"][0]),
                  ptr(w["PG"][1]), ptr(dS), ptr(dM[0]), ptr(dM[1]), ptr(w["da"][0]), ptr(w["da"][1]), ptr(w["dPG"][0]),
                  ptr(w["dPG"][1]), stream())
        # prefer gates on the content table (:344-345)
        for m, gate in enumerate(("gate_image_modal", "gate_text_modal")):
            self._bn_bwd(w, 8 + m, w["Zp"][m], N, ACT_SIGMOID, dy=w["dPG"][m], dz=dZ)
            self._linear_bwd(dZ, w["C"], gate + "_0", dx=dC, dx_beta=1.0)
        # attention scores (caculate_common on IMG / TXT, :313-323)
        dZ2 = w["dZ2"]
        for m in range(2):
            self._bn_bwd(w, 6 + m, w["Zc"][m], N, ACT_TANH, da=w["da"][m], dz=dZ2[m])
        self._linear_bwd(dZ2.view(2 * N, 64), w["MOD"].view(2 * N, 64), "caculate_common_0", dx=dM.view(2 * N, 64),
                         dx_beta=1.0)
        # item_item_GCN branches (:266-306)
        for m, (mod, gate) in enumerate((("image", "gate_image_modal"), ("text", "gate_text_modal"))):
            d = dM[m]
            self.RT.spmm(d[U:], [(d[:U],)], beta=1.0)                      # dP2 += R^T dU
            self._ii_T[m].spmm(w["dP"], [(d[U:],)])                        # dP = II^T dP2
            _lib.call("gmr_mul64_f32", I, ptr(w["dP"]), 64, ptr(w["Gt"][m]), 64, ptr(gE[U:]), 64, 1.0, 1, stream())
            self._bn_bwd(w, 3 * m + 2, w["Zg"][m], I, ACT_SIGMOID, dy=w["dP"], mul=iE, dz=w["dZi"])
            self._linear_bwd(w["dZi"], w["F"][m], gate + "_0", dx=w["dF"])
            _lib.call("gmr_dot64_f32", I, ptr(w["Xr"][m]), 64, ptr(w["dF"]), 64, ptr(w["parts"]), 1.0,
                      ptr(self.G("res_scale")), 1, stream())
            mk = w["masks"]
            self._bn_bwd(w, 3 * m + 1, w["Zm"][m], I, ACT_LEAKY, dy=w["dF"], keep=mk[2 * m + 1], dz=w["dZi"])
            self._linear_bwd(w["dZi"], w["Xr"][m], f"{mod}_modal_project_0", dx=w["dX"])
            _lib.call("gmr_axpy_dev_f32", I * 64, ptr(self.P("res_scale")), ptr(w["dF"]), ptr(w["dX"]), stream())
            self._bn_bwd(w, 3 * m, w["Zr"][m], I, ACT_LEAKY, dy=w["dX"], keep=mk[2 * m], dz=w["dZi"])
            X = self.v_feat if m == 0 else self.t_feat
            self._linear_bwd(w["dZi"], X, f"{mod}_residual_project_0")
        # content (user_item_GCN x 2, softmax weights) + regulariser
        self.norm_adj.spmm(w["T1"], [(dC,)])
        self.image_UI_matrix_T.spmm(w["T2"], [(dC,)])
        _lib.call("gmr_gr_content_bwd", N, ptr(E0), ptr(w["A1"]), ptr(w["A2"]), ptr(dC), ptr(w["T1"]), ptr(w["T2"]),
                  ptr(self.P("origin_weight")), ptr(self.P("generation_weight")), 2.0 * self.reg_weight * reg_share,
                  ptr(w["parts"]), ptr(gE), ptr(self.G("origin_weight")), ptr(self.G("generation_weight")), stream())

    def _plans(self, users, pos, neg):
        B = users.numel()
        dev = self.device
        keys = torch.stack([users, pos, neg]).contiguous()
        offs = torch.tensor([0, B], dtype=torch.int64, device=dev)
        p2 = lambda n: 1 << max(1, (n - 1).bit_length())  # noqa: E731
        pb = torch.empty((1, p2(3 * B)), dtype=torch.int64, device=dev)
        pc = torch.empty((1, p2(2 * B)), dtype=torch.int64, device=dev)
        ka = torch.tensor([0, self.n_users, self.n_users], dtype=torch.int32, device=dev)
        _lib.call("gmr_sort_batch_keys", 1, ptr(keys), ptr(offs), ptr(ka), 3, B, ptr(pb), pb.shape[1], pb.shape[1],
                  stream())
        _lib.call("gmr_sort_batch_keys", 1, ptr(keys), ptr(offs), ptr(ka), 2, B, ptr(pc), pc.shape[1], pc.shape[1],
                  stream())
        return pb[0], pc[0]

    # ================================================================= reference-facing API
    def calculate_loss(self, interaction):
        users, pos, neg = (interaction[i].to(torch.int32).contiguous() for i in range(3))
        params = [getattr(self, n) for n in self.param_names()]
        for p in params:
            p.grad = None
        return _RecLoss.apply(self, users, pos, neg, *params)

    def getImageFeats(self):
        w = self._work(1)
        return self._modal_feature(w, 0, self.training_mode)

    def getTextFeats(self):
        w = self._work(1)
        return self._modal_feature(w, 1, self.training_mode)

    @torch.no_grad()
    def forward_embeddings(self):
        """content embeddings (the only part of forward full_sort_predict uses, :417-427)."""
        w = self._work(1)
        if self.image_UI_matrix is None:  # :419-421 scores are zeros before the first rebuild
            K.zero_(w["C"])
            return w["C"][:self.n_users], w["C"][self.n_users:]
        C = self._content(w)
        return C[:self.n_users], C[self.n_users:]

    @torch.no_grad()
    def forward(self, train=None):
        """(content, side) like GenRecV1.forward; train defaults to the module mode."""
        w = self._work(1)
        return self._forward(w, self.training_mode if train is None else train)

    @torch.no_grad()
    def full_sort_predict(self, interaction):
        user = interaction[0].to(torch.int32)
        if self.image_UI_matrix is None:
            return torch.zeros((user.numel(), self.n_items), device=self.device)  # :419-421
        usr, itm = self.forward_embeddings()
        ub = torch.empty((user.numel(), 64), device=self.device)
        K.gather_rows(usr, user, ub)
        scores = torch.empty((user.numel(), self.n_items), device=self.device)
        self._score(ub, itm, scores)
        return scores

    @property
    def fused_eval(self):
        """The trainer's fused score -> mask -> top-k kernel computes fp32 scores; the opt-in fp16
        scoring keeps its own MFMA GEMM + mask + top-k."""
        return self.scoring_dtype == "fp32"

    def _score(self, ub, itm, out):
        """usr[users] @ itm^T (genrecv1.py:419-427): fp32 MFMA GEMM, or the opt-in fp16 MFMA one."""
        if self.scoring_dtype == "fp16":
            K.score_f16(ub, itm, out)
        else:
            K.gemm(ub, itm, out, trans_b=True)
        return out

    @torch.no_grad()
    def topk_from_embeddings(self, usr, itm, users_i32, mask_rows, mask_cols, k, out_idx, scores_buf, out_val=None):
        E = users_i32.numel()
        ub = scores_buf.new_empty((E, 64))
        K.gather_rows(usr, users_i32, ub)
        sc = scores_buf[:E, :self.n_items]
        self._score(ub, itm, sc)
        K.mask_scores(sc, mask_rows, mask_cols)
        K.topk_rows(sc, k, out_idx, out_val)
        return out_idx

    def extra_state(self):
        out = {"bn_state": {k: (v[0].cpu(), v[1].cpu()) for k, v in self.bn_state.items()}}
        if self.image_UI_matrix is not None:
            g = self.image_UI_matrix
            out["image_UI_matrix"] = {"rowptr": g.rowptr.cpu(), "col": g.col.cpu(), "val": g.val.cpu()}
            t = self.image_UI_matrix_T
            out["image_UI_matrix_T"] = {"rowptr": t.rowptr.cpu(), "col": t.col.cpu(), "val": t.val.cpu()}
        return out

    def load_extra_state(self, st):
        """Inverse of extra_state: BatchNorm running statistics and the rebuilt (dropped) UI graph."""
        for k, (mean, var) in (st.get("bn_state") or {}).items():
            self.bn_state[k][0].copy_(mean)
            self.bn_state[k][1].copy_(var)
        g = st.get("image_UI_matrix")
        if g is not None:
            dev = self.device
            mk = lambda d: K.CSR(d["rowptr"].to(dev), d["col"].to(dev), d["val"].to(dev), symmetric=False,  # noqa: E731
                                 class_split=self.n_users, side=True)
            t = st.get("image_UI_matrix_T")
            self.set_image_ui_matrix(mk(g), mk(t) if t is not None else None)


# GMR_GR_OVERLAP=0: GenRecV1's training step runs its value-only p_sample after the backward on one stream, and
# the rebuild chunks one after another (default 1: side stream 0 through a twin context, see FlipDiffusion.twin).
# Epoch 102.0-107.5 -> 92.3-93.8 ms (diffusion phase 45.1 -> 36.9 ms, rebuild 29.6 -> 22.8 ms;
# profiles/r05zb_genrecv1_overlap_*.txt)
OVERLAP_PSAMPLE = os.environ.get("GMR_GR_OVERLAP", "1") != "0"
# streams the rebuild chunks are dealt over (the main stream + REBUILD_STREAMS - 1 side streams, each chunk through
# its stream's context); GMR_GR_REBUILD_STREAMS overrides, for A/B runs.  Two beat three: epoch 88.6-90.2 vs
# 92.4 ms (profiles/r05zc_genrecv1_rebuild_streams_ab.txt)
REBUILD_STREAMS = int(os.environ.get("GMR_GR_REBUILD_STREAMS", "2"))


class FlipDiffusion:
    """FlipInterestDiffusion (models/genrecv1.py:460-648) over device batches of users.

    Batches are given as int32 user ids; x0 rows are densified from the train user CSR.  All draws
    are Philox (seed, step); parity tests inject the reference's draws through `inject`."""

    def __init__(self, model):
        self.m = model
        self.steps = model.steps
        self.base_temp = model.flip_temp
        self.sparse_temp = model.sparse_temp
        self._w = None
        self._parts = None

    def _work(self, B):
        if self._w is not None and self._w["B"] >= B:
            return self._w
        I = self.m.n_items
        Ip = (I + 3) // 4 * 4
        dev = self.m.device
        f = lambda *s, dt=torch.float32: torch.empty(s, dtype=dt, device=dev)  # noqa: E731
        self._w = {"B": B, "x0": f(B, Ip), "xt": f(B, Ip), "z": f(B, Ip), "dz": f(B, Ip), "probs": f(B, Ip),
                   "tab": f(2 * self.steps + 2), "t": f(B, dt=torch.int32), "bce": f(B, dt=torch.float64),
                   "kl": f(B, dt=torch.float64), "fe": f(I, 64), "o": f(2, B, 64), "nv": f(2, B, 64), "nrm": f(2, B),
                   "L": f(B, (B + 3) // 4 * 4), "rows": f(B), "loss": f(4, dt=torch.float64), "lossf": f(2), "lossv": f(4),
                   "topk": f(B, max(self.m.gen_topk, 1), dt=torch.int32)}
        return self._w

    def twin(self, den, k=1):
        """The k-th (FlipDiffusion, denoiser) context (k >= 1) over the same model and weights with private work
        buffers, made once per denoiser: work issued on side stream k - 1 through it touches none of another
        context's buffers (the training step's value-only p_sample beside its backward; the rebuild chunks)."""
        tws = self.__dict__.setdefault("_tw", {})
        tw = tws.get(k)
        if tw is None or tw[0] is not den:
            d2 = copy.copy(self)
            d2.__dict__.pop("_tw", None)
            d2._w, d2._parts, d2._picks, d2._npicks, d2._keys = None, None, None, None, None
            tw = tws[k] = (den, d2, den.twin())
        tw[2].training, tw[2].p = den.training, den.p
        return tw[1], tw[2]

    def side(self):
        """The side streams of the twin-context work (K.Streams(2)), made on first use."""
        st = self.__dict__.get("_side")
        if st is None:
            st = self._side = K.Streams(REBUILD_STREAMS - 1 if REBUILD_STREAMS > 1 else 1)
        return st

    def densify(self, users):
        B = users.numel()
        w = self._work(B)
        I = self.m.n_items
        x0 = w["x0"][:B, :I]
        _lib.call("gmr_diff_densify", B, I, ptr(users), ptr(self.m.user_ptr), ptr(self.m.user_items), ptr(x0),
                  x0.stride(0), stream())
        return x0

    def schedule(self, users):
        w = self._work(users.numel())
        _lib.call("gmr_flip_schedule", users.numel(), ptr(users), ptr(self.m.user_ptr), self.m.n_items, self.steps,
                  ptr(w["tab"]), stream())
        return w["tab"]

    def p_sample(self, den, x0, tab, seed, step, inject=None, probs_out=None, q_steps=None, row0=0):
        """p_sample(steps = q_steps, bayesian) (:528-548): q_sample at t = q_steps - 1 (none when
        q_steps = 0), then T model calls; the Bayesian step's coefficients are the q_sample tables at
        that t (:541-542 re-index the q_sample tensors).  Returns the final x and the last probs.
        Draws are keyed by (step, row0 + row): x0's rows are rows [row0, row0 + B) of the step."""
        B, I = x0.shape
        w = self._w
        T = self.steps
        qs = T if q_steps is None else int(q_steps)
        if qs == 0:
            raise NotImplementedError("p_sample with steps = 0 reads alpha tables left by an earlier call")
        xt, z = w["xt"][:B, :I], w["z"][:B, :I]
        inj = inject or {}
        flip = inj.get("flip")
        _lib.call("gmr_flip_qsample", B, I, ptr(x0), x0.stride(0), None, qs - 1, ptr(tab), T, self.base_temp,
                  ptr(flip), flip.stride(0) if flip is not None else 0, seed, step * 16, row0, ptr(xt), xt.stride(0),
                  stream())
        probs = probs_out if probs_out is not None else w["probs"][:B, :I]
        for j, i in enumerate(reversed(range(T))):
            den.forward(xt, t_const=i, T=T, out=z, seed=seed, step=step * 16 + 1 + j, row0=row0, reuse_tables=j > 0,
                        keep_acts=False)
            draws = inj.get("draws")
            dr = draws[j] if draws is not None else None
            _lib.call("gmr_flip_step", B, I, ptr(z), z.stride(0), ptr(tab), T, qs - 1, int(i == 0), ptr(dr),
                      dr.stride(0) if dr is not None else 0, seed, step * 16 + 8 + j, row0, ptr(xt), xt.stride(0),
                      ptr(probs) if i == 0 else None, probs.stride(0), stream())
        return xt, probs

    def training_step(self, den, users, item_embeds, feats, seed, step, norm_rows=None, sched_users=None,
                      inject=None, row0=0, rank_rows=None):
        """training_losses (:550-606) + the denoiser backward (only the BCE term carries gradient).
        Returns the device loss vector [bce, kl, cl, total] (fp64; the loss of the rows held here,
        normalised by norm_rows).  The BCE backward runs before the p_sample of the InfoNCE term
        (which reuses the denoiser workspace); the reference's value is unchanged by the order.
        Data parallel: users are rows [row0, row0 + B) of the step whose ranks hold rank_rows rows;
        every draw is keyed by the global row and the InfoNCE keys are the whole step's rows, so the
        SUM over ranks of the returned vector and of the gradients is the single-process step's."""
        B = users.numel()
        nr = float(norm_rows or B)
        w = self._work(B)
        I, T = self.m.n_items, self.steps
        inj = inject or {}
        x0 = self.densify(users)
        tab = self.schedule(sched_users if sched_users is not None else users)
        t = w["t"][:B]
        if "t" in inj:
            t.copy_(inj["t"])
        else:
            _lib.call("gmr_diff_sample_t", B, T, seed, step, row0, ptr(t), stream())
        xt, z, dz = w["xt"][:B, :I], w["z"][:B, :I], w["dz"][:B, :I]
        flip = inj.get("flip1")
        _lib.call("gmr_flip_qsample", B, I, ptr(x0), x0.stride(0), ptr(t), 0, ptr(tab), T, self.base_temp, ptr(flip),
                  flip.stride(0) if flip is not None else 0, seed, step * 16 + 15, row0, ptr(xt), xt.stride(0), stream())
        den.forward(xt, t_rows=t, T=T, out=z, masks=inj.get("den_masks"), seed=seed, step=step * 16 + 14, row0=row0)
        _lib.call("gmr_flip_loss_rows", B, I, ptr(x0), x0.stride(0), ptr(z), z.stride(0), ptr(t), ptr(tab), T,
                  1.0 / (nr * I), ptr(dz), dz.stride(0), ptr(w["bce"]), ptr(w["kl"]), stream())
        ps_inj = {"flip": inj.get("ps_flip"), "draws": inj.get("ps_draws")}
        if OVERLAP_PSAMPLE and (rank_rows is None or len(rank_rows) == 1):
            # the value-only p_sample + InfoNCE (:577-582) reads x0, the schedule and the weights, none of which
            # the backward writes: it runs on side stream 0 through the twin context, beside the backward;
            # the join below comes before the caller's Adam step
            d2, den2 = self.twin(den)
            d2._work(B)
            st = self.side()
            with st.on(0):
                gen, _ = d2.p_sample(den2, x0, tab, seed, step + 1, inject=ps_inj, row0=row0)
                cl = d2.infonce_value(x0, gen, item_embeds, feats, row0, rank_rows)
        den.backward(dz)
        loss = w["loss"]
        _lib.call("gmr_sum_f64", B, ptr(w["bce"]), 1.0 / (nr * I), ptr(loss[0:1]), 0, stream())
        _lib.call("gmr_sum_f64", B, ptr(w["kl"]), 1.0 / nr, ptr(loss[1:2]), 0, stream())
        if OVERLAP_PSAMPLE and (rank_rows is None or len(rank_rows) == 1):
            st.join(0)
        else:
            # InfoNCE(x0 (iE * feats), p_sample(x0) (iE * feats)) — value only (:577-582)
            gen, _ = self.p_sample(den, x0, tab, seed, step + 1, inject=ps_inj, row0=row0)
            cl = self.infonce_value(x0, gen, item_embeds, feats, row0, rank_rows)
        out = w["lossv"]
        _lib.call("gmr_flip_total", ptr(loss), ptr(cl), 0.01, ptr(out), stream())
        return out

    def infonce_value(self, x0, gen, item_embeds, feats, row0=0, rank_rows=None):
        """InfoNCE(x0 (iE * feats), gen (iE * feats)) of the step (:577-582), value only.  Data
        parallel: this rank's rows are the queries, the keys are all the step's rows (gathered), and
        the returned value is this rank's share of the step mean (the SUM over ranks is the mean)."""
        B, I = x0.shape
        w = self._w
        fe = w["fe"]
        _lib.call("gmr_mul64_f32", I, ptr(item_embeds), K._ld(item_embeds), ptr(feats), K._ld(feats), ptr(fe), 64,
                  1.0, 0, stream())
        o = w["o"]
        K.gemm(x0, fe, o[0][:B])
        K.gemm(gen, fe, o[1][:B])
        K.normalize_rows(o[0][:B], w["nv"][0][:B], w["nrm"][0][:B])
        K.normalize_rows(o[1][:B], w["nv"][1][:B], w["nrm"][1][:B])
        out = w["lossf"][:1]
        if rank_rows is None or len(rank_rows) == 1:
            L = w["L"][:B, :B]
            K.gemm(w["nv"][0][:B], w["nv"][1][:B], L, trans_b=True, alpha=1.0 / self.sparse_temp)
            _lib.call("gmr_nce_rows_f32", B, ptr(L), L.stride(0), 0.0, ptr(w["rows"]), stream())
            _lib.call("gmr_sum_f32", B, ptr(w["rows"]), 1.0 / B, ptr(out), 0, stream())
            return out
        keys = dist.gather_step_rows(w["nv"][1][:B], rank_rows)
        Bg = keys.shape[0]
        Lbuf = self.__dict__.get("_Ldp")
        if Lbuf is None or Lbuf.shape[0] < B or Lbuf.shape[1] < (Bg + 3) // 4 * 4:
            Lbuf = self._Ldp = torch.empty((B, (Bg + 3) // 4 * 4), dtype=torch.float32, device=self.m.device)
        L = Lbuf[:B, :Bg]
        K.gemm(w["nv"][0][:B], keys, L, trans_b=True, alpha=1.0 / self.sparse_temp)
        _lib.call("gmr_nce_rows_off_f32", B, Bg, ptr(L), L.stride(0), int(row0), 0.0, ptr(w["rows"]), stream())
        _lib.call("gmr_sum_f32", B, ptr(w["rows"]), 1.0 / Bg, ptr(out), 0, stream())
        return out

    def idle_step(self, rank_rows):
        """A rank holding no rows of a data-parallel step: joins the step's InfoNCE key gather."""
        dist.gather_step_rows(torch.zeros((0, 64), dtype=torch.float32, device=self.m.device), rank_rows)

    # ------------------------------------------------------------------ graph rebuild (trainer.py:736-789)
    @torch.no_grad()
    def rebuild_rows(self, den, users, out_topk, labels, ratio, seed, step, inject=None):
        """One rebuild batch: p_sample(sampling_steps) -> gen_topk mask on the probabilities ->
        InterestDebiase (labels given) -> top-rebuild_k of denoised * probs into out_topk
        (ties -> lowest index).  Returns (denoised, probs) views of the work buffers."""
        m = self.m
        inj = inject or {}
        B = users.numel()
        I = m.n_items
        x0 = self.densify(users)
        tab = self.schedule(users)
        w = self._w
        probs = w["probs"][:B, :I]
        xs, _ = self.p_sample(den, x0, tab, seed, step, inject=inj, probs_out=probs, q_steps=m.sampling_steps)
        tk = w["topk"][:B, :m.gen_topk]
        K.topk_rows(probs, m.gen_topk, tk)
        dn = w["dz"][:B, :I]
        assert dn.stride(0) == x0.stride(0) == xs.stride(0)
        _lib.call("gmr_gen_mask", B, I, m.gen_topk, ptr(tk), tk.stride(0), ptr(x0), ptr(xs), x0.stride(0), ptr(dn),
                  stream())
        self.gen_mask_topk = tk
        if labels is not None:
            self._debias(B, tk, x0, xs, dn, labels, ratio, seed, step, inj)
        score = w["z"][:B, :I]
        _lib.call("gmr_mul_f32", B * x0.stride(0), ptr(dn), ptr(probs), ptr(score), stream())
        K.topk_rows(score, m.rebuild_k, out_topk)
        return dn, probs

    def _debias(self, B, tk, x0, xs, dn, labels, ratio, seed, step, inj):
        """InterestDebiase.interest_query_debiase (interest_cluster.py:248-332)."""
        I = self.m.n_items
        kg = tk.shape[1]
        maxp = B * kg
        dev = self.m.device
        if getattr(self, "_picks", None) is None or self._picks.shape[1] < maxp:
            self._picks = torch.zeros((2, maxp, 2), dtype=torch.int32, device=dev)
            self._npicks = torch.zeros(2, dtype=torch.int32, device=dev)
        picks, npk = self._picks, self._npicks
        if "dislike" in inj:  # parity: the reference's random.sample picks
            cnt = []
            for t, key in enumerate(("dislike", "like")):
                pk = torch.as_tensor(np.asarray(inj[key]), dtype=torch.int32).reshape(-1, 2)
                if pk.shape[0]:
                    picks[t, :pk.shape[0]].copy_(pk)
                cnt.append(pk.shape[0])
            npk.copy_(torch.as_tensor(cnt, dtype=torch.int32))
        else:
            if getattr(self, "_keys", None) is None or self._keys.numel() < 2 * maxp:
                self._keys = torch.empty(2 * maxp, dtype=torch.int64, device=dev)
            _lib.call("gmr_debias_select", B, kg, ptr(tk), tk.stride(0), ptr(x0), ptr(xs), x0.stride(0), float(ratio),
                      seed, step, ptr(self._keys), ptr(picks), picks.shape[1], ptr(npk), stream())
        for t in range(2):
            _lib.call("gmr_debias_apply", t, ptr(picks[t]), ptr(npk), picks.shape[1], ptr(x0), x0.stride(0), I,
                      ptr(labels), ptr(dn), dn.stride(0), stream())
