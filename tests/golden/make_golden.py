"""Generate golden input/output vectors by importing the reference GenMMRec code.

Runs ONLY in the build container (the reference tree is mounted read-only at
/root/reference and never travels to the GPU box).  The outputs are small
.npz/.json fixtures under tests/golden/ that pin the CPU oracle (oracle/) and,
through it, the HIP path.

Reference entry points exercised (paths relative to GenMMRec/src):
  models/diffmm.py:88-107    DiffMM.get_norm_adj_mat
  models/diffmm.py:129-195   forward_MM / forward_cl_MM
  models/diffmm.py:203-258   calculate_loss / contrastLoss (+ autograd grads)
  models/diffmm.py:303-360   Denoise.forward
  models/diffmm.py:362-484   GaussianDiffusion tables / p_sample / training_losses
  common/trainer.py:464-485  DiffMMTrainer.normalizeAdj / buildUIMatrix
  common/trainer.py:369-388  Trainer.evaluate (mask + topk)
  utils/topk_evaluator.py:77-120 + utils/metrics.py   Recall/NDCG/Precision/MAP
  utils/dataset.py + utils/dataloader.py   split / eval-user order / masks
  models/diffrec.py, models/vbpr.py  (DiffRec / VBPR fixtures)

Usage:  python tests/golden/make_golden.py
"""
import json
import os
import sys
import tempfile
import types

import numpy as np

REF_SRC = "/root/reference/GenMMRec/src"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF_SRC)
    # torchvision/lmdb are imported but unused on this path (utils/dataset.py:17-18)
    du = types.ModuleType("utils.data_utils")
    for n in ["ImageResize", "ImagePad", "image_to_tensor", "load_decompress_img_from_lmdb_value"]:
        setattr(du, n, None)
    sys.modules["utils.data_utils"] = du
    sys.modules["lmdb"] = types.ModuleType("lmdb")
    np.float = float  # utils/metrics.py uses the removed alias
    import torch  # noqa
    import models.diffmm as diffmm
    import models.diffrec as diffrec
    import models.vbpr as vbpr
    import common.trainer as trainer
    import utils.topk_evaluator as topk_evaluator
    import utils.dataset as dataset
    import utils.dataloader as dataloader
    return dict(diffmm=diffmm, diffrec=diffrec, vbpr=vbpr, trainer=trainer,
                topk_evaluator=topk_evaluator, dataset=dataset, dataloader=dataloader)


class Cfg(dict):
    def __getitem__(self, k):
        return dict.get(self, k, None)

    def __contains__(self, k):
        return dict.__contains__(self, k)


def make_interactions(rng, U, I, min_deg=5):
    """Synthetic (user,item) train lists: every user >= min_deg distinct items."""
    rows, cols = [], []
    pop = rng.zipf(1.8, size=I).astype(np.float64)
    pop = pop / pop.sum()
    for u in range(U):
        deg = min(I - 1, min_deg + rng.poisson(2))
        items = rng.choice(I, size=deg, replace=False, p=pop)
        rows.extend([u] * deg)
        cols.extend(items.tolist())
    return np.asarray(rows, np.int64), np.asarray(cols, np.int64)


class MockDS:
    def __init__(self, U, I):
        self.U, self.I = U, I

    def get_user_num(self):
        return self.U

    def get_item_num(self):
        return self.I


class MockLoader:
    def __init__(self, U, I, rows, cols):
        import scipy.sparse as sp
        self.dataset = MockDS(U, I)
        self._m = sp.coo_matrix((np.ones(len(rows)), (rows, cols)), shape=(U, I))

    def inter_matrix(self, form="coo"):
        return self._m if form == "coo" else self._m.tocsr()


def coo_of(sp_tensor):
    t = sp_tensor.coalesce()
    return t.indices().numpy().astype(np.int64), t.values().numpy().astype(np.float32)


def gen_diffmm(ref, tmp):
    import torch
    diffmm = ref["diffmm"]
    rng = np.random.default_rng(7)
    U, I, d = 97, 61, 64
    DV, DT, H = 128, 48, 32
    rows, cols = make_interactions(rng, U, I)
    os.makedirs(os.path.join(tmp, "tiny"), exist_ok=True)
    v_feat = np.abs(rng.standard_normal((I, DV))).astype(np.float32)
    t_feat = rng.standard_normal((I, DT)).astype(np.float32)
    t_feat /= np.linalg.norm(t_feat, axis=1, keepdims=True)
    np.save(os.path.join(tmp, "tiny", "image_feat.npy"), v_feat)
    np.save(os.path.join(tmp, "tiny", "text_feat.npy"), t_feat)
    cfg = Cfg(USER_ID_FIELD="userID", ITEM_ID_FIELD="itemID", NEG_PREFIX="neg__", train_batch_size=40,
              device=torch.device("cpu"), end2end=False, is_multimodal_model=True, data_path=tmp + "/",
              dataset="tiny", vision_feature_file="image_feat.npy", text_feature_file="text_feat.npy",
              embedding_size=d, n_layers=1, reg_weight=1e-6, ssl_reg=1e-2, temperature=0.1, keep_rate=1,
              dims=[H], d_emb_size=10, norm=False, steps=5, noise_scale=0.1, noise_min=1e-4, noise_max=0.02,
              sampling_noise=False, sampling_steps=0, rebuild_k=1, e_loss=0.5, ris_lambda=0.1,
              ris_adj_lambda=0.2, trans_type=0, cl_method=0)
    torch.manual_seed(999)
    loader = MockLoader(U, I, rows, cols)
    model = diffmm.DiffMM(cfg, loader)
    out = {}
    out["U"], out["I"], out["d"] = np.int64(U), np.int64(I), np.int64(d)
    out["train_rows"], out["train_cols"] = rows, cols
    out["v_feat"], out["t_feat"] = v_feat, t_feat
    for name in ["uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight"]:
        out["p_" + name] = getattr(model, name).detach().numpy().copy()
    idx, val = coo_of(model.norm_adj)
    out["norm_adj_idx"], out["norm_adj_val"] = idx, val
    # rebuilt UI graphs (trainer.py:464-485) from fixed top-1 edges
    tr = object.__new__(ref["trainer"].DiffMMTrainer)
    tr.user_num, tr.item_num, tr.device = U, I, torch.device("cpu")
    ui_img = rng.integers(0, I, size=U)
    ui_txt = rng.integers(0, I, size=U)
    img_adj = tr.buildUIMatrix(np.arange(U), ui_img, np.ones(U))
    txt_adj = tr.buildUIMatrix(np.arange(U), ui_txt, np.ones(U))
    out["ui_img_items"], out["ui_txt_items"] = ui_img.astype(np.int64), ui_txt.astype(np.int64)
    out["img_adj_idx"], out["img_adj_val"] = coo_of(img_adj)
    out["txt_adj_idx"], out["txt_adj_val"] = coo_of(txt_adj)
    # buildUIMatrix with rebuild_k = 3 (distinct items per user)
    k3 = np.stack([rng.choice(I, size=3, replace=False) for _ in range(U)])
    adj3 = tr.buildUIMatrix(np.repeat(np.arange(U), 3), k3.reshape(-1), np.ones(3 * U))
    out["ui_k3_items"] = k3.astype(np.int64)
    out["ui_k3_idx"], out["ui_k3_val"] = coo_of(adj3)
    model.image_UI_matrix = model.edgeDropper(img_adj)
    model.text_UI_matrix = model.edgeDropper(txt_adj)
    with torch.no_grad():
        out["img_feats"] = model.getImageFeats().numpy()
        out["txt_feats"] = model.getTextFeats().numpy()
        u_e, i_e = model.forward_MM(model.norm_adj, model.image_UI_matrix, model.text_UI_matrix)
        out["fwd_usr"], out["fwd_itm"] = u_e.numpy(), i_e.numpy()
        cl = model.forward_cl_MM(model.norm_adj, model.image_UI_matrix, model.text_UI_matrix)
        for n, t in zip(["cl_u1", "cl_i1", "cl_u2", "cl_i2"], cl):
            out[n] = t.numpy()
    # calculate_loss + autograd grads (diffmm.py:203-249)
    B = 40
    users = torch.as_tensor(rng.integers(0, U, size=B))
    pos = torch.as_tensor(rng.integers(0, I, size=B))
    neg = torch.as_tensor(rng.integers(0, I, size=B))
    out["bpr_users"], out["bpr_pos"], out["bpr_neg"] = users.numpy(), pos.numpy(), neg.numpy()
    model.zero_grad()
    loss = model.calculate_loss(torch.stack([users, pos, neg]))
    loss.backward()
    out["rec_loss"] = np.float32(loss.item())
    for name in ["uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight"]:
        out["g_" + name] = getattr(model, name).grad.numpy().copy()
    # loss parts
    with torch.no_grad():
        u1, i1, u2, i2 = model.forward_cl_MM(model.norm_adj, model.image_UI_matrix, model.text_UI_matrix)
        out["cl_user"] = np.float32(model.contrastLoss(u1, u2, users, 0.1).item())
        out["cl_item"] = np.float32(model.contrastLoss(i1, i2, pos, 0.1).item())
    # cl_method = 1 variant of the loss
    model.cl_method = 1
    model.zero_grad()
    loss1 = model.calculate_loss(torch.stack([users, pos, neg]))
    loss1.backward()
    out["rec_loss_cl1"] = np.float32(loss1.item())
    out["g_cl1_uEmbeds"] = model.uEmbeds.grad.numpy().copy()
    out["g_cl1_image_trans"] = model.image_trans.grad.numpy().copy()
    model.cl_method = 0

    # ---- Denoise + GaussianDiffusion (diffmm.py:303-484)
    den = model.denoise_model_image
    for n, p in den.named_parameters():
        out["den_" + n.replace(".", "_")] = p.detach().numpy().copy()
    dm = model.diffusion_model
    for n in ["betas", "alphas_cumprod", "sqrt_alphas_cumprod", "sqrt_one_minus_alphas_cumprod",
              "posterior_mean_coef1", "posterior_mean_coef2", "posterior_variance",
              "posterior_log_variance_clipped"]:
        out["sched_" + n] = getattr(dm, n).numpy().astype(np.float64)
    Bd = 24
    x0 = np.zeros((Bd, I), np.float32)
    for b in range(Bd):
        x0[b, cols[rows == b]] = 1.0
    out["dif_x0"] = x0
    x0t = torch.from_numpy(x0)
    tq = torch.as_tensor(rng.integers(0, 5, size=Bd))
    with torch.no_grad():
        out["den_t"] = tq.numpy()
        out["den_out_eval"] = den(x0t, tq, mess_dropout=False).numpy()
    # training_losses under torch RNG, with the draws recovered by replaying the seed
    # (randint -> randn_like -> dropout bernoulli, diffmm.py:456-463,349-350)
    iE = model.getItemEmbeds().detach()
    feats = model.getImageFeats().detach()
    den.train()
    torch.manual_seed(1234)
    den.zero_grad()
    diff_loss, gc_loss = dm.training_losses(den, x0t, iE, torch.arange(Bd).float(), feats)
    (diff_loss.mean() + gc_loss.mean() * 0.5).backward()
    out["dif_diff_loss"], out["dif_gc_loss"] = diff_loss.detach().numpy(), gc_loss.detach().numpy()
    for n, p in den.named_parameters():
        out["dif_grad_" + n.replace(".", "_")] = p.grad.numpy().copy()
    torch.manual_seed(1234)
    ts = torch.randint(0, 5, (Bd,)).long()
    noise = torch.randn_like(x0t)
    keep = torch.empty_like(x0t).bernoulli_(0.5)
    out["dif_t"], out["dif_noise"], out["dif_keep"] = ts.numpy(), noise.numpy(), keep.numpy()
    out["dif_item_embeds"], out["dif_feats"] = iE.numpy(), feats.numpy()
    # p_sample + top-1 (diffmm.py:408-426, trainer.py:545-546)
    with torch.no_grad():
        xs = dm.p_sample(den, x0t, 0, False)
        out["psample_out"] = xs.numpy()
        out["psample_top1"] = torch.topk(xs, k=1)[1].numpy()

    # ---- full-rank eval (trainer.py:369-388) + metrics (topk_evaluator.py:77-120)
    eval_users = np.arange(0, U, 2)
    with torch.no_grad():
        scores = model.full_sort_predict([torch.as_tensor(eval_users)])
    out["eval_users"] = eval_users
    out["eval_scores_raw"] = scores.numpy().copy()
    mu, mi = [], []
    for r, u in enumerate(eval_users):
        its = cols[rows == u]
        mu.extend([r] * len(its))
        mi.extend(its.tolist())
    mu, mi = np.asarray(mu), np.asarray(mi)
    scores[mu, mi] = -1e10
    _, topk = torch.topk(scores, 50, dim=-1)
    out["eval_mask_rows"], out["eval_mask_cols"] = mu, mi
    out["eval_scores_masked"] = scores.numpy()
    out["eval_topk"] = topk.numpy()
    # eval positives: random held-out items not in train
    pos_lists = []
    for u in eval_users:
        cand = np.setdiff1d(np.arange(I), cols[rows == u])
        pos_lists.append(np.sort(rng.choice(cand, size=int(rng.integers(1, 4)), replace=False)))
    out["eval_pos_flat"] = np.concatenate(pos_lists)
    out["eval_pos_len"] = np.asarray([len(p) for p in pos_lists])
    metrics = _metrics(ref, topk.numpy(), pos_lists)
    return out, metrics


def _metrics(ref, topk, pos_lists, ks=(5, 10, 20, 50)):
    ev = ref["topk_evaluator"].TopKEvaluator(Cfg(metrics=["Recall", "NDCG", "Precision", "MAP"],
                                                  topk=list(ks), save_recommended_topk=False))

    class ED:
        def get_eval_items(self):
            return pos_lists

        def get_eval_len_list(self):
            return np.asarray([len(p) for p in pos_lists])

    rounded = ev.evaluate([__import__("torch").as_tensor(topk)], ED(), is_test=False)
    bool_rec = np.asarray([[i in m for i in n] for m, n in zip(pos_lists, topk)])
    raw = ev._calculate_metrics(np.asarray([len(p) for p in pos_lists]), bool_rec)
    return {"rounded": rounded, "raw": {m: raw[j].tolist() for j, m in
                                        enumerate(["recall", "ndcg", "precision", "map"])}}


def gen_metrics_edge(ref):
    """Metric edge cases: pos lists longer than K, all hits, no hits, single user."""
    rng = np.random.default_rng(3)
    topk = rng.integers(0, 500, size=(6, 50))
    pos = [np.arange(60) * 7 % 500, topk[1, :3].copy(), np.array([499]), topk[3].copy(),
           np.array([topk[4, 49]]), np.array([topk[5, 0], 999])]
    return {"topk": topk.tolist(), "pos": [p.tolist() for p in pos], "metrics": _metrics(ref, topk, pos)}


def gen_dataset(ref, tmp):
    """Dataset split + eval loaders (utils/dataset.py:65-82, utils/dataloader.py:330-416)."""
    import torch
    rng = np.random.default_rng(11)
    U, I = 53, 41
    lines = []
    for u in range(U):
        n = int(rng.integers(4, 14))
        items = rng.choice(I, size=n, replace=False)
        if n < 10:
            labels = [0] * (n - 2) + [1, 2]
        else:
            nt = int(n * 0.2) // 2
            labels = [0] * (n - 2 * nt) + [1] * nt + [2] * nt
        for it, lb in zip(items, labels):
            lines.append((u, int(it), lb))
    order = rng.permutation(len(lines))
    lines = [lines[i] for i in order]
    # a cold user that only appears in valid/test
    lines.append((U, 3, 1))
    lines.append((U, 4, 2))
    ddir = os.path.join(tmp, "tinyds")
    os.makedirs(ddir, exist_ok=True)
    with open(os.path.join(ddir, "tinyds.inter"), "w") as f:
        f.write("userID\titemID\tx_label\trating\n")
        for u, i, lb in lines:
            f.write(f"{u}\t{i}\t{lb}\t5\n")
    cfg = Cfg(dataset="tinyds", data_path=tmp + "/", USER_ID_FIELD="userID", ITEM_ID_FIELD="itemID",
              RATING_FIELD="rating", inter_splitting_label="x_label", field_separator="\t",
              inter_file_name="tinyds.inter", filter_out_cod_start_users=True, device=torch.device("cpu"),
              use_full_sampling=False, use_neg_sampling=True, use_neighborhood_loss=False)
    ds = ref["dataset"].RecDataset(cfg)
    str(ds)
    tr, va, te = ds.split()
    for part in (tr, va, te):  # quick_start.py:42-44 logs str(...), which sets inter_num
        str(part)
    out = {"inter": np.asarray(lines, np.int64), "user_num": ds.get_user_num(), "item_num": ds.get_item_num()}
    for name, part in [("valid", va), ("test", te)]:
        ed = ref["dataloader"].EvalDataLoader(cfg, part, additional_dataset=tr, batch_size=16)
        out[name + "_eval_u"] = ed.eval_u.numpy()
        out[name + "_mask"] = ed.pos_items_per_u.numpy()
        out[name + "_eval_len"] = ed.get_eval_len_list()
        out[name + "_eval_items"] = np.concatenate(ed.get_eval_items())
        batches = []
        for b in ed:
            batches.append((b[0].numpy(), b[1].numpy()))
        out[name + "_batch0_users"], out[name + "_batch0_mask"] = batches[0]
        out[name + "_nbatches"] = len(batches)
    tl = ref["dataloader"].TrainDataLoader(cfg, tr, batch_size=16, shuffle=True)
    m = tl.inter_matrix(form="coo")
    out["train_coo_rows"], out["train_coo_cols"] = m.row.astype(np.int64), m.col.astype(np.int64)
    out["train_len"] = len(tr)
    return out


def gen_diffrec(ref, tmp):
    import torch
    diffrec = ref["diffrec"]
    rng = np.random.default_rng(5)
    U, I, E, H, T = 40, 37, 16, 24, 10
    gd = diffrec.GaussianDiffusion("x0", "linear", 1e-4, 1e-4, 0.02, T, torch.device("cpu"))
    torch.manual_seed(5)
    dnn = diffrec.DNN([I, H], [H, I], E, norm=False, dropout=0.5)
    out = {"I": I, "E": E, "H": H, "T": T}
    for n in ["betas", "alphas_cumprod", "posterior_mean_coef1", "posterior_mean_coef2"]:
        out["sched_" + n] = getattr(gd, n).numpy()
    for n, p in dnn.named_parameters():
        out["dnn_" + n.replace(".", "_")] = p.detach().numpy().copy()
    x0 = (rng.random((U, I)) < 0.15).astype(np.float32)
    out["x0"] = x0
    dnn.eval()
    with torch.no_grad():
        out["psample"] = gd.p_sample(dnn, torch.from_numpy(x0), 0, False).numpy()
        t = torch.as_tensor(rng.integers(0, T, size=U))
        out["fwd_t"] = t.numpy()
        out["fwd_out"] = dnn(torch.from_numpy(x0), t).numpy()
    # training_losses(reweight=True) while the Lt histories fill (uniform t): draws replayed from
    # the seed (randint -> randn_like -> dropout bernoulli, diffrec.py:232-262, :80)
    dnn.train()
    xs = torch.from_numpy(x0)
    steps = []
    for s in range(12):
        if bool((gd.Lt_count == gd.history_num_per_term).all()):
            break
        torch.manual_seed(100 + s)
        for p_ in dnn.parameters():
            p_.grad = None
        terms = gd.training_losses(dnn, xs, reweight=True)
        terms["loss"].mean().backward()
        torch.manual_seed(100 + s)
        ts = torch.randint(0, T, (U,)).long()
        noise = torch.randn_like(xs)
        keep = torch.empty_like(xs).bernoulli_(0.5)
        rec = {"t": ts.numpy(), "noise": noise.numpy(), "keep": keep.numpy(),
               "loss": terms["loss"].detach().numpy().astype(np.float64),
               "hist": gd.Lt_history.numpy().copy(), "count": gd.Lt_count.numpy().astype(np.int64).copy()}
        if s == 0:
            for n, p_ in dnn.named_parameters():
                rec["g_" + n.replace(".", "_")] = p_.grad.numpy().copy()
        steps.append(rec)
    out["train_steps"] = len(steps)
    for s, rec in enumerate(steps):
        for k, v in rec.items():
            out[f"train{s}_{k}"] = v
    # importance sampling once every history is full (diffrec.py:234-250): pt = pt_all[t] * T
    assert bool((gd.Lt_count == gd.history_num_per_term).all())
    torch.manual_seed(7)
    it, ipt = gd.sample_timesteps(4000, torch.device("cpu"), "importance")
    out["imp_hist"] = gd.Lt_history.numpy().copy()
    out["imp_t"] = it.numpy()
    out["imp_pt"] = ipt.numpy()
    return out


def gen_vbpr(ref, tmp):
    import torch
    vbpr = ref["vbpr"]
    rng = np.random.default_rng(9)
    U, I, d, DV, DT = 33, 29, 64, 40, 24
    os.makedirs(os.path.join(tmp, "tv"), exist_ok=True)
    v = np.abs(rng.standard_normal((I, DV))).astype(np.float32)
    t = rng.standard_normal((I, DT)).astype(np.float32)
    np.save(os.path.join(tmp, "tv", "image_feat.npy"), v)
    np.save(os.path.join(tmp, "tv", "text_feat.npy"), t)
    rows, cols = make_interactions(rng, U, I)
    cfg = Cfg(USER_ID_FIELD="userID", ITEM_ID_FIELD="itemID", NEG_PREFIX="neg__", train_batch_size=16,
              device=torch.device("cpu"), end2end=False, is_multimodal_model=True, data_path=tmp + "/",
              dataset="tv", vision_feature_file="image_feat.npy", text_feature_file="text_feat.npy",
              embedding_size=d, reg_weight=2.0)
    torch.manual_seed(3)
    m = vbpr.VBPR(cfg, MockLoader(U, I, rows, cols))
    out = {"v_feat": v, "t_feat": t}
    for n, p in m.named_parameters():
        out["p_" + n.replace(".", "_")] = p.detach().numpy().copy()
    users = torch.as_tensor(rng.integers(0, U, 16))
    pos = torch.as_tensor(rng.integers(0, I, 16))
    neg = torch.as_tensor(rng.integers(0, I, 16))
    loss = m.calculate_loss(torch.stack([users, pos, neg]))
    loss.backward()
    out["users"], out["pos"], out["neg"] = users.numpy(), pos.numpy(), neg.numpy()
    out["loss"] = np.float32(loss.item())
    for n, p in m.named_parameters():
        out["g_" + n.replace(".", "_")] = p.grad.numpy().copy()
    with torch.no_grad():
        out["scores"] = m.full_sort_predict([torch.arange(U)]).numpy()
    return out


def gen_phases(ref, tmp):
    """D16 / D18: the reference's diffusion-phase loop (common/trainer.py:491-527) and BPR loop
    (:144-208) run on the tiny DiffMM of diffmm_tiny.npz with recorded draws / batches, for a
    phase-level parity test through the optimiser steps (tests/test_phases_gpu.py)."""
    import torch
    import torch.optim as optim
    diffmm = ref["diffmm"]
    g = dict(np.load(os.path.join(OUT, "diffmm_tiny.npz"), allow_pickle=False))
    U, I = int(g["U"]), int(g["I"])
    rows, cols = g["train_rows"], g["train_cols"]
    os.makedirs(os.path.join(tmp, "tiny"), exist_ok=True)
    np.save(os.path.join(tmp, "tiny", "image_feat.npy"), g["v_feat"])
    np.save(os.path.join(tmp, "tiny", "text_feat.npy"), g["t_feat"])
    cfg = Cfg(USER_ID_FIELD="userID", ITEM_ID_FIELD="itemID", NEG_PREFIX="neg__", train_batch_size=40,
              device=torch.device("cpu"), end2end=False, is_multimodal_model=True, data_path=tmp + "/",
              dataset="tiny", vision_feature_file="image_feat.npy", text_feature_file="text_feat.npy",
              embedding_size=64, n_layers=1, reg_weight=1e-6, ssl_reg=1e-2, temperature=0.1, keep_rate=1,
              dims=[32], d_emb_size=10, norm=False, steps=5, noise_scale=0.1, noise_min=1e-4, noise_max=0.02,
              sampling_noise=False, sampling_steps=0, rebuild_k=1, e_loss=0.5, ris_lambda=0.1,
              ris_adj_lambda=0.2, trans_type=0, cl_method=0)
    torch.manual_seed(999)
    model = diffmm.DiffMM(cfg, MockLoader(U, I, rows, cols))
    assert np.array_equal(model.uEmbeds.detach().numpy(), g["p_uEmbeds"])  # same model as diffmm_tiny
    out = {}
    for mod in ("image", "text"):
        for n, p in getattr(model, "denoise_model_" + mod).named_parameters():
            out[f"init_{mod}_" + n.replace(".", "_")] = p.detach().numpy().copy()
    # ---- D16: diffusion phase over all users in batches of 40 (permutation recorded)
    B = 40
    rng = np.random.default_rng(21)
    perm = rng.permutation(U)
    out["dif_perm"] = perm
    opt_i = optim.Adam(model.denoise_model_image.parameters(), lr=1e-3, weight_decay=0)
    opt_t = optim.Adam(model.denoise_model_text.parameters(), lr=1e-3, weight_decay=0)
    iE = model.getItemEmbeds().detach()
    feats_i = model.getImageFeats().detach()
    feats_t = model.getTextFeats().detach()
    model.train()
    dm = model.diffusion_model
    losses = []
    for b, lo in enumerate(range(0, U, B)):
        users = perm[lo:lo + B]
        x0 = np.zeros((len(users), I), np.float32)
        for r, u in enumerate(users):
            x0[r, cols[rows == u]] = 1.0
        xt = torch.from_numpy(x0)
        idx = torch.as_tensor(users).float()
        opt_i.zero_grad()
        opt_t.zero_grad()
        torch.manual_seed(700 + b)
        di, gi = dm.training_losses(model.denoise_model_image, xt, iE, idx, feats_i)
        dt, gt = dm.training_losses(model.denoise_model_text, xt, iE, idx, feats_t)
        li = di.mean() + gi.mean() * 0.5
        lt = dt.mean() + gt.mean() * 0.5
        (li + lt).backward()
        opt_i.step()
        opt_t.step()
        losses.append((li.item(), lt.item()))
        torch.manual_seed(700 + b)   # replay: randint, randn_like, dropout bernoulli for image, then text
        for mod in ("image", "text"):
            out[f"dif{b}_{mod}_t"] = torch.randint(0, 5, (len(users),)).long().numpy()
            out[f"dif{b}_{mod}_noise"] = torch.randn_like(xt).numpy()
            out[f"dif{b}_{mod}_keep"] = torch.empty_like(xt).bernoulli_(0.5).numpy()
    out["dif_batches"] = np.int64(len(losses))
    out["dif_losses"] = np.asarray(losses, np.float64)
    for mod in ("image", "text"):
        for n, p in getattr(model, "denoise_model_" + mod).named_parameters():
            out[f"final_{mod}_" + n.replace(".", "_")] = p.detach().numpy().copy()
    # ---- D18: BPR loop, three batches through Adam over model.parameters() (trainer.py:125-208)
    tr = object.__new__(ref["trainer"].DiffMMTrainer)
    tr.user_num, tr.item_num, tr.device = U, I, torch.device("cpu")
    ones = np.ones(U)
    model.image_UI_matrix = model.edgeDropper(tr.buildUIMatrix(np.arange(U), g["ui_img_items"], ones))
    model.text_UI_matrix = model.edgeDropper(tr.buildUIMatrix(np.arange(U), g["ui_txt_items"], ones))
    for name in ["uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight"]:
        out["bpr_init_" + name] = getattr(model, name).detach().numpy().copy()
    opt = optim.Adam(model.parameters(), lr=1e-3, weight_decay=0.0)
    bl = []
    for s_ in range(3):
        inter = torch.as_tensor(np.stack([rng.integers(0, U, B), rng.integers(0, I, B), rng.integers(0, I, B)]))
        out[f"bpr{s_}_inter"] = inter.numpy()
        opt.zero_grad()
        loss = model.calculate_loss(inter)
        loss.backward()
        opt.step()
        bl.append(loss.item())
    out["bpr_losses"] = np.asarray(bl, np.float64)
    for name in ["uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight"]:
        out["bpr_final_" + name] = getattr(model, name).detach().numpy().copy()
    out.update(gen_csv(ref, tmp))
    return out


def gen_csv(ref, tmp):
    """The top-K CSV the reference writes on a test evaluation (utils/topk_evaluator.py:93-106) and the
    test-time extras it returns next to it (pop / niche, cold / warm, coverage / gini / tail)."""
    import glob
    import torch
    rng = np.random.default_rng(33)
    n, k, I = 9, 50, 80
    topk = np.stack([rng.permutation(I)[:k] for _ in range(n)])
    users = np.array([5, 2, 11, 7, 3, 30, 1, 8, 4])
    pos = [np.sort(rng.choice(I, size=int(rng.integers(1, 6)), replace=False)) for _ in range(n)]
    d = os.path.join(tmp, "topk_csv")
    cfg = Cfg(metrics=["Recall", "NDCG", "Precision", "MAP"], topk=[5, 10, 20, 50], save_recommended_topk=True,
              recommend_topk=d, dataset="tiny", model="DiffMM", pop_items=set(range(0, I, 3)),
              warm_users={5, 7, 30, 4})

    class DS:
        item_num = I

    class ED:
        dataset = DS()

        def get_eval_items(self):
            return pos

        def get_eval_len_list(self):
            return np.asarray([len(p) for p in pos])

        def get_eval_users(self):
            return torch.as_tensor(users)

    res = ref["topk_evaluator"].TopKEvaluator(cfg).evaluate([torch.as_tensor(topk)], ED(), is_test=True, idx=0)
    files = glob.glob(os.path.join(d, "*.csv"))
    assert len(files) == 1
    with open(files[0]) as f:
        text = f.read()
    return {"csv_topk": topk, "csv_users": users, "csv_pos_flat": np.concatenate(pos),
            "csv_pos_len": np.asarray([len(p) for p in pos]), "csv_text": np.array(text),
            "csv_name": np.array(os.path.basename(files[0])), "csv_extras_json": np.array(json.dumps(res))}


def main():
    ref = _import_reference()
    if "--phases" in sys.argv:  # only the phase-level fixture (the others stay as committed)
        with tempfile.TemporaryDirectory(dir=os.path.join(os.path.dirname(os.path.dirname(OUT)), ".golden_tmp")
                                         if os.path.isdir(os.path.join(os.path.dirname(os.path.dirname(OUT)),
                                                                       ".golden_tmp")) else None) as tmp:
            np.savez_compressed(os.path.join(OUT, "diffmm_phases_tiny.npz"), **gen_phases(ref, tmp))
        print("wrote", os.path.join(OUT, "diffmm_phases_tiny.npz"))
        return
    import torch
    meta = {"torch": torch.__version__, "numpy": np.__version__, "reference": REF_SRC,
            "generator": "tests/golden/make_golden.py"}
    with tempfile.TemporaryDirectory() as tmp:
        dm, dm_metrics = gen_diffmm(ref, tmp)
        np.savez_compressed(os.path.join(OUT, "diffmm_tiny.npz"), **dm)
        ds = gen_dataset(ref, tmp)
        np.savez_compressed(os.path.join(OUT, "dataset_tiny.npz"), **ds)
        dr = gen_diffrec(ref, tmp)
        np.savez_compressed(os.path.join(OUT, "diffrec_tiny.npz"), **dr)
        vb = gen_vbpr(ref, tmp)
        np.savez_compressed(os.path.join(OUT, "vbpr_tiny.npz"), **vb)
    meta["diffmm_metrics"] = dm_metrics
    meta["metrics_edge"] = gen_metrics_edge(ref)
    with open(os.path.join(OUT, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, default=float)
    print("wrote fixtures to", OUT)


if __name__ == "__main__":
    main()
