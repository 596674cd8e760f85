"""Baby-shape golden vectors from the reference ("a few baby-shape spot checks").

Runs ONLY in the build container: it imports the reference from /root/reference (read-only,
through make_golden._import_reference) and writes small fixtures:
  tests/golden/diffmm_baby.npz        top-k index/value arrays (int16 / fp32)
  tests/golden/diffmm_baby_meta.json  parameter digests, metric curves and dicts

Inputs are the SURVEY.md 8d synthetic Amazon-baby data of gmr/synthetic.py (seed 0: 19,445
users x 7,050 items, image 4096-d, text 384-d), written as the reference's on-disk format
(<data_path>/baby/baby.inter + image_feat.npy / text_feat.npy) and read back by the reference's
own RecDataset / TrainDataLoader / EvalDataLoader; the model is the reference DiffMM with the
repository's DiffMM.yaml + baby.yaml + overall.yaml (H = 1000), seeded as quick_start does
(utils.init_seed(999), quick_start.py:171-176).

Reference code exercised (paths relative to GenMMRec/src):
  models/diffmm.py:14-86         __init__: parameter init order (digests)
  models/diffmm.py:408-426       GaussianDiffusion.p_sample (steps 0, no noise), both denoisers
  common/trainer.py:529-576      graph rebuild: topk(k = rebuild_k = 1) + buildUIMatrix + edgeDropper
  models/diffmm.py:260-278       full_sort_predict
  common/trainer.py:369-388      evaluate: mask train items with -1e10, topk(50)
  utils/topk_evaluator.py:77-270 TopKEvaluator.evaluate (valid: is_test False; test: is_test True
                                 with pop / niche, warm / cold and coverage / gini / tail extras)
  utils/quick_start.py:46-102    pop_items (top 20 % train items) and warm users (> 5 train inter.)

Usage:  python tests/golden/make_golden_baby.py [baby|sports|diffrec|diffrec_train|diffmm_train|vbpr]
  baby   (default) -> diffmm_baby.npz / diffmm_baby_meta.json, about a minute on 8 cores
  sports (config 4: 35,598 users x 18,357 items) -> diffmm_sports.npz / _meta.json:
         the same checks on the valid split only (the is_test extras are pinned at baby), a few
         minutes on 8 cores
  diffrec (config 2: DiffRec.yaml at the baby shape) -> diffrec_baby.npz / _meta.json: the seed-999
         DNN init digests (models/diffrec.py:313-353), the valid split's full_sort_predict = the
         100-step p_sample (:291-310, :372-388) -> mask -> top-50, and the unrounded metrics;
         about two minutes on 8 cores
  diffrec_train -> diffrec_baby_train.npz / _meta.json: three training calls at the baby shape
         (main_diffrec_train's docstring)
  diffmm_train -> diffmm_baby_train.npz / _meta.json: one diffusion step per denoiser and one rec step at
         the baby shape with the reference's draws / batch (main_diffmm_train's docstring), ~30 s
  diffmm_train_sports -> diffmm_sports_train.npz / _meta.json: the same at config 4's sports shape, ~2 min
  vbpr   (config 1) -> vbpr_baby.npz / _meta.json: VBPR init digests, one loss + backward, valid top-50 +
         metrics, each also in fp64 (main_vbpr's docstring), about a minute
"""
import hashlib
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

from make_golden import REF_SRC, _import_reference  # noqa: E402

TMP = os.path.join(ROOT, ".golden_tmp")  # git- and gpurun-ignored scratch for the on-disk dataset
SAMPLE = 2048                            # users whose full top-50 score rows are stored


def digest(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    return hashlib.sha256(a.tobytes()).hexdigest()


def write_dataset(path, shape="baby"):
    """The shape's synthetic data in the reference's on-disk layout, under the dataset name the
    reference's configs know (sports-shaped data is written as 'sports': configs/dataset/sports.yaml)."""
    from gmr.synthetic import SHAPES, make_features, make_interactions
    U, I, n, dv, dt = SHAPES[shape]
    u, i, lb = make_interactions(U, I, n, 0)
    v, t = make_features(I, dv, dt, 0)
    d = os.path.join(path, shape)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, f"{shape}.inter"), "w") as f:
        f.write("userID\titemID\tx_label\trating\n")
        for a, b, c in zip(u.tolist(), i.tolist(), lb.tolist()):
            f.write(f"{a}\t{b}\t{c}\t5\n")
    np.save(os.path.join(d, "image_feat.npy"), v)
    np.save(os.path.join(d, "text_feat.npy"), t)


def reference_config(ref_mods, shape="baby"):
    import utils.configurator as configurator
    cwd = os.getcwd()
    os.chdir(REF_SRC)  # the reference's Config reads ./configs (utils/configurator.py:72-76)
    try:
        cfg = configurator.Config("DiffMM", shape, {"use_gpu": False, "data_path": TMP + "/", "epochs": 1,
                                                    "save_recommended_topk": False})
    finally:
        os.chdir(cwd)
    return cfg


def _reference_diffrec():
    """The reference DiffRec at the baby shape after init_seed(999), as quick_start builds it."""
    ref = _import_reference()
    import torch
    import utils.configurator as configurator
    import utils.utils as rutils
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if os.path.isdir(TMP):
        shutil.rmtree(TMP)
    write_dataset(TMP, "baby")
    cwd = os.getcwd()
    os.chdir(REF_SRC)
    try:
        cfg = configurator.Config("DiffRec", "baby", {"use_gpu": False, "data_path": TMP + "/", "epochs": 1,
                                                      "save_recommended_topk": False})
    finally:
        os.chdir(cwd)
    ds = ref["dataset"].RecDataset(cfg)
    tr, va, te = ds.split()
    for part in (tr, va, te):
        str(part)
    tl = ref["dataloader"].TrainDataLoader(cfg, tr, batch_size=cfg["train_batch_size"], shuffle=True)
    vl = ref["dataloader"].EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=cfg["eval_batch_size"])
    rutils.init_seed(999)
    tl.pretrain_setup()
    model = ref["diffrec"].DiffRec(cfg, tl)
    return ref, cfg, tr, tl, vl, model


def main_diffrec():
    import torch
    ref, cfg, tr, tl, vl, model = _reference_diffrec()
    meta = {"U": model.n_users, "I": model.n_items, "n_train": len(tr), "torch": torch.__version__,
            "numpy": np.__version__, "generator": "tests/golden/make_golden_baby.py diffrec", "reference": REF_SRC,
            "steps": int(cfg["steps"]),
            "param_sha256": {n: digest(p.detach().numpy()) for n, p in model.model.named_parameters()}}
    ev = ref["topk_evaluator"].TopKEvaluator(cfg)
    kmax = max(cfg["topk"])
    model.eval()
    mats, vals = [], []
    with torch.no_grad():
        for batch in vl:
            scores = model.full_sort_predict(batch)
            m = batch[1]
            scores[m[0], m[1]] = -1e10
            v, ix = torch.topk(scores, kmax, dim=-1)
            mats.append(ix)
            vals.append(v)
    topk = torch.cat(mats).numpy()
    out = {"valid_top50": topk.astype(np.int16), "valid_top50_val_sample": torch.cat(vals)[:SAMPLE].numpy()}
    res = ev.evaluate([torch.as_tensor(topk)], vl, is_test=False)
    pos = vl.get_eval_items()
    bool_rec = np.asarray([[i in p for i in row] for p, row in zip(pos, topk)])
    raw = ev._calculate_metrics(vl.get_eval_len_list(), bool_rec)
    meta["valid"] = {"n_users": int(len(topk)), "rounded": res,
                     "raw": {mname: np.asarray(raw[j], np.float64).tolist()
                             for j, mname in enumerate(["recall", "ndcg", "precision", "map"])}}
    np.savez_compressed(os.path.join(HERE, "diffrec_baby.npz"), **out)
    with open(os.path.join(HERE, "diffrec_baby_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, default=float)
    shutil.rmtree(TMP)
    print("wrote", os.path.join(HERE, "diffrec_baby.npz"))


def main_diffrec_train():
    """DiffRec training at the baby shape (VERDICT r3 missing #6): three calculate_loss + backward calls
    (models/diffrec.py:355-368 -> training_losses :252-289) on the reference loader's first batch from
    the seed-999 init (no optimiser step between them).  Calls 0 and 1 run while the Lt histories fill
    (uniform t, pt = 1); call 2, with every history full, draws t by importance (:234-250).  The
    2,048 x 7,050 noise and dropout draws are too large to store: each call is seeded
    (torch.manual_seed(100 + s)) and the test replays the reference's draw order on the CPU (t, then
    randn_like(x_start) :255, then the dropout's bernoulli :80); the replay is checked here against the
    draws the reference actually made (captured) and its SHA-256 is stored for the test to check its
    own replay.  Stored: users, t, pt, pt_all, per-row losses, Lt_history / Lt_count after each call and
    the gradients (whole for the small tensors; row / column sums and 4,096 sampled entries of W1 / W2).
    """
    import torch
    ref, cfg, tr, tl, vl, model = _reference_diffrec()
    gd, dnn = model.diffusion, model.model
    users = next(iter(tl))[0].clone()
    B, I, T = users.numel(), model.n_items, model.steps
    meta = {"U": model.n_users, "I": I, "n_train": len(tr), "B": int(B), "steps": int(T), "torch": torch.__version__,
            "numpy": np.__version__, "generator": "tests/golden/make_golden_baby.py diffrec_train",
            "reference": REF_SRC, "calls": []}
    out = {"users": users.numpy().astype(np.int32)}
    rs = np.random.default_rng(17)
    big = {"in_layers.0.weight", "out_layers.0.weight"}
    pick = {n: rs.integers(0, p.numel(), 4096) for n, p in dnn.named_parameters() if n in big}
    for n, ix in pick.items():
        out["pick_" + n.replace(".", "_")] = ix.astype(np.int64)
    orig_randn_like = torch.randn_like
    cap = {}

    def randn_like(x, *a, **k):
        r = orig_randn_like(x, *a, **k)
        cap["noise"] = r.clone()
        return r
    hook = dnn.drop.register_forward_hook(lambda mod, i, o: cap.update(drop_in=i[0].detach().clone(),
                                                                        drop_out=o.detach().clone()))
    dnn.train()
    for s in range(3):
        full = bool((gd.Lt_count == gd.history_num_per_term).all())
        pt_all = None
        if full:
            Lt_sqrt = torch.sqrt(torch.mean(gd.Lt_history ** 2, axis=-1))
            pt_all = Lt_sqrt / torch.sum(Lt_sqrt)
            pt_all *= 1 - 0.001
            pt_all += 0.001 / len(pt_all)
        for p_ in dnn.parameters():
            p_.grad = None
        torch.manual_seed(100 + s)
        torch.randn_like = randn_like
        try:
            loss = model.calculate_loss([users])
        finally:
            torch.randn_like = orig_randn_like
        loss.backward()
        # replay (what the test does) and compare with the captured draws
        torch.manual_seed(100 + s)
        if full:
            ts = torch.multinomial(pt_all, num_samples=B, replacement=True)
            pt = pt_all.gather(dim=0, index=ts) * len(pt_all)
        else:
            ts = torch.randint(0, T, (B,)).long()
            pt = torch.ones_like(ts).float()
        noise = torch.randn(B, I)
        keep = torch.empty(B, I).bernoulli_(1 - dnn.drop.p)
        assert torch.equal(noise, cap["noise"]), "noise replay differs from the reference's draw"
        want = cap["drop_in"] * keep / (1 - dnn.drop.p)
        assert torch.equal(want, cap["drop_out"]), "dropout replay differs from the reference's draw"
        # the reference's per-row loss of this call: weight * mse / pt (training_losses :263-288)
        x0 = torch.from_numpy(model.interaction_csr[users.numpy()].toarray()).float()
        with torch.no_grad():
            xt = gd.q_sample(x0, ts, noise)
            h = torch.cat([xt * keep / (1 - dnn.drop.p), dnn.emb_layer(
                ref["diffrec"].timestep_embedding(ts, dnn.time_emb_dim))], dim=-1)
            o = dnn.out_layers[0](torch.tanh(dnn.in_layers[0](h)))
            mse = ((x0 - o) ** 2).mean(dim=1)
            wgt = gd.SNR(ts - 1) - gd.SNR(ts)
            wgt = torch.where(ts == 0, torch.tensor(1.0), wgt)
            rows = (wgt * mse / pt).double()
        np.testing.assert_allclose(rows.mean().item(), loss.item(), rtol=1e-6)
        c = f"call{s}_"
        out[c + "t"] = ts.numpy().astype(np.int16)
        out[c + "pt"] = pt.numpy().astype(np.float32)
        if pt_all is not None:
            out[c + "pt_all"] = pt_all.numpy()
        out[c + "loss_rows"] = rows.numpy()
        out[c + "hist"] = gd.Lt_history.numpy().copy()
        out[c + "count"] = gd.Lt_count.numpy().astype(np.int64).copy()
        for n, p_ in dnn.named_parameters():
            g = p_.grad.detach().numpy().astype(np.float32)
            k = c + "g_" + n.replace(".", "_")
            if n in big:
                out[k + "_rowsum"] = g.sum(1, dtype=np.float64)
                out[k + "_colsum"] = g.sum(0, dtype=np.float64)
                out[k + "_pick"] = g.reshape(-1)[pick[n]]
            else:
                out[k] = g
        meta["calls"].append({"seed": 100 + s, "importance": full, "loss": float(loss.item()),
                              "noise_sha256": hashlib.sha256(noise.numpy().tobytes()).hexdigest(),
                              "keep_sha256": hashlib.sha256(keep.numpy().tobytes()).hexdigest()})
    hook.remove()
    np.savez_compressed(os.path.join(HERE, "diffrec_baby_train.npz"), **out)
    with open(os.path.join(HERE, "diffrec_baby_train_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, default=float)
    shutil.rmtree(TMP)
    print("wrote", os.path.join(HERE, "diffrec_baby_train.npz"), meta["calls"])


def _grad_record(out, key, g, pick):
    """A gradient tensor as a fixture: whole when small, else fp64 row / column sums plus the entries
    at `pick` (flat indices), the way diffrec_baby_train.npz stores W1 / W2."""
    g = np.ascontiguousarray(g, dtype=np.float32)
    if g.size <= 32768:
        out[key] = g
        return
    g2 = g.reshape(g.shape[0], -1)
    out[key + "_rowsum"] = g2.sum(1, dtype=np.float64)
    out[key + "_colsum"] = g2.sum(0, dtype=np.float64)
    out[key + "_pick"] = g2.reshape(-1)[pick]


def _reference_diffmm(shape="baby"):
    """The reference DiffMM at `shape` after init_seed(999), built as quick_start builds it."""
    ref = _import_reference()
    import torch
    import utils.utils as rutils
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if os.path.isdir(TMP):
        shutil.rmtree(TMP)
    write_dataset(TMP, shape)
    cfg = reference_config(ref, shape)
    ds = ref["dataset"].RecDataset(cfg)
    tr, va, te = ds.split()
    for part in (tr, va, te):
        str(part)
    tl = ref["dataloader"].TrainDataLoader(cfg, tr, batch_size=cfg["train_batch_size"], shuffle=True)
    rutils.init_seed(999)
    tl.pretrain_setup()
    model = ref["diffmm"].DiffMM(cfg, tl)
    return ref, cfg, tr, tl, model


def main_diffmm_train(shape="baby"):
    """DiffMM training at the baby shape (VERDICT r4 missing #1) or, with shape = "sports", at config 4's
    35,598 x 18,357 shape (VERDICT r5 missing #3), from the seed-999 init:

    diffusion  one step of the reference's diffusion loop (common/trainer.py:505-527) on 2,048 users
               (the first 2,048 of a seeded permutation, x0 = their train rows as the DiffusionDataset
               builds them): training_losses (models/diffmm.py:453-477) of the image denoiser, then of
               the text denoiser, under one torch seed, and the backward of loss_image + loss_text
               (e_loss-weighted gc terms).  The draws (randint t, randn_like noise, the Denoise input
               dropout's bernoulli - image first, then text) are replayed on the CPU from the seed and
               compared with what the reference drew (captured); their SHA-256 is stored so the test can
               check its own replay.  Stored: users, t per denoiser, per-row diff / gc losses, every
               denoiser gradient (whole when small, else row / column sums + 4,096 sampled entries).
    rec step   calculate_loss (models/diffmm.py:203-249) + backward on the reference loader's first
               2,048-row batch, with the UI graphs built from the reference's own top-1 p_sample edges
               (diffmm_<shape>.npz, trainer.py:545-576): loss, its parts, and every rec gradient.
    Round 6: the reference's own image / text feats of the diffusion step (getImageFeats / getTextFeats,
    models/diffmm.py:115-127) are stored too, so the test can feed the denoiser step exactly the reference's
    inputs (the gc loss rows then compare the diffusion kernels alone, not the projection GEMM's rounding).
    """
    import torch
    ref, cfg, tr, tl, model = _reference_diffmm(shape)
    U, I = model.n_users, model.n_items
    B = int(cfg["train_batch_size"])
    e_loss = float(cfg["e_loss"])
    dm = model.diffusion_model
    meta = {"U": U, "I": I, "n_train": len(tr), "B": B, "e_loss": e_loss, "torch": torch.__version__,
            "numpy": np.__version__, "generator": f"tests/golden/make_golden_baby.py diffmm_train {shape}",
            "reference": REF_SRC, "shape": shape}
    out = {}
    rs = np.random.default_rng(31)
    users = rs.permutation(U)[:B]
    out["dif_users"] = users.astype(np.int32)
    uid, iid = cfg["USER_ID_FIELD"], cfg["ITEM_ID_FIELD"]
    inter = tr.df.groupby(uid)[iid].apply(list).to_dict()
    x0 = torch.zeros(B, I)
    for r, u in enumerate(users.tolist()):
        it = inter.get(u, [])
        if it:
            x0[r, it] = 1.0
    iE = model.getItemEmbeds().detach()
    feats = {"image": model.getImageFeats().detach(), "text": model.getTextFeats().detach()}
    for m in feats:
        out[f"dif_feats_{m}"] = feats[m].numpy().astype(np.float32)
    dens = {m: getattr(model, "denoise_model_" + m) for m in ("image", "text")}
    picks = {}
    for mod, den in dens.items():
        for n, p in den.named_parameters():
            if p.numel() > 32768:
                picks[(mod, n)] = rs.integers(0, p.numel(), 4096)
                out[f"dif_pick_{mod}_" + n.replace(".", "_")] = picks[(mod, n)].astype(np.int64)
    # capture the draws the reference makes (randn_like in training_losses, the dropout in Denoise)
    orig_randn_like = torch.randn_like
    cap = {"noise": [], "drop": []}

    def randn_like(x, *a, **k):
        r = orig_randn_like(x, *a, **k)
        cap["noise"].append(r.clone())
        return r
    hooks = [den.drop.register_forward_hook(lambda mod_, i, o: cap["drop"].append((i[0].detach().clone(),
                                                                                   o.detach().clone())))
             for den in dens.values()]
    model.train()
    for den in dens.values():
        den.zero_grad()
    seed = 4242
    torch.manual_seed(seed)
    torch.randn_like = randn_like
    try:
        res = {m: dm.training_losses(dens[m], x0, iE, torch.as_tensor(users).float(), feats[m])
               for m in ("image", "text")}
    finally:
        torch.randn_like = orig_randn_like
    for h in hooks:
        h.remove()
    lossd = {m: res[m][0].mean() + res[m][1].mean() * e_loss for m in res}
    (lossd["image"] + lossd["text"]).backward()
    # replay (what the test does) and compare with the captured draws
    torch.manual_seed(seed)
    meta["diffusion"] = {"seed": seed}
    for j, mod in enumerate(("image", "text")):
        p = dens[mod].drop.p
        ts = torch.randint(0, dm.steps, (B,)).long()
        noise = torch.randn(B, I)
        keep = torch.empty(B, I).bernoulli_(1 - p)
        assert torch.equal(noise, cap["noise"][j]), "noise replay differs from the reference's draw"
        d_in, d_out = cap["drop"][j]
        assert torch.equal(d_in * keep / (1 - p), d_out), "dropout replay differs from the reference's draw"
        # the per-row diff loss recomputed from the replayed draws equals the reference's
        with torch.no_grad():
            xt = dm.q_sample(x0, ts, noise)
            assert torch.equal(xt, d_in), "x_t replay differs"
        out[f"dif_{mod}_t"] = ts.numpy().astype(np.int8)
        out[f"dif_{mod}_diff_rows"] = res[mod][0].detach().numpy().astype(np.float64)
        out[f"dif_{mod}_gc_rows"] = res[mod][1].detach().numpy().astype(np.float64)
        meta["diffusion"][mod] = {"loss": float(lossd[mod].item()), "keep_prob": 1 - p,
                                  "noise_sha256": hashlib.sha256(noise.numpy().tobytes()).hexdigest(),
                                  "keep_sha256": hashlib.sha256(keep.numpy().tobytes()).hexdigest()}
        for n, p_ in dens[mod].named_parameters():
            _grad_record(out, f"dif_g_{mod}_" + n.replace(".", "_"), p_.grad.detach().numpy(), picks.get((mod, n)))
        # the same step evaluated in float64 (round 6): the reference's parameters, inputs and draws widened (the
        # fp32 schedule coefficients and time embedding as the reference computes them), so the per-row diff / gc
        # losses have a truth that both the reference's fp32 run and the HIP path are measured against
        import copy
        den64 = copy.deepcopy(dens[mod]).double()
        den64.emb_layer.register_forward_pre_hook(lambda m_, a: (a[0].double(),))
        keep64 = keep.double()
        den64.drop.register_forward_hook(lambda m_, i, o, k=keep64, q=p: i[0] * k / (1 - q))
        orig_randint = torch.randint
        rng_state = torch.get_rng_state()  # (the widened Dropout still draws: the replay loop's stream is kept)
        torch.randn_like = lambda x, *a, **k: noise.double()
        torch.randint = lambda *a, **k: ts.clone()
        try:
            cap64 = []
            hz = den64.register_forward_hook(lambda m_, i, o: cap64.append(o.detach().clone()))
            with torch.no_grad():
                d64, g64 = dm.training_losses(den64, x0.double(), iE.double(), torch.as_tensor(users).double(),
                                              feats[mod].double())
            hz.remove()
            # Z = out @ feats (the gc term's model embeddings) and 4,096 sampled entries of the output, in fp64
            out[f"dif_{mod}_Z64"] = (cap64[0] @ feats[mod].double()).numpy()
            out[f"dif_{mod}_out64_pick"] = cap64[0].reshape(-1).numpy()[out[f"dif_pick_{mod}_out_layers_0_weight"]]
        finally:
            torch.randn_like = orig_randn_like
            torch.randint = orig_randint
            torch.set_rng_state(rng_state)
        out[f"dif_{mod}_diff_rows64"] = d64.numpy().astype(np.float64)
        out[f"dif_{mod}_gc_rows64"] = g64.numpy().astype(np.float64)
        rel = lambda a, b: float(np.max(np.abs(a - b) / np.abs(b)))  # noqa: E731
        meta["diffusion"][mod]["fp32_vs_fp64_rel"] = {"diff_rows": rel(out[f"dif_{mod}_diff_rows"], d64.numpy()),
                                                      "gc_rows": rel(out[f"dif_{mod}_gc_rows"], g64.numpy())}
    # ---- rec step on the reference's UI graphs (its own top-1 edges, diffmm_baby.npz)
    gb = np.load(os.path.join(HERE, f"diffmm_{shape}.npz"), allow_pickle=False)
    rb = object.__new__(ref["trainer"].DiffMMTrainer)
    rb.user_num, rb.item_num, rb.device = U, I, torch.device("cpu")
    ones = np.ones(U)
    with torch.no_grad():
        for mod in ("image", "text"):
            top1 = gb[f"psample_{mod}_top5_idx"][:, 0].astype(np.int64)
            setattr(model, mod + "_UI_matrix", model.edgeDropper(rb.buildUIMatrix(np.arange(U), top1, ones)))
    batch = next(iter(tl))
    out["bpr_inter"] = batch.numpy().astype(np.int32)
    model.zero_grad()
    loss = model.calculate_loss(batch)
    loss.backward()
    with torch.no_grad():
        ue, ie = model.forward_MM(model.norm_adj, model.image_UI_matrix, model.text_UI_matrix)
        a, p_, n_ = ue[batch[0]], ie[batch[1]], ie[batch[2]]
        bpr = -torch.log(1e-10 + torch.sigmoid((a * p_).sum(1) - (a * n_).sum(1))).mean()
        u1, i1, u2, i2 = model.forward_cl_MM(model.norm_adj, model.image_UI_matrix, model.text_UI_matrix)
        clu = model.contrastLoss(u1, u2, batch[0], model.temp)
        cli = model.contrastLoss(i1, i2, batch[1], model.temp)
    meta["rec"] = {"loss": float(loss.item()), "bpr": float(bpr.item()), "reg": float(model.reg_loss().item()
                                                                                      * model.reg_weight),
                   "cl_user": float(clu.item()), "cl_item": float(cli.item()), "ssl_reg": float(model.ssl_reg)}
    for name in ["uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight"]:
        g = getattr(model, name).grad.detach().numpy()
        pk = rs.integers(0, g.size, 4096) if g.size > 32768 else None
        if pk is not None:
            out["rec_pick_" + name] = pk.astype(np.int64)
        _grad_record(out, "rec_g_" + name, g, pk)
        # the batch's own rows (users of the batch / its positive items) in full, 256 of each
    gu = model.uEmbeds.grad.detach().numpy()
    gi = model.iEmbeds.grad.detach().numpy()
    out["rec_g_uEmbeds_rows"] = gu[batch[0][:256].numpy()].astype(np.float32)
    out["rec_g_iEmbeds_rows"] = gi[batch[1][:256].numpy()].astype(np.float32)
    np.savez_compressed(os.path.join(HERE, f"diffmm_{shape}_train.npz"), **out)
    with open(os.path.join(HERE, f"diffmm_{shape}_train_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, default=float)
    shutil.rmtree(TMP)
    print("wrote", os.path.join(HERE, f"diffmm_{shape}_train.npz"), meta["diffusion"], meta["rec"])


def main_vbpr():
    """Config 1 - VBPR at the baby shape (VERDICT r4 missing #2; models/vbpr.py:20-106 with VBPR.yaml:
    embedding 64, reg_weight 2.0), built as quick_start builds it after init_seed(999):
      * SHA-256 of every parameter (the RNG order of vbpr.py:31-45 and xavier_normal_initialization);
      * calculate_loss + backward on the reference loader's first 2,048-row batch (vbpr.py:76-97):
        the loss and every gradient (whole when small, else row / column sums + sampled entries);
      * the valid split's full_sort_predict (vbpr.py:99-104) -> mask -> top-50 (trainer.py:369-388),
        the top-50 scores of a user sample, and the unrounded Recall/NDCG/Precision/MAP.
    """
    ref = _import_reference()
    import importlib
    import torch
    import utils.configurator as configurator
    import utils.utils as rutils
    vbpr = importlib.import_module("models.vbpr")
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if os.path.isdir(TMP):
        shutil.rmtree(TMP)
    write_dataset(TMP, "baby")
    cwd = os.getcwd()
    os.chdir(REF_SRC)
    try:
        cfg = configurator.Config("VBPR", "baby", {"use_gpu": False, "data_path": TMP + "/", "epochs": 1,
                                                   "save_recommended_topk": False})
    finally:
        os.chdir(cwd)
    ds = ref["dataset"].RecDataset(cfg)
    tr, va, te = ds.split()
    for part in (tr, va, te):
        str(part)
    tl = ref["dataloader"].TrainDataLoader(cfg, tr, batch_size=cfg["train_batch_size"], shuffle=True)
    vl = ref["dataloader"].EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=cfg["eval_batch_size"])
    rutils.init_seed(999)
    tl.pretrain_setup()
    model = vbpr.VBPR(cfg, tl)
    meta = {"U": model.n_users, "I": model.n_items, "n_train": len(tr), "torch": torch.__version__,
            "numpy": np.__version__, "generator": "tests/golden/make_golden_baby.py vbpr", "reference": REF_SRC,
            "reg_weight": float(cfg["reg_weight"]), "train_batch_size": int(cfg["train_batch_size"]),
            "param_sha256": {n: digest(p.detach().numpy()) for n, p in model.named_parameters()}}
    out = {}
    rs = np.random.default_rng(41)
    batch = next(iter(tl))
    out["inter"] = batch.numpy().astype(np.int32)
    model.zero_grad()
    loss = model.calculate_loss(batch)
    loss.backward()
    meta["loss"] = float(loss.item())
    for n, p in model.named_parameters():
        g = p.grad.detach().numpy()
        pk = rs.integers(0, g.size, 4096) if g.size > 32768 else None
        if pk is not None:
            out["pick_" + n.replace(".", "_")] = pk.astype(np.int64)
        _grad_record(out, "g_" + n.replace(".", "_"), g, pk)
    ev = ref["topk_evaluator"].TopKEvaluator(cfg)
    kmax = max(cfg["topk"])

    def valid_eval(tag):
        model.eval()
        mats, vals = [], []
        with torch.no_grad():
            for b in vl:
                scores = model.full_sort_predict(b)
                m = b[1]
                scores[m[0], m[1]] = -1e10
                v, ix = torch.topk(scores, kmax, dim=-1)
                mats.append(ix)
                vals.append(v)
        topk = torch.cat(mats).numpy()
        out[f"valid_top50{tag}"] = topk.astype(np.int16)
        out[f"valid_top50_val_sample{tag}"] = torch.cat(vals)[:SAMPLE].numpy().astype(np.float32)
        res = ev.evaluate([torch.as_tensor(topk)], vl, is_test=False)
        pos = vl.get_eval_items()
        bool_rec = np.asarray([[i in p for i in row] for p, row in zip(pos, topk)])
        raw = ev._calculate_metrics(vl.get_eval_len_list(), bool_rec)
        meta[f"valid{tag}"] = {"n_users": int(len(topk)), "rounded": res,
                               "raw": {mname: np.asarray(raw[j], np.float64).tolist()
                                       for j, mname in enumerate(["recall", "ndcg", "precision", "map"])}}
        return res
    res = valid_eval("")
    # the same reference calls in fp64 (model.double(): the same parameters, widened): the reference's fp32
    # loss is 2.1e-5 off its own fp64 value (EmbLoss's fp32 torch.norm over 2,048 x 128-wide rows of the
    # 4,480-term item projection), so the HIP path is pinned to the fp64 values, the fp32 ones recorded beside
    model.double()
    model.item_raw_features = model.item_raw_features.double()
    model.train()
    model.zero_grad()
    loss64 = model.calculate_loss(batch)
    loss64.backward()
    meta["loss64"] = float(loss64.item())
    for n, p in model.named_parameters():
        g = p.grad.detach().numpy()
        k = n.replace(".", "_")
        _grad_record(out, "g64_" + k, g, out.get("pick_" + k))
    valid_eval("64")
    # the fp32 top-50 kept as its differences from the fp64 one (54 positions; the fixture stays small)
    t32, t64 = out.pop("valid_top50").reshape(-1), out["valid_top5064"].reshape(-1)
    dpos = np.nonzero(t32 != t64)[0]
    out["valid_top50_fp32_diff_pos"] = dpos.astype(np.int32)
    out["valid_top50_fp32_diff_val"] = t32[dpos]
    np.savez_compressed(os.path.join(HERE, "vbpr_baby.npz"), **out)
    with open(os.path.join(HERE, "vbpr_baby_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, default=float)
    shutil.rmtree(TMP)
    print("wrote", os.path.join(HERE, "vbpr_baby.npz"), meta["loss"], res)


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "baby"
    if shape == "diffrec":
        return main_diffrec()
    if shape == "diffrec_train":
        return main_diffrec_train()
    if shape == "diffmm_train":
        return main_diffmm_train()
    if shape == "diffmm_train_sports":
        return main_diffmm_train("sports")
    if shape == "vbpr":
        return main_vbpr()
    if shape not in ("baby", "sports"):
        raise SystemExit("shape: baby, sports, diffrec, diffrec_train, diffmm_train, diffmm_train_sports or vbpr")
    ref = _import_reference()
    import torch
    import utils.utils as rutils
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if os.path.isdir(TMP):
        shutil.rmtree(TMP)
    write_dataset(TMP, shape)
    cfg = reference_config(ref, shape)
    ds = ref["dataset"].RecDataset(cfg)
    tr, va, te = ds.split()
    for part in (tr, va, te):
        str(part)
    # quick_start.py:46-102
    tdf = tr.df
    items = tdf[cfg["ITEM_ID_FIELD"]].value_counts().index.tolist()
    cfg["pop_items"] = set(items[:int(len(items) * 0.2)])
    uc = tdf[cfg["USER_ID_FIELD"]].value_counts()
    cfg["warm_users"] = set(uc[uc > 5].index.tolist())
    tl = ref["dataloader"].TrainDataLoader(cfg, tr, batch_size=cfg["train_batch_size"], shuffle=True)
    vl = ref["dataloader"].EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=cfg["eval_batch_size"])
    tel = ref["dataloader"].EvalDataLoader(cfg, te, additional_dataset=tr, batch_size=cfg["eval_batch_size"])
    rutils.init_seed(999)
    tl.pretrain_setup()
    model = ref["diffmm"].DiffMM(cfg, tl)
    U, I = model.n_users, model.n_items
    meta = {"U": U, "I": I, "n_train": len(tr), "torch": torch.__version__, "numpy": np.__version__,
            "generator": f"tests/golden/make_golden_baby.py {shape}", "reference": REF_SRC, "shape": shape}
    dg = {n: digest(getattr(model, n).detach().numpy()) for n in
          ("uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight")}
    for mod in ("image", "text"):
        den = getattr(model, "denoise_model_" + mod)
        for n, p in den.named_parameters():
            dg[f"den_{mod}_{n}"] = digest(p.detach().numpy())
    meta["param_sha256"] = dg
    out = {}
    # ---- graph rebuild (trainer.py:529-576): p_sample over every user, top-1 per modality
    uid, iid = cfg["USER_ID_FIELD"], cfg["ITEM_ID_FIELD"]
    inter = tdf.groupby(uid)[iid].apply(list).to_dict()
    B = cfg["train_batch_size"]
    tops = {}
    with torch.no_grad():
        for mod in ("image", "text"):
            den = getattr(model, "denoise_model_" + mod)
            idx5, val5 = [], []
            for lo in range(0, U, B):
                hi = min(U, lo + B)
                x = torch.zeros(hi - lo, I)
                for r, u in enumerate(range(lo, hi)):
                    it = inter.get(u, [])
                    if it:
                        x[r, it] = 1.0
                xs = model.diffusion_model.p_sample(den, x, model.sampling_steps, model.sampling_noise)
                v, ix = torch.topk(xs, k=5)
                idx5.append(ix.numpy())
                val5.append(v.numpy())
            idx5, val5 = np.concatenate(idx5), np.concatenate(val5)
            out[f"psample_{mod}_top5_idx"] = idx5.astype(np.int16)
            out[f"psample_{mod}_top5_val"] = val5.astype(np.float32)
            tops[mod] = idx5[:, 0]
        rb = object.__new__(ref["trainer"].DiffMMTrainer)
        rb.user_num, rb.item_num, rb.device = U, I, torch.device("cpu")
        ones = np.ones(U)
        model.image_UI_matrix = model.edgeDropper(rb.buildUIMatrix(np.arange(U), tops["image"], ones))
        model.text_UI_matrix = model.edgeDropper(rb.buildUIMatrix(np.arange(U), tops["text"], ones))
    # ---- full-rank evaluation (trainer.py:369-388) on valid (is_test False) and test (is_test True)
    ev = ref["topk_evaluator"].TopKEvaluator(cfg)
    kmax = max(cfg["topk"])
    splits = (("valid", vl, False), ("test", tel, True)) if shape == "baby" else (("valid", vl, False),)
    for name, ld, is_test in splits:
        mats, vals = [], []
        with torch.no_grad():
            for batch in ld:
                scores = model.full_sort_predict(batch)
                m = batch[1]
                scores[m[0], m[1]] = -1e10
                v, ix = torch.topk(scores, kmax, dim=-1)
                mats.append(ix)
                vals.append(v)
        topk = torch.cat(mats).numpy()
        out[f"{name}_top50"] = topk.astype(np.int16)
        out[f"{name}_top50_val_sample"] = torch.cat(vals)[:SAMPLE].numpy().astype(np.float32)
        res = ev.evaluate([torch.as_tensor(topk)], ld, is_test=is_test)
        pos = ld.get_eval_items()
        bool_rec = np.asarray([[i in p for i in row] for p, row in zip(pos, topk)])
        raw = ev._calculate_metrics(ld.get_eval_len_list(), bool_rec)
        meta[name] = {"n_users": int(len(topk)), "rounded": res,
                      "raw": {mname: np.asarray(raw[j], np.float64).tolist()
                              for j, mname in enumerate(["recall", "ndcg", "precision", "map"])},
                      "eval_users_head": np.asarray(ld.get_eval_users())[:16].tolist()}
    np.savez_compressed(os.path.join(HERE, f"diffmm_{shape}.npz"), **out)
    with open(os.path.join(HERE, f"diffmm_{shape}_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, default=float)
    shutil.rmtree(TMP)
    print("wrote", os.path.join(HERE, f"diffmm_{shape}.npz"))


if __name__ == "__main__":
    main()
