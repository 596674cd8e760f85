"""Pin the CPU oracle against golden vectors produced by the reference itself."""
import numpy as np
import pytest
import torch

from oracle import eval_ref, graph_ref, model_ref


def _params(g):
    return {k: torch.tensor(g["p_" + k], requires_grad=True)
            for k in ["uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight"]}


def _graphs(g):
    U, I = int(g["U"]), int(g["I"])
    N = U + I
    adj = graph_ref.norm_adj_csr(U, I, g["train_rows"], g["train_cols"])
    iadj = graph_ref.ui_adj_csr(U, I, np.arange(U), g["ui_img_items"])
    tadj = graph_ref.ui_adj_csr(U, I, np.arange(U), g["ui_txt_items"])
    return [model_ref.sparse_from_csr(*c, N) for c in (adj, iadj, tadj)], (adj, iadj, tadj)


def _feats(g):
    return {"v": torch.as_tensor(g["v_feat"]), "t": torch.as_tensor(g["t_feat"])}


def test_norm_adj_bit_exact(golden):
    g = golden("diffmm_tiny")
    U, I = int(g["U"]), int(g["I"])
    rp, col, val = graph_ref.norm_adj_csr(U, I, g["train_rows"], g["train_cols"])
    rp2, col2, val2 = graph_ref.coo_to_csr(U + I, g["norm_adj_idx"], g["norm_adj_val"])
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2)
    assert np.array_equal(val.view(np.uint32), val2.view(np.uint32))


@pytest.mark.parametrize("which", ["img", "txt", "k3"])
def test_ui_adj_bit_exact(golden, which):
    g = golden("diffmm_tiny")
    U, I = int(g["U"]), int(g["I"])
    if which == "k3":
        items = g["ui_k3_items"]
        users = np.repeat(np.arange(U), items.shape[1])
        items = items.reshape(-1)
    else:
        items = g[f"ui_{which}_items"]
        users = np.arange(U)
    rp, col, val = graph_ref.ui_adj_csr(U, I, users, items)
    key = "ui_k3" if which == "k3" else which + "_adj"
    rp2, col2, val2 = graph_ref.coo_to_csr(U + I, g[key + "_idx"], g[key + "_val"])
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2)
    assert np.array_equal(val.view(np.uint32), val2.view(np.uint32))


def test_forward_mm(golden):
    g = golden("diffmm_tiny")
    (adj, iadj, tadj), _ = _graphs(g)
    p = _params(g)
    with torch.no_grad():
        usr, itm = model_ref.forward_mm(p, _feats(g), adj, iadj, tadj)
        cl = model_ref.forward_cl_mm(p, _feats(g), adj, iadj, tadj)
    np.testing.assert_allclose(usr.numpy(), g["fwd_usr"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(itm.numpy(), g["fwd_itm"], rtol=1e-5, atol=1e-6)
    for n, t in zip(["cl_u1", "cl_i1", "cl_u2", "cl_i2"], cl):
        np.testing.assert_allclose(t.numpy(), g[n], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("cl_method", [0, 1])
def test_rec_loss_and_grads(golden, cl_method):
    g = golden("diffmm_tiny")
    (adj, iadj, tadj), _ = _graphs(g)
    p = _params(g)
    u, po, ne = (torch.as_tensor(g[k]) for k in ("bpr_users", "bpr_pos", "bpr_neg"))
    loss = model_ref.rec_loss(p, _feats(g), adj, iadj, tadj, u, po, ne, cl_method=cl_method)
    loss.backward()
    if cl_method == 0:
        np.testing.assert_allclose(loss.item(), g["rec_loss"], rtol=1e-5)
        for k in p:
            np.testing.assert_allclose(p[k].grad.numpy(), g["g_" + k], rtol=1e-4, atol=1e-7)
    else:
        np.testing.assert_allclose(loss.item(), g["rec_loss_cl1"], rtol=1e-5)
        np.testing.assert_allclose(p["uEmbeds"].grad.numpy(), g["g_cl1_uEmbeds"], rtol=1e-4, atol=1e-7)
        np.testing.assert_allclose(p["image_trans"].grad.numpy(), g["g_cl1_image_trans"], rtol=1e-4, atol=1e-7)


def _den(g):
    m = {"emb_W": "emb_layer_weight", "emb_b": "emb_layer_bias", "W1": "in_layers_0_weight",
         "b1": "in_layers_0_bias", "W2": "out_layers_0_weight", "b2": "out_layers_0_bias"}
    return {k: torch.tensor(g["den_" + v], requires_grad=True) for k, v in m.items()}


def test_schedule(golden):
    g = golden("diffmm_tiny")
    tab = model_ref.diffmm_schedule()
    for n in ["betas", "alphas_cumprod", "sqrt_alphas_cumprod", "sqrt_one_minus_alphas_cumprod",
              "posterior_mean_coef1", "posterior_mean_coef2", "posterior_variance"]:
        np.testing.assert_allclose(tab[n], g["sched_" + n], rtol=1e-12, atol=0)


def test_denoise_eval(golden):
    g = golden("diffmm_tiny")
    with torch.no_grad():
        out = model_ref.denoise(_den(g), torch.as_tensor(g["dif_x0"]), torch.as_tensor(g["den_t"]), 10)
    np.testing.assert_allclose(out.numpy(), g["den_out_eval"], rtol=1e-5, atol=1e-6)


def test_training_losses_and_grads(golden):
    g = golden("diffmm_tiny")
    w = _den(g)
    tab = model_ref.diffmm_schedule()
    diff, gc = model_ref.diffmm_training_losses(
        w, tab, torch.as_tensor(g["dif_x0"]), g["dif_t"], torch.as_tensor(g["dif_noise"]),
        torch.as_tensor(g["dif_keep"]), torch.as_tensor(g["dif_item_embeds"]), torch.as_tensor(g["dif_feats"]))
    np.testing.assert_allclose(diff.detach().numpy(), g["dif_diff_loss"], rtol=1e-5)
    np.testing.assert_allclose(gc.detach().numpy(), g["dif_gc_loss"], rtol=1e-5)
    (diff.mean() + gc.mean() * 0.5).backward()
    names = {"emb_W": "emb_layer_weight", "emb_b": "emb_layer_bias", "W1": "in_layers_0_weight",
             "b1": "in_layers_0_bias", "W2": "out_layers_0_weight", "b2": "out_layers_0_bias"}
    for k, v in names.items():
        np.testing.assert_allclose(w[k].grad.numpy(), g["dif_grad_" + v], rtol=1e-4, atol=1e-6)


def test_p_sample_top1(golden):
    g = golden("diffmm_tiny")
    with torch.no_grad():
        x = model_ref.diffmm_p_sample(_den(g), model_ref.diffmm_schedule(), torch.as_tensor(g["dif_x0"]))
    np.testing.assert_allclose(x.numpy(), g["psample_out"], rtol=1e-5, atol=1e-6)
    assert np.array_equal(eval_ref.topk_rows(x.numpy(), 1), g["psample_top1"])


def test_eval_topk_and_metrics(golden, golden_meta):
    g = golden("diffmm_tiny")
    s = eval_ref.mask_scores(g["eval_scores_raw"], g["eval_mask_rows"], g["eval_mask_cols"])
    assert np.array_equal(s, g["eval_scores_masked"])
    top = eval_ref.topk_rows(s, 50)
    ref_top = g["eval_topk"]
    # identical selection up to tie groups (torch.topk tie order is implementation-defined)
    for r in range(s.shape[0]):
        assert np.array_equal(np.sort(s[r, top[r]]), np.sort(s[r, ref_top[r]]))
        for v in np.unique(s[r, top[r]]):
            a = set(top[r][s[r, top[r]] == v])
            b = set(ref_top[r][s[r, ref_top[r]] == v])
            if v != s[r, top[r]].min():
                assert a == b
    pos_len = g["eval_pos_len"]
    pos = np.split(g["eval_pos_flat"], np.cumsum(pos_len)[:-1])
    curves = eval_ref.metric_curves(eval_ref.hit_matrix(ref_top, pos), pos_len)
    want = golden_meta["diffmm_metrics"]
    for m, arr in want["raw"].items():
        np.testing.assert_allclose(curves[m], arr, rtol=1e-12, atol=1e-15)
    got = eval_ref.metric_dict(curves)
    assert got == want["rounded"]


def test_metric_edge_cases(golden_meta):
    e = golden_meta["metrics_edge"]
    topk = np.asarray(e["topk"])
    pos = [np.asarray(p) for p in e["pos"]]
    curves = eval_ref.metric_curves(eval_ref.hit_matrix(topk, pos), [len(p) for p in pos])
    for m, arr in e["metrics"]["raw"].items():
        np.testing.assert_allclose(curves[m], arr, rtol=1e-12, atol=1e-15)
    assert eval_ref.metric_dict(curves) == e["metrics"]["rounded"]


def test_diffrec_psample(golden):
    g = golden("diffrec_tiny")
    tab = model_ref.diffrec_schedule(steps=int(g["T"]))
    for n in ["betas", "alphas_cumprod", "posterior_mean_coef1", "posterior_mean_coef2"]:
        np.testing.assert_allclose(tab[n], g["sched_" + n], rtol=1e-12)
    w = {"emb_W": g["dnn_emb_layer_weight"], "emb_b": g["dnn_emb_layer_bias"], "W1": g["dnn_in_layers_0_weight"],
         "b1": g["dnn_in_layers_0_bias"], "W2": g["dnn_out_layers_0_weight"], "b2": g["dnn_out_layers_0_bias"]}
    w = {k: torch.as_tensor(v) for k, v in w.items()}
    with torch.no_grad():
        out = model_ref.denoise(w, torch.as_tensor(g["x0"]), torch.as_tensor(g["fwd_t"]), int(g["E"]))
        ps = model_ref.diffrec_p_sample(w, tab, torch.as_tensor(g["x0"]), int(g["E"]), int(g["T"]))
    np.testing.assert_allclose(out.numpy(), g["fwd_out"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ps.numpy(), g["psample"], rtol=1e-4, atol=1e-6)


def _diffrec_w(g, grad=False):
    w = {"emb_W": g["dnn_emb_layer_weight"], "emb_b": g["dnn_emb_layer_bias"], "W1": g["dnn_in_layers_0_weight"],
         "b1": g["dnn_in_layers_0_bias"], "W2": g["dnn_out_layers_0_weight"], "b2": g["dnn_out_layers_0_bias"]}
    return {k: torch.tensor(v, requires_grad=grad) for k, v in w.items()}


def test_diffrec_training_losses_and_history(golden):
    """training_losses(reweight=True) rows, gradients and the Lt history/count after each step."""
    g = golden("diffrec_tiny")
    T = int(g["T"])
    tab = model_ref.diffrec_schedule(steps=T)
    x0 = torch.as_tensor(g["x0"])
    hist = np.zeros((T, 10))
    count = np.zeros(T, np.int64)
    for s in range(int(g["train_steps"])):
        w = _diffrec_w(g, grad=(s == 0))
        t = g[f"train{s}_t"]
        wl, loss = model_ref.diffrec_training_losses(w, tab, x0, t, torch.as_tensor(g[f"train{s}_noise"]),
                                                     torch.as_tensor(g[f"train{s}_keep"]), np.ones(len(t), np.float32),
                                                     int(g["E"]))
        np.testing.assert_allclose(loss.detach().numpy(), g[f"train{s}_loss"], rtol=1e-5, atol=1e-9)
        if s == 0:
            loss.mean().backward()
            for k, n in [("emb_W", "emb_layer_weight"), ("emb_b", "emb_layer_bias"), ("W1", "in_layers_0_weight"),
                         ("b1", "in_layers_0_bias"), ("W2", "out_layers_0_weight"), ("b2", "out_layers_0_bias")]:
                want = g[f"train0_g_{n}"]  # fp32 reassociation: atol relative to the tensor's scale
                np.testing.assert_allclose(w[k].grad.numpy(), want, rtol=1e-4, atol=1e-5 * np.abs(want).max())
        # the history holds the reference's own fp32 losses: feed those (bit-exact bookkeeping)
        hist, count = model_ref.lt_history_update(hist, count, t, g[f"train{s}_loss"])
        np.testing.assert_array_equal(count, g[f"train{s}_count"])
        np.testing.assert_array_equal(hist, g[f"train{s}_hist"])
    pt_all = model_ref.importance_pt_all(g["imp_hist"])
    np.testing.assert_allclose(pt_all[g["imp_t"]] * T, g["imp_pt"], rtol=1e-12)


def test_vbpr(golden):
    g = golden("vbpr_tiny")
    p = {k[2:]: torch.tensor(g[k], requires_grad=True) for k in g if k.startswith("p_")}
    v, t = torch.as_tensor(g["v_feat"]), torch.as_tensor(g["t_feat"])
    loss = model_ref.vbpr_loss(p, v, t, torch.as_tensor(g["users"]), torch.as_tensor(g["pos"]),
                               torch.as_tensor(g["neg"]), 2.0)
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-5)
    for k in p:
        np.testing.assert_allclose(p[k].grad.numpy(), g["g_" + k], rtol=1e-4, atol=1e-7)
    with torch.no_grad():
        ue, ie = model_ref.vbpr_forward(p, v, t)
    np.testing.assert_allclose((ue @ ie.T).detach().numpy(), g["scores"], rtol=1e-5, atol=1e-6)


def test_adam_matches_torch():
    rng = np.random.default_rng(0)
    ps = [rng.standard_normal((7, 5)).astype(np.float32)]
    gs = [[rng.standard_normal((7, 5)).astype(np.float32)] for _ in range(3)]
    out = model_ref.adam_reference(ps, gs)
    assert out[0].shape == (7, 5)


_DEN = {"emb_W": "emb_layer_weight", "emb_b": "emb_layer_bias", "W1": "in_layers_0_weight",
        "b1": "in_layers_0_bias", "W2": "out_layers_0_weight", "b2": "out_layers_0_bias"}


def test_diffusion_phase_oracle(golden):
    """D16: the oracle's training_losses + torch Adam over the reference's recorded diffusion phase
    (common/trainer.py:491-527, diffmm_phases_tiny.npz) reproduce its losses and final weights."""
    g, ph = golden("diffmm_tiny"), golden("diffmm_phases_tiny")
    U, I = int(g["U"]), int(g["I"])
    tab = model_ref.diffmm_schedule()
    p = _params(g)
    feats = {"image": model_ref.modal_feats(_feats(g)["v"], p["image_trans"]).detach(),
             "text": model_ref.modal_feats(_feats(g)["t"], p["text_trans"]).detach()}
    iE = p["iEmbeds"].detach()
    ws = {m: {k: torch.tensor(ph[f"init_{m}_{v}"], requires_grad=True) for k, v in _DEN.items()}
          for m in ("image", "text")}
    opts = {m: torch.optim.Adam(list(ws[m].values()), lr=1e-3, foreach=False) for m in ws}
    rows, cols = g["train_rows"], g["train_cols"]
    perm = ph["dif_perm"]
    for b in range(int(ph["dif_batches"])):
        users = perm[b * 40:(b + 1) * 40]
        x0 = np.zeros((len(users), I), np.float32)
        for r, u in enumerate(users):
            x0[r, cols[rows == u]] = 1.0
        total = 0.0
        for m in ("image", "text"):
            opts[m].zero_grad()
            diff, gc = model_ref.diffmm_training_losses(
                ws[m], tab, torch.as_tensor(x0), ph[f"dif{b}_{m}_t"], torch.as_tensor(ph[f"dif{b}_{m}_noise"]),
                torch.as_tensor(ph[f"dif{b}_{m}_keep"]), iE, feats[m])
            loss = diff.mean() + 0.5 * gc.mean()
            np.testing.assert_allclose(loss.item(), ph["dif_losses"][b, 0 if m == "image" else 1], rtol=1e-5)
            total = total + loss
        total.backward()
        for m in ("image", "text"):
            opts[m].step()
    for m in ("image", "text"):
        for k, v in _DEN.items():
            np.testing.assert_allclose(ws[m][k].detach().numpy(), ph[f"final_{m}_{v}"], rtol=1e-4, atol=1e-7)


def test_bpr_phase_oracle(golden):
    """D18: the oracle's rec_loss + torch Adam over the reference's three recorded BPR steps
    (common/trainer.py:144-208) reproduce its losses and final rec parameters."""
    g, ph = golden("diffmm_tiny"), golden("diffmm_phases_tiny")
    (adj, iadj, tadj), _ = _graphs(g)
    p = _params(g)
    names = ["uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight"]
    opt = torch.optim.Adam([p[n] for n in names], lr=1e-3, foreach=False)
    for st in range(3):
        inter = torch.as_tensor(ph[f"bpr{st}_inter"])
        opt.zero_grad()
        loss = model_ref.rec_loss(p, _feats(g), adj, iadj, tadj, inter[0], inter[1], inter[2])
        loss.backward()
        opt.step()
        np.testing.assert_allclose(loss.item(), ph["bpr_losses"][st], rtol=1e-5)
    for n in names:
        np.testing.assert_allclose(p[n].detach().numpy(), ph["bpr_final_" + n], rtol=1e-4, atol=1e-7)
