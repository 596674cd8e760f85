"""GenRecV1 HIP path vs the reference's golden vectors (genrecv1_tiny.npz) and the CPU oracle.

Tolerances: index / graph structure / masks bit-exact; forward activations rtol 1e-5; losses 1e-5
relative; gradients rtol 2e-4 (fp32 reassociation over batch and graph sums); transformer
outputs 1e-4.  Rebuild top-k: bit-exact on the picks with a non-zero score, zero-valued ties only
checked to be zero-valued (the reference's CPU top-k breaks those ties in an unspecified order).
"""
import types

import numpy as np
import pytest
import torch

from oracle import genrec_ref, graph_ref
from genrec_fixture import BN_NAMES, masks_of, model_graphs, sub

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def G(golden):
    g = golden("genrecv1_tiny")
    return {"m": sub(g, "m_"), "d": sub(g, "d_"), "r": sub(g, "r_")}


def _config(**over):
    from gmr.configurator import Config
    cfg = {"train_batch_size": 24, "eval_batch_size": 32, "epochs": 1, "seed": [999], "save_recommended_topk": False}
    cfg.update(over)
    return Config("GenRecV1", "baby", cfg)


def _dev(a, dt=None):
    t = torch.as_tensor(np.ascontiguousarray(a))
    return (t.to(dt) if dt is not None else t).to(DEV)


def build_model(m):
    from gmr.dataloader import TrainDataLoader
    from gmr.dataset import RecDataset
    from gmr.genrecv1 import GenRecV1
    from gmr import kernels as K
    cfg = _config()
    U, I = int(m["U"]), int(m["I"])
    ds = RecDataset.from_arrays(cfg, m["train_rows"], m["train_cols"], np.zeros(len(m["train_rows"])), U, I,
                                m["v_feat"], m["t_feat"])
    tl = TrainDataLoader(cfg, ds, batch_size=24)
    torch.manual_seed(999)
    model = GenRecV1(cfg, tl)
    s = model.rec_slab
    s.view("E0")[:U].copy_(torch.as_tensor(m["p_user_embedding_weight"]))
    s.view("E0")[U:].copy_(torch.as_tensor(m["p_item_id_embedding_weight"]))
    for n in model._pnames:
        s.load(n, torch.as_tensor(m["p_" + n]))
    # graphs: kNN II on the device, the rebuilt UI graph from the fixture's edges + keep flags
    model.build_item_item_graphs(10)
    uptr = torch.arange(0, 10 * U + 1, 10, dtype=torch.int32, device=DEV)
    items = np.sort(m["ui_k10_items"], axis=1).reshape(-1)
    ui = K.bipartite_symnorm(U, I, uptr, _dev(items, torch.int32), True, 0.0)
    model.set_image_ui_matrix(K.csr_drop_edges(ui, 0.5, keep=_dev(m["ui_keep_sorted"], torch.uint8)))
    return model, ui


@pytest.fixture(scope="module")
def M(G):
    return build_model(G["m"])


def _csr_np(c):
    return c.rowptr.cpu().numpy(), c.col.cpu().numpy(), c.val.cpu().numpy()


def test_graphs(G, M):
    m = G["m"]
    model, ui = M
    csrs, _ = model_graphs(m)
    for name, mine in (("norm_adj", model.norm_adj), ("R", model.R), ("ui_full", ui), ("ui_img", model.image_UI_matrix)):
        rp, col, val = _csr_np(mine)
        assert np.array_equal(rp, csrs[name][0]) and np.array_equal(col, csrs[name][1]), name
        assert np.array_equal(val.view(np.uint32), csrs[name][2].view(np.uint32)), name
    for name, mine in (("ii_img", model.image_II_matrix), ("ii_txt", model.text_II_matrix)):
        rp, col, val = _csr_np(mine)
        assert np.array_equal(rp, csrs[name][0]) and np.array_equal(col, csrs[name][1]), name
        np.testing.assert_allclose(val, csrs[name][2], rtol=1e-5, atol=1e-7)


def test_csr_transpose(M):
    import scipy.sparse as sp
    model, _ = M
    for a, at in ((model.R, model.RT), (model.image_UI_matrix, model.image_UI_matrix_T),
                  (model.image_II_matrix, model._ii_T[0])):
        rp, col, val = _csr_np(a)
        S = sp.csr_matrix((val, col, rp), shape=(a.n_rows, a.n_cols)).T.tocsr()
        S.sort_indices()
        trp, tcol, tval = _csr_np(at)
        assert np.array_equal(trp, S.indptr) and np.array_equal(tcol, S.indices)
        assert np.array_equal(tval.view(np.uint32), S.data.astype(np.float32).view(np.uint32))


def test_csr_transpose_long_rows():
    """Transposed rows above 256 entries take the LDS-bitmap ordering path."""
    import scipy.sparse as sp
    from gmr import kernels as K
    rng = np.random.default_rng(4)
    n_r, n_c = 3000, 40
    S = sp.random(n_r, n_c, density=0.3, random_state=np.random.RandomState(4), format="csr", dtype=np.float32)
    S.sort_indices()
    a = K.CSR(_dev(S.indptr.astype(np.int32)), _dev(S.indices.astype(np.int32)), _dev(S.data), n_cols=n_c,
              symmetric=False)
    at = K.csr_transpose(a)
    T = S.T.tocsr()
    T.sort_indices()
    trp, tcol, tval = _csr_np(at)
    assert np.array_equal(trp, T.indptr) and np.array_equal(tcol, T.indices)
    assert np.array_equal(tval, T.data)


def test_drop_edges_statistics(M):
    from gmr import kernels as K
    _, ui = M
    d = K.csr_drop_edges(ui, 0.5, seed=3, step=1)
    frac = d.nnz / ui.nnz
    assert 0.4 < frac < 0.6
    assert np.allclose(np.unique(d.val.cpu().numpy() / 2.0)[:3] > 0, True)
    d2 = K.csr_drop_edges(ui, 0.5, seed=3, step=1)
    assert np.array_equal(d.col.cpu().numpy(), d2.col.cpu().numpy())  # deterministic per (seed, step)


def test_drop_edges_transposed(M):
    """transposed=True on the symmetric rebuilt graph equals the transpose of the dropped graph."""
    from gmr import kernels as K
    _, ui = M
    d = K.csr_drop_edges(ui, 0.5, seed=4, step=2)
    dt = K.csr_drop_edges(ui, 0.5, seed=4, step=2, transposed=True)
    ref = K.csr_transpose(d)
    for x, y in zip(_csr_np(dt), _csr_np(ref)):
        assert np.array_equal(x, y)


def _inject_masks(m, prefix):
    return {k: v for k, v in masks_of(m, prefix).items()}


def test_forward_train_and_bn_stats(G, M):
    m = G["m"]
    model, _ = M
    for n in BN_NAMES:
        model.bn_state[n][0].zero_()
        model.bn_state[n][1].fill_(1.0)
    w = model._work(24)
    C, S = model._forward(w, True, _inject_masks(m, "fwd"))
    np.testing.assert_allclose(C.cpu().numpy(), m["fwd_content"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(S.cpu().numpy(), m["fwd_side"], rtol=1e-4, atol=1e-6)
    for n in BN_NAMES[:-1]:
        np.testing.assert_allclose(model.bn_state[n][0].cpu().numpy(), m[f"fwd_bn_{n}_mean"], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(model.bn_state[n][1].cpu().numpy(), m[f"fwd_bn_{n}_var"], rtol=1e-5, atol=1e-7)


def test_rec_step_unfused_nce_matches_golden(G, M, monkeypatch):
    """GMR_NCE_FUSED=0 (the in-batch InfoNCE terms through the B x B logit GEMMs instead of the fused contrast
    kernel): the same loss and gradients as the reference (the default fused form is checked below)."""
    from gmr import genrecv1 as gv
    monkeypatch.setattr(gv, "NCE_FUSED", False)
    m = G["m"]
    model, _ = M
    for n in BN_NAMES:
        model.bn_state[n][0].zero_()
        model.bn_state[n][1].fill_(1.0)
    model._forward(model._work(24), True, _inject_masks(m, "fwd"))
    t = lambda k: _dev(m[k].astype(np.int32))  # noqa: E731
    loss = model.rec_step(t("bpr_users"), t("bpr_pos"), t("bpr_neg"), masks=_inject_masks(m, "loss"))
    np.testing.assert_allclose(loss.item(), float(m["loss"]), rtol=1e-5)
    for n in [str(s) for s in m["g_names"]]:
        k = n.replace(".", "_")
        np.testing.assert_allclose(model.grad_view(k).cpu().numpy().reshape(m["g_" + k].shape), m["g_" + k],
                                   rtol=2e-4, atol=2e-7, err_msg=n)


def test_rec_step_loss_grads_and_eval(G, M):
    m = G["m"]
    model, _ = M
    # BN running stats as the reference's after its forward call, then calculate_loss
    for n in BN_NAMES:
        model.bn_state[n][0].zero_()
        model.bn_state[n][1].fill_(1.0)
    model._forward(model._work(24), True, _inject_masks(m, "fwd"))
    t = lambda k: _dev(m[k].astype(np.int32))  # noqa: E731
    loss = model.rec_step(t("bpr_users"), t("bpr_pos"), t("bpr_neg"), masks=_inject_masks(m, "loss"))
    np.testing.assert_allclose(loss.item(), float(m["loss"]), rtol=1e-5)
    for n in [str(s) for s in m["g_names"]]:
        k = n.replace(".", "_")
        np.testing.assert_allclose(model.grad_view(k).cpu().numpy().reshape(m["g_" + k].shape), m["g_" + k],
                                   rtol=2e-4, atol=2e-7, err_msg=n)
    for n in BN_NAMES[:-1]:
        np.testing.assert_allclose(model.bn_state[n][0].cpu().numpy(), m[f"loss_bn_{n}_mean"], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(model.bn_state[n][1].cpu().numpy(), m[f"loss_bn_{n}_var"], rtol=1e-5, atol=1e-7)
    # eval mode: full_sort_predict and the full forward with running statistics
    model.eval()
    sc = model.full_sort_predict([_dev(m["eval_users"])])
    np.testing.assert_allclose(sc.cpu().numpy(), m["eval_scores"], rtol=1e-5, atol=1e-6)
    # opt-in fp16 MFMA scoring (config 5): inputs rounded to fp16, fp32 accumulation.  Tolerance
    # from the rounding: |err| <= 2^-10 * sum_k |u_k i_k| per score (parity unpinned: the
    # reference has no fp16 path)
    model.scoring_dtype = "fp16"
    try:
        s16 = model.full_sort_predict([_dev(m["eval_users"])]).cpu().numpy()
    finally:
        model.scoring_dtype = "fp32"
    want = m["eval_scores"]
    np.testing.assert_allclose(s16, want, rtol=0, atol=2e-3 * float(np.abs(want).max()) + 1e-6)
    top16, top32 = np.argsort(-s16, 1)[:, :10], np.argsort(-want, 1)[:, :10]
    overlap = np.mean([len(set(a) & set(b)) / 10 for a, b in zip(top16, top32)])
    assert overlap >= 0.8, overlap
    C, S = model.forward(train=False)
    np.testing.assert_allclose(S.cpu().numpy(), m["eval_side"], rtol=1e-4, atol=1e-6)
    model.train()


def _denoiser(d, dropout=0.0):
    from gmr.transformer import TransformerDenoiser
    I = int(d["I"])
    den = TransformerDenoiser(I, I, 10, DEV, nhead=8, num_layers=int(d["n_layers"]), dim_feedforward=int(d["d_model"]),
                              dropout=dropout)
    den.load_state({k[4:]: v for k, v in d.items() if k.startswith("den_") and k != "den_names"})
    return den


def _pad(x):
    x = np.asarray(x, np.float32)
    B, I = x.shape
    buf = torch.zeros((B, (I + 3) // 4 * 4), dtype=torch.float32, device=DEV)
    buf[:, :I].copy_(torch.as_tensor(x))
    return buf[:, :I]


def test_denoiser_forward_eval(G):
    d = G["d"]
    den = _denoiser(d)
    den.eval()
    out = den.forward(_pad(d["fwd_x"]), t_rows=_dev(d["fwd_t"], torch.int32))
    np.testing.assert_allclose(out.cpu().numpy(), d["fwd_out"], rtol=1e-4, atol=1e-5)


def _flip_model(x0, I, gen_topk=5, rebuild_k=10, sampling_steps=5):
    B = x0.shape[0]
    rows, cols = np.nonzero(x0)
    uptr = np.zeros(B + 1, np.int32)
    np.add.at(uptr, rows + 1, 1)
    uptr = np.cumsum(uptr).astype(np.int32)
    ns = types.SimpleNamespace(steps=5, flip_temp=1.0, sparse_temp=0.5, n_items=I, device=DEV,
                               user_ptr=_dev(uptr), user_items=_dev(cols.astype(np.int32)), gen_topk=gen_topk,
                               rebuild_k=rebuild_k, sampling_steps=sampling_steps)
    return ns


def test_flip_schedule_bit_exact(G):
    from gmr.genrecv1 import FlipDiffusion
    d = G["d"]
    x0 = d["x0"]
    fd = FlipDiffusion(_flip_model(x0, int(d["I"])))
    tab = fd.schedule(torch.arange(x0.shape[0], dtype=torch.int32, device=DEV)).cpu().numpy()
    T = 5
    assert np.array_equal(tab[:T].view(np.uint32), d["gamma_cum"].view(np.uint32))
    assert np.array_equal(tab[T:2 * T].view(np.uint32), d["eps_cum"].view(np.uint32))
    x = torch.as_tensor(x0)
    pw = (torch.sum(1 - x) / (torch.sum(x) + 1e-8)).item()
    assert tab[2 * T] == np.float32(pw)


def test_training_step_vs_reference(G):
    """FlipInterestDiffusion.training_losses + backward with the reference's draws injected
    (denoiser dropout p = 0 as in the fixture)."""
    from gmr.genrecv1 import FlipDiffusion
    d = G["d"]
    I, B = int(d["I"]), int(d["B"])
    den = _denoiser(d, dropout=0.0)
    den.train()
    fd = FlipDiffusion(_flip_model(d["x0"], I))
    users = torch.arange(B, dtype=torch.int32, device=DEV)
    u8 = lambda a: _dev(np.asarray(a).astype(np.uint8))  # noqa: E731
    inj = {"t": _dev(d["tl_t"], torch.int32), "flip1": u8(d["tl_flip1"]), "ps_flip": u8(d["tl_flip2"]),
           "ps_draws": [u8(d[f"tl_ps{s}"]) for s in range(5)]}
    iE = _dev(d["item_embeds"])
    feats = _dev(d["img_feats"])
    lv = fd.training_step(den, users, iE, feats, seed=1, step=0, inject=inj).cpu().numpy()
    np.testing.assert_allclose(lv[0], float(d["loss_bce"]), rtol=1e-5)
    np.testing.assert_allclose(lv[1], float(d["loss_kl"]), rtol=1e-5)
    np.testing.assert_allclose(lv[2], float(d["loss_cl"]), rtol=1e-5)
    np.testing.assert_allclose(lv[3], float(d["loss_total"]), rtol=1e-5)
    for n in [str(s) for s in d["g_names"]]:
        k = n.replace(".", "_")
        got = den.g(k).cpu().numpy().reshape(d["g_" + k].shape)
        np.testing.assert_allclose(got, d["g_" + k], rtol=2e-3, atol=2e-6, err_msg=n)


def test_training_step_logits(G):
    from gmr.genrecv1 import FlipDiffusion
    d = G["d"]
    I, B = int(d["I"]), int(d["B"])
    den = _denoiser(d, dropout=0.0)
    den.train()
    x = _pad(d["tl_call0_x"])
    out = den.forward(x, t_rows=_dev(d["tl_call0_t"], torch.int32))
    np.testing.assert_allclose(out.cpu().numpy(), d["tl_call0_logits"], rtol=1e-4, atol=1e-5)


def test_rebuild_rows_vs_reference(G):
    from gmr.genrecv1 import FlipDiffusion
    r = G["r"]
    d = G["d"]
    x0 = r["x0"]
    B, I = x0.shape
    den = _denoiser({**{k: v for k, v in r.items() if k.startswith("den_")}, "I": I, "n_layers": 2, "d_model": 64},
                    dropout=0.0)
    den.train()
    fd = FlipDiffusion(_flip_model(x0, I))
    u8 = lambda a: _dev(np.asarray(a).astype(np.uint8))  # noqa: E731
    inj = {"flip": u8(r["ps_flip"]), "draws": [u8(r[f"ps_step{s}"]) for s in range(5)],
           "dislike": r["ps_dislike_sample"], "like": r["ps_like_sample"]}
    out = torch.zeros((B, 10), dtype=torch.int32, device=DEV)
    labels = _dev(r["km_labels"].astype(np.int32))
    dn, probs = fd.rebuild_rows(den, torch.arange(B, dtype=torch.int32, device=DEV), out, labels, 0.1, 1, 0,
                                inject=inj)
    np.testing.assert_allclose(probs.cpu().numpy(), r["ps_probs"], rtol=1e-5, atol=1e-6)
    assert np.array_equal(dn.cpu().numpy(), r["debiased"])
    score = r["debiased"] * r["ps_probs"]
    mine = out.cpu().numpy()
    ref_i, ref_v = r["rebuild_top_idx"], r["rebuild_top_vals"]
    for b in range(B):
        nz = ref_v[b] > 0
        assert np.array_equal(mine[b][nz], ref_i[b][nz])
        assert np.all(score[b][mine[b][~nz]] == 0)


def test_debias_select_exact_counts(G):
    """Device picks: exactly int(count * ratio) of each flip type, distinct, of the right type."""
    from gmr.genrecv1 import FlipDiffusion
    r = G["r"]
    x0 = r["x0"]
    B, I = x0.shape
    fd = FlipDiffusion(_flip_model(x0, I))
    fd._work(B)
    x0d = _pad(x0)
    xs = _pad(r["ps_out"])
    tk = torch.empty((B, 5), dtype=torch.int32, device=DEV)
    from gmr import kernels as K
    K.topk_rows(_pad(r["ps_probs"]), 5, tk)
    dn = _pad(np.zeros_like(x0))
    fd._debias(B, tk, x0d, xs, dn, _dev(r["km_labels"].astype(np.int32)), 0.1, 7, 3, {})
    npk = fd._npicks.cpu().numpy()
    assert npk[0] == int(int(r["ps_n_dislike"]) * 0.1) and npk[1] == int(int(r["ps_n_like"]) * 0.1)
    for t in range(2):
        pk = fd._picks[t, :npk[t]].cpu().numpy()
        assert len({tuple(p) for p in pk}) == len(pk)
        for b, i in pk:
            assert (x0[b, i], r["ps_out"][b, i]) == ((0.0, 1.0) if t == 0 else (1.0, 0.0))


def test_kmeans_recovers_planted_clusters(G):
    from gmr.kmeans import kmeans_labels
    r = G["r"]
    lab = kmeans_labels(_dev(r["km_feat"]), 4, seed=11).cpu().numpy()
    true = r["km_true"]
    pairs = set(zip(lab.tolist(), true.tolist()))
    assert len(pairs) == 4 and len(set(lab.tolist())) == 4


def test_denoiser_dropout_grads_vs_torch(G):
    """Train-mode dropout path: the HIP forward/backward against a torch fp32 twin fed the same
    masks (attention-weight head masks, residual-branch masks, feed-forward mask)."""
    d = G["d"]
    I, L, D = int(d["I"]), int(d["n_layers"]), int(d["d_model"])
    den = _denoiser(d, dropout=0.2)
    den.train()
    rng = np.random.default_rng(5)
    B = 16
    x = (rng.random((B, I)) < 0.3).astype(np.float32)
    t = rng.integers(0, 5, B).astype(np.int32)
    out = den.forward(_pad(x), t_rows=_dev(t), seed=9, step=2)
    dout = rng.standard_normal((B, I)).astype(np.float32)
    do = _pad(dout)
    den.backward(do)
    w = den._ws
    masks = {s: w["mask_" + s][:, :B].cpu().numpy().astype(np.float32) for s in ("a", "c", "1", "2", "3", "f")}
    # torch twin
    P = {k[4:]: torch.tensor(v, requires_grad=True) for k, v in d.items() if k.startswith("den_") and k != "den_names"}
    te = genrec_ref.time_embedding(t) @ P["emb_layer_weight"].t() + P["emb_layer_bias"]
    h = torch.cat([torch.tensor(x), te], -1) @ P["input_proj_weight"].t() + P["input_proj_bias"]
    ada = torch.nn.functional.silu(te) @ P["adaLN_modulation_1_weight"].t() + P["adaLN_modulation_1_bias"]
    h = h * (1 + ada[:, D:]) + ada[:, :D]
    k = 1 / 0.8
    hm = lambda mk: torch.tensor(np.repeat(mk, D // 8, axis=1))  # noqa: E731
    F = torch.nn.functional
    for l in range(L):
        p = f"transformer_decoder_layers_{l}_"
        v = h @ P[p + "self_attn_in_proj_weight"][2 * D:].t() + P[p + "self_attn_in_proj_bias"][2 * D:]
        sa = (v * hm(masks["a"][l]) * k) @ P[p + "self_attn_out_proj_weight"].t() + P[p + "self_attn_out_proj_bias"]
        h = F.layer_norm(h + sa * torch.tensor(masks["1"][l]) * k, (D,), P[p + "norm1_weight"], P[p + "norm1_bias"])
        bc = P[p + "multihead_attn_in_proj_bias"][2 * D:].expand(B, D) * hm(masks["c"][l]) * k
        ca = bc @ P[p + "multihead_attn_out_proj_weight"].t() + P[p + "multihead_attn_out_proj_bias"]
        h = F.layer_norm(h + ca * torch.tensor(masks["2"][l]) * k, (D,), P[p + "norm2_weight"], P[p + "norm2_bias"])
        ff = F.relu(h @ P[p + "linear1_weight"].t() + P[p + "linear1_bias"]) * torch.tensor(masks["f"][l]) * k
        ff = ff @ P[p + "linear2_weight"].t() + P[p + "linear2_bias"]
        h = F.layer_norm(h + ff * torch.tensor(masks["3"][l]) * k, (D,), P[p + "norm3_weight"], P[p + "norm3_bias"])
    o = h @ P["output_proj_0_weight"].t() + P["output_proj_0_bias"]
    o = F.gelu(F.layer_norm(o, (o.shape[1],), P["output_proj_1_weight"], P["output_proj_1_bias"]))
    o = o @ P["output_proj_3_weight"].t() + P["output_proj_3_bias"]
    np.testing.assert_allclose(out.cpu().numpy(), o.detach().numpy(), rtol=1e-4, atol=1e-5)
    (o * torch.tensor(dout)).sum().backward()
    for n, p_ in P.items():
        want = p_.grad.numpy() if p_.grad is not None else np.zeros_like(p_.detach().numpy())
        got = den.g(n).cpu().numpy().reshape(want.shape)
        np.testing.assert_allclose(got, want, rtol=2e-3, atol=2e-5, err_msg=n)
    # keep rates of the drawn masks ~ 0.8
    assert 0.7 < masks["1"].mean() < 0.9 and 0.7 < masks["f"].mean() < 0.9


def test_trainer_epoch_and_eval():
    """End-to-end: GenRecV1Trainer epoch (diffusion + rebuild + BPR) and a full-rank evaluation on a
    tiny synthetic dataset; losses finite, metrics in range, graphs rebuilt."""
    from gmr.configurator import Config
    from gmr.dataloader import EvalDataLoader, TrainDataLoader
    from gmr.genrecv1 import GenRecV1
    from gmr.synthetic import make_dataset
    from gmr.trainer import GenRecV1Trainer
    from gmr.utils import init_seed
    cfg = Config("GenRecV1", "tiktok", {"synthetic": "tiny", "train_batch_size": 256, "eval_batch_size": 256,
                                         "epochs": 1, "save_recommended_topk": False, "num_layers": 2})
    init_seed(999)
    ds = make_dataset(cfg, "tiny", seed=0)
    tr, va, te = ds.split()
    tl = TrainDataLoader(cfg, tr, batch_size=256, shuffle=True)
    vl = EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=256)
    model = GenRecV1(cfg, tl)
    trainer = GenRecV1Trainer(cfg, model)
    loss, _ = trainer._train_epoch(tl, 0)
    assert np.isfinite(loss)
    assert model.image_UI_matrix is not None and model.image_UI_matrix.nnz > 0
    dl = trainer._dloss.cpu().numpy()
    assert np.all(np.isfinite(dl))
    res = trainer.evaluate(vl)
    assert 0.0 <= res["recall@20"] <= 1.0


@pytest.mark.parametrize("n", [6710, 100, 1024, 4097])
def test_kmeans_pp_pick_weighted_draw(n):
    """gmr_kmeans_pp_pick (k-means++ candidate draw with probability mind[r] / sum, csrc/gengraph.hip): a single
    non-zero weight is always picked (first, last and inner points; n below, at and above the 1,024 partials);
    two weights are picked in their ratio (binomial 5-sigma bound over 600 draws); mind = NULL picks uniformly."""
    from gmr import _lib
    from gmr.kernels import ptr, stream
    draws = 600
    out = torch.empty(draws, dtype=torch.int32, device=DEV)

    def pick(mind, k=draws):
        for i in range(k):
            _lib.call("gmr_kmeans_pp_pick", n, ptr(mind) if mind is not None else None, 7, 100 + i, ptr(out[i:i + 1]),
                      stream())
        return out[:k].cpu().numpy()

    for p in (0, n - 1, n // 3):
        mind = torch.zeros(n, device=DEV)
        mind[p] = 0.37
        assert (pick(mind, 20) == p).all()
    p1, p2 = n // 5, n - 2
    mind = torch.zeros(n, device=DEV)
    mind[p1], mind[p2] = 1.0, 3.0
    got = pick(mind)
    assert set(np.unique(got)) <= {p1, p2}
    f = (got == p1).mean()
    assert abs(f - 0.25) < 5 * np.sqrt(0.25 * 0.75 / draws)
    got = pick(None)
    assert got.min() >= 0 and got.max() < n
    hist = np.bincount(got * 4 // n, minlength=4) / draws
    assert np.abs(hist - 0.25).max() < 5 * np.sqrt(0.25 * 0.75 / draws)
