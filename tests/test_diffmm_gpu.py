"""DiffMM fused HIP path vs golden vectors from the reference (tiny shape), through the C-ABI."""
import numpy as np
import pytest
import torch

from oracle import eval_ref, graph_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def tiny_config(**over):
    from gmr.configurator import Config
    cfg = {"dims": [32], "train_batch_size": 40, "eval_batch_size": 16, "epochs": 1, "seed": [999],
           "save_recommended_topk": False}
    cfg.update(over)
    return Config("DiffMM", "baby", cfg)


def build_model(g):
    from gmr.dataloader import TrainDataLoader
    from gmr.dataset import RecDataset
    from gmr.diffmm import DiffMM
    cfg = tiny_config()
    U, I = int(g["U"]), int(g["I"])
    ds = RecDataset.from_arrays(cfg, g["train_rows"], g["train_cols"], np.zeros(len(g["train_rows"])), U, I,
                                g["v_feat"], g["t_feat"])
    tl = TrainDataLoader(cfg, ds, batch_size=40)
    m = DiffMM(cfg, tl)
    s = m.rec_slab
    s.view("E0")[:U].copy_(torch.as_tensor(g["p_uEmbeds"]))
    s.view("E0")[U:].copy_(torch.as_tensor(g["p_iEmbeds"]))
    s.load("image_trans", torch.as_tensor(g["p_image_trans"]))
    s.load("text_trans", torch.as_tensor(g["p_text_trans"]))
    s.load("modal_weight", torch.as_tensor(g["p_modal_weight"]))
    den = m.denoise_model_image.slab
    for ours, ref in [("emb_W", "emb_layer_weight"), ("emb_b", "emb_layer_bias"), ("W1", "in_layers_0_weight"),
                      ("b1", "in_layers_0_bias"), ("W2", "out_layers_0_weight"), ("b2", "out_layers_0_bias")]:
        den.load(ours, torch.as_tensor(g["den_" + ref]))
    from gmr import kernels as K

    def ui(items):
        uptr = torch.arange(U + 1, dtype=torch.int32, device=DEV)
        return K.bipartite_symnorm(U, I, uptr, torch.as_tensor(items.astype(np.int32)).to(DEV), True, 0.0)

    m.image_UI_matrix = ui(g["ui_img_items"])
    m.text_UI_matrix = ui(g["ui_txt_items"])
    return m


@pytest.fixture(scope="module")
def model(golden):
    return build_model(golden("diffmm_tiny"))


def test_forward_mm(model, golden):
    g = golden("diffmm_tiny")
    usr, itm = model.forward_embeddings()
    np.testing.assert_allclose(usr.cpu().numpy(), g["fwd_usr"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(itm.cpu().numpy(), g["fwd_itm"], rtol=1e-5, atol=2e-6)


def test_rec_step_loss_and_grads(model, golden):
    g = golden("diffmm_tiny")
    t = lambda k: torch.as_tensor(g[k].astype(np.int32)).to(DEV)  # noqa: E731
    loss = model.rec_step(t("bpr_users"), t("bpr_pos"), t("bpr_neg"))
    np.testing.assert_allclose(loss.item(), g["rec_loss"], rtol=1e-5)
    U = int(g["U"])
    gE0 = model.rec_slab.gview("E0").cpu().numpy()
    np.testing.assert_allclose(gE0[:U], g["g_uEmbeds"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(gE0[U:], g["g_iEmbeds"], rtol=1e-4, atol=1e-7)
    for n in ("image_trans", "text_trans", "modal_weight"):
        np.testing.assert_allclose(model.rec_slab.gview(n).cpu().numpy(), g["g_" + n], rtol=1e-4, atol=1e-7)
    # the cl parts
    # (contrast terms are inside rec_loss; checked through the total and the gradients)


def test_rec_step_fused_spmm_launches_bit_identical(model, golden):
    """The multi-job SpMM launches of rec_step (gmr_spmm_jobs_f32: Qi/Qt/G, Tcl/T1, OutI/OutT/T2,
    OutI/OutT) give exactly the per-product launches' loss and gradients (GMR_SPMM_FUSE=0 path)."""
    import gmr.diffmm as D
    g = golden("diffmm_tiny")
    t = lambda k: torch.as_tensor(g[k].astype(np.int32)).to(DEV)  # noqa: E731
    out = {}
    saved = D.SPMM_FUSE
    try:
        for fuse in (True, False):
            # all fusions (the OutI/OutT/T2 variant subsumes the side-stream OutI/OutT one) vs none
            D.SPMM_FUSE = (D.FUSE_FWD | D.FUSE_BWD_CL | D.FUSE_BWD3) if fuse else 0
            loss = model.rec_step(t("bpr_users"), t("bpr_pos"), t("bpr_neg"))
            out[fuse] = (loss.clone(), model.rec_slab.grad.clone())
    finally:
        D.SPMM_FUSE = saved
    assert torch.equal(out[True][0].view(torch.int32), out[False][0].view(torch.int32))
    assert torch.equal(out[True][1].view(torch.int32), out[False][1].view(torch.int32))
    try:
        D.SPMM_FUSE = D.FUSE_FWD | D.FUSE_UI_T
        loss = model.rec_step(t("bpr_users"), t("bpr_pos"), t("bpr_neg"))
    finally:
        D.SPMM_FUSE = saved
    assert torch.equal(loss.view(torch.int32), out[False][0].view(torch.int32))
    assert torch.equal(model.rec_slab.grad.view(torch.int32), out[False][1].view(torch.int32))


def test_calculate_loss_autograd(model, golden):
    """Reference-style drop-in: loss.backward() leaves the gradients in .grad."""
    g = golden("diffmm_tiny")
    inter = torch.stack([torch.as_tensor(g[k]) for k in ("bpr_users", "bpr_pos", "bpr_neg")]).to(DEV)
    loss = model.calculate_loss(inter)
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["rec_loss"], rtol=1e-5)
    np.testing.assert_allclose(model.uEmbeds.grad.cpu().numpy(), g["g_uEmbeds"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(model.image_trans.grad.cpu().numpy(), g["g_image_trans"], rtol=1e-4, atol=1e-7)


def test_diffusion_step_injected(model, golden):
    g = golden("diffmm_tiny")
    den = model.denoise_model_image
    Bd = g["dif_x0"].shape[0]
    users = torch.arange(Bd, dtype=torch.int32, device=DEV)
    feats = torch.as_tensor(g["dif_feats"]).to(DEV)
    ie = torch.as_tensor(g["dif_item_embeds"]).to(DEV)
    diff, gc = model.diffusion_step(den, users, feats, ie, 0, noise=torch.as_tensor(g["dif_noise"]).to(DEV),
                                    keep=torch.as_tensor(g["dif_keep"]).to(DEV),
                                    t=torch.as_tensor(g["dif_t"].astype(np.int32)).to(DEV))
    np.testing.assert_allclose(diff.cpu().numpy(), g["dif_diff_loss"], rtol=1e-5)
    np.testing.assert_allclose(gc.cpu().numpy(), g["dif_gc_loss"], rtol=1e-5)
    names = [("emb_W", "emb_layer_weight"), ("emb_b", "emb_layer_bias"), ("W1", "in_layers_0_weight"),
             ("b1", "in_layers_0_bias"), ("W2", "out_layers_0_weight"), ("b2", "out_layers_0_bias")]
    for ours, ref in names:
        want = g["dif_grad_" + ref]
        # fp32 sums over the batch: absolute tolerance relative to the tensor's scale
        np.testing.assert_allclose(den.slab.gview(ours).cpu().numpy(), want, rtol=2e-4,
                                   atol=2e-6 * max(1.0, float(np.abs(want).max())), err_msg=ours)


def test_p_sample_and_top1(model, golden):
    g = golden("diffmm_tiny")
    Bd = g["dif_x0"].shape[0]
    x = torch.empty((Bd, int(g["I"])), device=DEV)
    top = torch.empty((int(g["U"]), 1), dtype=torch.int32, device=DEV)
    model.p_sample_topk(model.denoise_model_image, 0, Bd, top, 1, x_out=x)
    np.testing.assert_allclose(x.cpu().numpy(), g["psample_out"], rtol=1e-5, atol=1e-6)
    assert np.array_equal(top[:Bd].cpu().numpy(), g["psample_top1"])


def test_rebuild_graphs_match_oracle(golden):
    g = golden("diffmm_tiny")
    m = build_model(g)
    m.rebuild_ui_graphs()
    U, I = int(g["U"]), int(g["I"])
    # recompute the image top-1 through p_sample on all users and compare the CSR with the oracle builder
    top = torch.empty((U, 1), dtype=torch.int32, device=DEV)
    m.p_sample_topk(m.denoise_model_image, 0, U, top, 1)
    want = graph_ref.ui_adj_csr(U, I, np.arange(U), top[:, 0].cpu().numpy())
    gi = m.image_UI_matrix
    assert np.array_equal(gi.rowptr.cpu().numpy(), want[0])
    assert np.array_equal(gi.col.cpu().numpy(), want[1])
    assert np.array_equal(gi.val.cpu().numpy().view(np.uint32), want[2].view(np.uint32))


def test_full_sort_predict_and_topk(model, golden):
    g = golden("diffmm_tiny")
    users = torch.as_tensor(g["eval_users"]).to(DEV)
    scores = model.full_sort_predict([users])
    np.testing.assert_allclose(scores.cpu().numpy(), g["eval_scores_raw"], rtol=1e-5, atol=2e-6)
    usr, itm = model.forward_embeddings()
    out = torch.empty((users.numel(), 50), dtype=torch.int32, device=DEV)
    sb = torch.empty((users.numel(), (int(g["I"]) + 3) // 4 * 4), device=DEV)
    model.topk_from_embeddings(usr, itm, users.int(), torch.as_tensor(g["eval_mask_rows"].astype(np.int32)).to(DEV),
                               torch.as_tensor(g["eval_mask_cols"].astype(np.int32)).to(DEV), 50, out, sb)
    # bit-exact selection on our scores; vs the reference top-K up to near-ties
    ours = sb[:users.numel(), :int(g["I"])].cpu().numpy()
    assert np.array_equal(out.cpu().numpy(), eval_ref.topk_rows(ours, 50))
    ref_top = g["eval_topk"]
    s_ref = g["eval_scores_masked"]
    for r in range(len(ref_top)):
        a, b = out[r].cpu().numpy(), ref_top[r]
        diff = np.setdiff1d(a, b)
        # any disagreement must be inside a near-tie group at the K-th boundary
        if len(diff):
            kth = np.sort(s_ref[r][b])[0]
            assert np.all(np.abs(s_ref[r][diff] - kth) <= 1e-6 * max(1.0, abs(kth)))


def test_train_epoch_runs(golden):
    """One full DiffMM epoch (diffusion + rebuild + BPR) and an eval pass on the tiny data."""
    from gmr.dataloader import EvalDataLoader, TrainDataLoader
    from gmr.dataset import RecDataset
    from gmr.trainer import DiffMMTrainer
    g = golden("diffmm_tiny")
    m = build_model(g)
    cfg = m_cfg = tiny_config()
    U, I = int(g["U"]), int(g["I"])
    rng = np.random.default_rng(0)
    lab = (rng.random(len(g["train_rows"])) < 0.2).astype(np.int64)
    ds = RecDataset.from_arrays(cfg, g["train_rows"], g["train_cols"], lab, U, I, g["v_feat"], g["t_feat"])
    tr, va, te = ds.split()
    tl = TrainDataLoader(cfg, tr, batch_size=40)
    vl = EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=16)
    from gmr.diffmm import DiffMM
    model = DiffMM(m_cfg, tl)
    trainer = DiffMMTrainer(cfg, model)
    loss, _ = trainer._train_epoch(tl, 0)
    assert np.isfinite(loss)
    res = trainer.evaluate(vl)
    assert 0.0 <= res["recall@20"] <= 1.0


def test_rec_step_edge_dropped_ui_graphs(golden):
    """D10 SpAdjDropEdge at keep_rate 0.5 (models/diffmm.py:287-301): the dropped UI graphs are no
    longer symmetric, so the backward runs on their transposes (same draws).  Loss and every rec
    gradient against the oracle's autograd on the same dropped graphs."""
    from oracle import model_ref
    from gmr import kernels as K
    g = golden("diffmm_tiny")
    m = build_model(g)
    U, I = int(g["U"]), int(g["I"])
    N = U + I
    drop = {}
    for name in ("image_UI_matrix", "text_UI_matrix"):
        a = getattr(m, name)
        d = K.csr_drop_edges(a, 0.5, seed=11, step=3 + len(drop))
        dt = K.csr_drop_edges(a, 0.5, seed=11, step=3 + len(drop), transposed=True)
        rp, cl, vl = (x.cpu().numpy() for x in (d.rowptr, d.col, d.val))
        assert 0 < d.nnz < a.nnz
        dense = graph_ref.csr_to_dense(rp, cl, vl, N)
        dense_t = graph_ref.csr_to_dense(*(x.cpu().numpy() for x in (dt.rowptr, dt.col, dt.val)), N)
        assert np.array_equal(dense.T, dense_t)          # the transpose holds the same draws
        kept = dense[dense != 0]
        assert np.allclose(kept, graph_ref.csr_to_dense(*(x.cpu().numpy() for x in (a.rowptr, a.col, a.val)),
                                                        N)[dense != 0] / 0.5)
        drop[name] = (d, dt, model_ref.sparse_from_csr(rp, cl, vl, N))
    m.set_ui_matrices(drop["image_UI_matrix"][0], drop["text_UI_matrix"][0], drop["image_UI_matrix"][1],
                      drop["text_UI_matrix"][1])
    t = lambda k: torch.as_tensor(g[k].astype(np.int32)).to(DEV)  # noqa: E731
    loss = m.rec_step(t("bpr_users"), t("bpr_pos"), t("bpr_neg"))
    adj = model_ref.sparse_from_csr(*graph_ref.norm_adj_csr(U, I, g["train_rows"], g["train_cols"]), N)
    names = ["uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight"]
    p = {k: torch.tensor(g["p_" + k], requires_grad=True) for k in names}
    feats = {"v": torch.as_tensor(g["v_feat"]), "t": torch.as_tensor(g["t_feat"])}
    want = model_ref.rec_loss(p, feats, adj, drop["image_UI_matrix"][2], drop["text_UI_matrix"][2],
                              *(torch.as_tensor(g[k]) for k in ("bpr_users", "bpr_pos", "bpr_neg")))
    want.backward()
    np.testing.assert_allclose(loss.item(), want.item(), rtol=1e-5)
    gE0 = m.rec_slab.gview("E0").cpu().numpy()
    np.testing.assert_allclose(gE0[:U], p["uEmbeds"].grad.numpy(), rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(gE0[U:], p["iEmbeds"].grad.numpy(), rtol=1e-4, atol=1e-7)
    for n in ("image_trans", "text_trans", "modal_weight"):
        np.testing.assert_allclose(m.rec_slab.gview(n).cpu().numpy(), p[n].grad.numpy(), rtol=1e-4, atol=1e-7)


def test_rebuild_with_edge_drop(golden):
    """DiffMMTrainer graph rebuild at keep_rate < 1 installs dropped graphs and their transposes."""
    g = golden("diffmm_tiny")
    m = build_model(g)
    m.keepRate = 0.5
    m.rebuild_ui_graphs()
    for a in (m.image_UI_matrix, m.text_UI_matrix):
        at = m._transpose_of(a)
        assert at is not a and at.nnz == a.nnz
        d = graph_ref.csr_to_dense(*(x.cpu().numpy() for x in (a.rowptr, a.col, a.val)), a.n_rows)
        dt = graph_ref.csr_to_dense(*(x.cpu().numpy() for x in (at.rowptr, at.col, at.val)), a.n_rows)
        assert np.array_equal(d.T, dt)
