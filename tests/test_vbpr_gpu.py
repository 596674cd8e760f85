"""VBPR on the HIP path vs golden vectors from the reference (models/vbpr.py; tiny shape)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def build_vbpr(g):
    from gmr.configurator import Config
    from gmr.dataloader import TrainDataLoader
    from gmr.dataset import RecDataset
    from gmr.vbpr import VBPR
    U, I = g["p_u_embedding"].shape[0], g["p_i_embedding"].shape[0]
    cfg = Config("VBPR", "baby", {"train_batch_size": 16, "eval_batch_size": 16, "seed": [999],
                                  "save_recommended_topk": False, "topk": [5, 10], "valid_metric": "Recall@10"})
    rng = np.random.default_rng(0)
    rows = np.repeat(np.arange(U), 4)
    cols = rng.integers(0, I, rows.size)
    labels = np.zeros(rows.size)
    labels[3::4] = 1
    labels[2::8] = 2
    ds = RecDataset.from_arrays(cfg, rows, cols, labels, U, I, g["v_feat"], g["t_feat"])
    tl = TrainDataLoader(cfg, ds, batch_size=16)
    m = VBPR(cfg, tl)
    U_ = m.n_users
    ui = m.slab.view("UI")
    ui[:U_].copy_(torch.as_tensor(g["p_u_embedding"]))
    ui[U_:, :64].copy_(torch.as_tensor(g["p_i_embedding"]))
    m.slab.load("W", torch.as_tensor(g["p_item_linear_weight"]))
    m.slab.load("b", torch.as_tensor(g["p_item_linear_bias"]))
    return m, cfg, ds, tl


def test_vbpr_loss_grads_scores(golden):
    g = golden("vbpr_tiny")
    m, *_ = build_vbpr(g)
    t = lambda k: torch.as_tensor(g[k].astype(np.int32)).to(DEV)  # noqa: E731
    loss = m.rec_step(t("users"), t("pos"), t("neg"))
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-5)
    got = [v.cpu().numpy() for v in m.grad_views()]
    for v, k in zip(got, ["u_embedding", "i_embedding", "item_linear_weight", "item_linear_bias"]):
        want = g["g_" + k]
        np.testing.assert_allclose(v, want, rtol=1e-4, atol=1e-6 * np.abs(want).max(), err_msg=k)
    U = g["p_u_embedding"].shape[0]
    scores = m.full_sort_predict([torch.arange(U, device=DEV)])
    np.testing.assert_allclose(scores.cpu().numpy(), g["scores"], rtol=1e-5, atol=1e-5)


def test_vbpr_calculate_loss_autograd(golden):
    g = golden("vbpr_tiny")
    m, *_ = build_vbpr(g)
    inter = torch.stack([torch.as_tensor(g[k]) for k in ("users", "pos", "neg")]).to(DEV)
    loss = m.calculate_loss(inter)
    loss.backward()
    np.testing.assert_allclose(m.item_linear.weight.grad.cpu().numpy(), g["g_item_linear_weight"], rtol=1e-4,
                               atol=1e-6 * np.abs(g["g_item_linear_weight"]).max())
    np.testing.assert_allclose(m.u_embedding.grad.cpu().numpy(), g["g_u_embedding"], rtol=1e-4,
                               atol=1e-6 * np.abs(g["g_u_embedding"]).max())


def test_vbpr_fit(golden):
    from gmr.dataloader import EvalDataLoader
    from gmr.trainer import Trainer
    g = golden("vbpr_tiny")
    m, cfg, ds, tl = build_vbpr(g)
    cfg["epochs"] = 2
    tr, va, te = ds.split()
    vl = EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=16)
    trainer = Trainer(cfg, m)
    best, valid, test = trainer.fit(tl, valid_data=vl, test_data=vl, saved=False)
    assert np.isfinite(trainer.train_loss_dict[0]) and "recall@10" in valid
