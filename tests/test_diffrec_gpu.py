"""DiffRec fused HIP path vs golden vectors from the reference (tiny shape), through the C-ABI.

Pins: p_sample over all steps (diffrec.py:291-310), training_losses(reweight=True) loss and
gradients with injected t/noise/dropout (:252-289), the Lt_history/Lt_count bookkeeping
(:279-286, bit-exact) and the importance-sampling distribution (:234-250)."""
import numpy as np
import pytest
import torch

from oracle import model_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
PAIRS = [("emb_W", "emb_layer_weight"), ("emb_b", "emb_layer_bias"), ("W1", "in_layers_0_weight"),
         ("b1", "in_layers_0_bias"), ("W2", "out_layers_0_weight"), ("b2", "out_layers_0_bias")]


def build_diffrec(g, **over):
    from gmr.configurator import Config
    from gmr.dataloader import TrainDataLoader
    from gmr.dataset import RecDataset
    from gmr.diffrec import DiffRec
    U, I = g["x0"].shape
    cfg = {"embedding_size": int(g["E"]), "dims": [int(g["H"])], "steps": int(g["T"]), "train_batch_size": 16,
           "eval_batch_size": 16, "epochs": 1, "seed": [999], "save_recommended_topk": False}
    cfg.update(over)
    cfg = Config("DiffRec", "baby", cfg)
    rows, cols = np.nonzero(g["x0"])
    rng = np.random.default_rng(0)
    labels = np.zeros(len(rows))  # train everything (the fixture's x0); eval splits only feed fit()
    labels[::5], labels[1::7] = 1, 2
    ds = RecDataset.from_arrays(cfg, rows, cols, labels, U, I,
                                rng.standard_normal((I, 8)).astype(np.float32), None)
    tl = TrainDataLoader(cfg, ds, batch_size=16)
    m = DiffRec(cfg, tl)
    for ours, ref in PAIRS:
        m.model.slab.load(ours, torch.as_tensor(g["dnn_" + ref]))
    return m, cfg, ds, tl


def test_diffrec_p_sample(golden):
    g = golden("diffrec_tiny")
    m, *_ = build_diffrec(g)
    m.eval()
    U = g["x0"].shape[0]
    got = m.full_sort_predict([torch.arange(U, device=DEV)])
    np.testing.assert_allclose(got.cpu().numpy(), g["psample"], rtol=1e-4, atol=1e-6)


def test_diffrec_training_step_injected(golden):
    g = golden("diffrec_tiny")
    m, *_ = build_diffrec(g)
    m.train()
    U = g["x0"].shape[0]
    dv = lambda k, dt=torch.float32: torch.as_tensor(g[k]).to(DEV, dt)  # noqa: E731
    users = torch.arange(U, dtype=torch.int32, device=DEV)
    loss = m.rec_step(users, t=dv("train0_t", torch.int32), pt=torch.ones(U, device=DEV),
                      noise=dv("train0_noise"), keep=dv("train0_keep"))
    np.testing.assert_allclose(loss.item(), g["train0_loss"].mean(), rtol=1e-5)
    diff = m._dw["diff"][:U].cpu().numpy()
    np.testing.assert_allclose(diff, g["train0_loss"], rtol=1e-5, atol=1e-12)
    for ours, ref in PAIRS:
        want = g["train0_g_" + ref]
        np.testing.assert_allclose(m.model.slab.gview(ours).cpu().numpy(), want, rtol=1e-4,
                                   atol=2e-5 * np.abs(want).max(), err_msg=ours)
    # the injected-pt path divides the row loss (and its gradient) by pt
    pt = torch.full((U,), 2.0, device=DEV)
    loss2 = m.rec_step(users, t=dv("train0_t", torch.int32), pt=pt, noise=dv("train0_noise"), keep=dv("train0_keep"))
    np.testing.assert_allclose(loss2.item(), g["train0_loss"].mean() / 2.0, rtol=1e-5)


def test_history_update_bit_exact(golden):
    """Feed the reference's own per-row losses: Lt_history / Lt_count must match bit for bit."""
    from gmr import _lib
    from gmr.kernels import ptr, stream
    g = golden("diffrec_tiny")
    T = int(g["T"])
    hist = torch.zeros((T, 10), dtype=torch.float64, device=DEV)
    count = torch.zeros(T, dtype=torch.int32, device=DEV)
    for s in range(int(g["train_steps"])):
        t = torch.as_tensor(g[f"train{s}_t"].astype(np.int32)).to(DEV)
        lv = torch.as_tensor(g[f"train{s}_loss"]).to(DEV, torch.float64)
        _lib.call("gmr_diff_history_update", t.numel(), T, 10, ptr(t), ptr(lv), ptr(hist), ptr(count), stream())
        np.testing.assert_array_equal(count.cpu().numpy(), g[f"train{s}_count"])
        np.testing.assert_array_equal(hist.cpu().numpy(), g[f"train{s}_hist"])
    # many repeats of one t in a batch longer than the LDS chunk: only the last 10 survive, in order
    t = torch.full((3000,), 3, dtype=torch.int32, device=DEV)
    t[::7] = 5
    lv = torch.arange(3000, dtype=torch.float64, device=DEV)
    h0, c0 = hist.cpu().numpy(), count.cpu().numpy()
    _lib.call("gmr_diff_history_update", 3000, T, 10, ptr(t), ptr(lv), ptr(hist), ptr(count), stream())
    want_h, want_c = model_ref.lt_history_update(h0, c0, t.cpu().numpy(), lv.cpu().numpy())
    np.testing.assert_array_equal(hist.cpu().numpy(), want_h)
    np.testing.assert_array_equal(count.cpu().numpy(), want_c)


def test_importance_sampling(golden):
    from gmr import _lib
    from gmr.kernels import ptr, stream
    g = golden("diffrec_tiny")
    T = int(g["T"])
    B = 200000
    hist = torch.as_tensor(g["imp_hist"]).to(DEV)
    t = torch.empty(B, dtype=torch.int32, device=DEV)
    pt = torch.empty(B, dtype=torch.float32, device=DEV)
    # histories not yet full -> uniform t, pt = 1
    partial = torch.full((T,), 10, dtype=torch.int32, device=DEV)
    partial[2] = 9
    _lib.call("gmr_diff_sample_t_importance", B, T, 10, ptr(hist), ptr(partial), 0.001, 7, 0, 0, ptr(t), ptr(pt), stream())
    assert (pt == 1).all() and int(t.min()) >= 0 and int(t.max()) < T
    full = torch.full((T,), 10, dtype=torch.int32, device=DEV)
    _lib.call("gmr_diff_sample_t_importance", B, T, 10, ptr(hist), ptr(full), 0.001, 7, 1, 0, ptr(t), ptr(pt), stream())
    pt_all = model_ref.importance_pt_all(g["imp_hist"])
    tn = t.cpu().numpy()
    np.testing.assert_allclose(pt.cpu().numpy(), (pt_all[tn] * T).astype(np.float32), rtol=1e-6)
    np.testing.assert_allclose(g["imp_pt"], pt_all[g["imp_t"]] * T, rtol=1e-12)  # fixture ties the formula
    freq = np.bincount(tn, minlength=T) / B
    np.testing.assert_allclose(freq, pt_all, atol=5 * np.sqrt(pt_all.max() / B))


def test_diffrec_fit_one_epoch(golden):
    from gmr.dataloader import EvalDataLoader
    from gmr.trainer import Trainer
    g = golden("diffrec_tiny")
    m, cfg, ds, tl = build_diffrec(g, epochs=2, topk=[5, 10], valid_metric="Recall@10")  # I = 37 < 50
    tr, va, te = ds.split()
    vl = EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=16)
    trainer = Trainer(cfg, m)
    best, valid, test = trainer.fit(tl, valid_data=vl, test_data=vl, saved=False)
    assert np.isfinite(trainer.train_loss_dict[0])
    assert "recall@10" in valid
    assert int(m.Lt_count.sum()) > 0
