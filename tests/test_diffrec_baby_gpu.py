"""Config 2 — DiffRec at the Amazon-baby shape (19,445 users x 7,050 items; DiffRec.yaml: 100 steps,
dims [300], embedding 64) against the reference's own outputs on the same inputs
(tests/golden/diffrec_baby.npz + diffrec_baby_meta.json, made by `make_golden_baby.py diffrec`, which
ran the reference in the build container).  Through the HIP path:
  * R1   DNN initialisation after init_seed(999): SHA-256 of every parameter equals the reference's
         (models/diffrec.py:313-353, the CPU RNG order) - bit-exact;
  * R3   full_sort_predict = the 100-step p_sample (:291-310, :372-388) of the valid users, masked
         (common/trainer.py:384) and top-50: equal to the reference BY POSITION except inside
         near-tie groups of our own scores (|ds| <= 1e-5 relative: each of the 100 chained denoiser
         steps re-associates its fp32 GEMM sums, ten times the single-product rule of the DiffMM
         tests); the reference's top-50 scores for the stored user sample within 1e-4;
  * D21  Recall/NDCG/Precision/MAP@{5,10,20,50} unrounded within 1e-4 (north-star bar).
"""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = "cuda"
NAMES = {"emb_layer.weight": "emb_W", "emb_layer.bias": "emb_b", "in_layers.0.weight": "W1",
         "in_layers.0.bias": "b1", "out_layers.0.weight": "W2", "out_layers.0.bias": "b2"}


@pytest.fixture(scope="module")
def drb():
    from gmr.configurator import Config
    from gmr.dataloader import EvalDataLoader, TrainDataLoader
    from gmr.synthetic import make_dataset
    from gmr.utils import get_model, get_trainer, init_seed
    cfg = Config("DiffRec", "baby", {"synthetic": "baby", "save_recommended_topk": False, "epochs": 1})
    ds = make_dataset(cfg, "baby", seed=0)
    tr, va, te = ds.split()
    tl = TrainDataLoader(cfg, tr, batch_size=cfg["train_batch_size"], shuffle=True)
    vl = EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=cfg["eval_batch_size"])
    init_seed(999)
    model = get_model("DiffRec")(cfg, tl)
    trainer = get_trainer("DiffRec")(cfg, model)
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "diffrec_baby.npz"), allow_pickle=False))
    with open(os.path.join(ROOT, "tests", "golden", "diffrec_baby_meta.json")) as f:
        meta = json.load(f)
    assert (model.n_users, model.n_items, tl.n_inter, model.steps) == (meta["U"], meta["I"], meta["n_train"],
                                                                        meta["steps"])
    return {"model": model, "trainer": trainer, "vl": vl, "g": g, "meta": meta}


def _sha(t):
    a = np.ascontiguousarray(t.detach().contiguous().cpu().numpy().astype(np.float32))
    return hashlib.sha256(a.tobytes()).hexdigest()


def test_diffrec_baby_init_matches_reference_bit_exact(drb):
    s, want = drb["model"].model.slab, drb["meta"]["param_sha256"]
    got = {ref: _sha(s.view(ours)) for ref, ours in NAMES.items()}
    assert set(got) == set(want)
    bad = [k for k in want if got[k] != want[k]]
    assert not bad, f"DNN parameters differing from the reference init: {bad}"


def test_diffrec_baby_valid_topk_by_position_and_metrics(drb):
    from gmr import kernels as K
    m, g, tr, vl = drb["model"], drb["g"], drb["trainer"], drb["vl"]
    m.eval()
    d = vl.to_device()
    n, E = vl.pr_end, vl.step
    out = torch.empty((n, 50), dtype=torch.int32, device=DEV)
    scores = []
    for lo in range(0, n, E):
        hi = min(n, lo + E)
        sc = m.full_sort_predict([d["eval_u32"][lo:hi].long()])
        m0, m1 = int(d["mask_ptr"][lo]), int(d["mask_ptr"][hi])
        K.mask_scores(sc, d["mask_rows"][m0:m1] - lo, d["mask_cols"][m0:m1])
        K.topk_rows(sc, 50, out[lo:hi])
        scores.append(sc.cpu().numpy())
    scores = np.concatenate(scores)
    ours = out.cpu().numpy().astype(np.int64)
    ref = g["valid_top50"].astype(np.int64)
    assert ours.shape == ref.shape
    S = g["valid_top50_val_sample"].shape[0]
    np.testing.assert_allclose(np.take_along_axis(scores[:S], ref[:S], 1), g["valid_top50_val_sample"], rtol=1e-4,
                               atol=1e-6)
    r, c = np.nonzero(ours != ref)
    s_o, s_r = scores[r, ours[r, c]], scores[r, ref[r, c]]
    tie = np.abs(s_o - s_r) <= 1e-5 * np.maximum(np.abs(s_o), 1e-3)
    assert tie.all(), (f"{int((~tie).sum())} top-50 positions differ outside near ties "
                       f"(first rows {np.unique(r[~tie])[:5]}); {len(r)} differing positions in all")
    sums = tr.evaluator.device_sums(out, vl).cpu().numpy().reshape(4, 8)
    raw = drb["meta"]["valid"]["raw"]
    for j, name in enumerate(["recall", "ndcg", "precision", "map"]):
        for q, k in enumerate([5, 10, 20, 50]):
            assert abs(sums[j, q] / n - raw[name][k - 1]) <= 1e-4, (name, k, sums[j, q] / n, raw[name][k - 1])


def _replay_draws(call, meta_call, B, I, T, keep_prob):
    """The reference's draw order in one training call (models/diffrec.py:234-262, :80) replayed on
    the CPU from the call's seed: t (randint, or multinomial over pt_all once the histories are full),
    randn_like(x_start), then the input dropout's bernoulli."""
    torch.manual_seed(meta_call["seed"])
    if meta_call["importance"]:
        pt_all = torch.as_tensor(call["pt_all"])
        t = torch.multinomial(pt_all, num_samples=B, replacement=True)
        pt = pt_all.gather(dim=0, index=t) * len(pt_all)
    else:
        t = torch.randint(0, T, (B,)).long()
        pt = torch.ones_like(t).float()
    noise = torch.randn(B, I)
    keep = torch.empty(B, I).bernoulli_(keep_prob)
    return t, pt.float(), noise, keep


def test_diffrec_baby_training_calls_vs_reference(drb):
    """R2/R3 training at the baby shape (VERDICT r3 missing #6): three training_losses + backward calls
    of the reference on its loader's first 2,048-user batch from the seed-999 init
    (tests/golden/diffrec_baby_train.npz, `make_golden_baby.py diffrec_train`).  The draws are the
    reference's own, replayed on the CPU from the stored seeds (SHA-256 checked) and injected; the Lt
    histories are set to the reference's state before each call.  Per-row losses rtol 1e-5, the batch
    loss 1e-5, Lt_count exact and Lt_history 1e-5 after each call (call 2 samples t by importance:
    its pt divides the loss), gradients: the small tensors whole, W1 / W2 through row and column
    sums and 4,096 sampled entries, rtol 1e-4."""
    m = drb["model"]
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "diffrec_baby_train.npz"), allow_pickle=False))
    with open(os.path.join(ROOT, "tests", "golden", "diffrec_baby_train_meta.json")) as f:
        meta = json.load(f)
    B, I, T = meta["B"], meta["I"], meta["steps"]
    assert (m.n_items, m.steps) == (I, T)
    users = torch.as_tensor(g["users"]).to(DEV)
    m.train()
    slab = m.model.slab
    keep_prob = float(m.model.keep_prob)
    for s, mc in enumerate(meta["calls"]):
        c = {k[len(f"call{s}_"):]: v for k, v in g.items() if k.startswith(f"call{s}_")}
        t, pt, noise, keep = _replay_draws(c, mc, B, I, T, keep_prob)
        assert hashlib.sha256(noise.numpy().tobytes()).hexdigest() == mc["noise_sha256"], "noise replay differs"
        assert hashlib.sha256(keep.numpy().tobytes()).hexdigest() == mc["keep_sha256"], "dropout replay differs"
        np.testing.assert_array_equal(t.numpy(), c["t"])
        if s == 0:
            m.Lt_history.zero_()
            m.Lt_count.zero_()
        else:
            m.Lt_history.copy_(torch.as_tensor(g[f"call{s - 1}_hist"]))
            m.Lt_count.copy_(torch.as_tensor(g[f"call{s - 1}_count"]))
        slab.zero_grad()
        loss = m.rec_step(users, t=t.to(DEV, torch.int32), pt=pt.to(DEV), noise=noise.to(DEV), keep=keep.to(DEV))
        rows = c["loss_rows"]
        np.testing.assert_allclose(loss.item(), rows.mean(), rtol=1e-5, err_msg=f"call {s}")
        # the history keeps w * mse before the division by pt (:279-288)
        diff = m._dw["diff"][:B].cpu().numpy()
        np.testing.assert_allclose(diff, rows * c["pt"], rtol=1e-5, atol=1e-9, err_msg=f"call {s}")
        np.testing.assert_array_equal(m.Lt_count.cpu().numpy(), c["count"])
        np.testing.assert_allclose(m.Lt_history.cpu().numpy(), c["hist"], rtol=1e-5, atol=1e-9)
        for ref, ours in NAMES.items():
            got = slab.gview(ours).cpu().numpy().astype(np.float64)
            k = "g_" + ref.replace(".", "_")
            if k in c:
                want = c[k]
                np.testing.assert_allclose(got, want, rtol=1e-4, atol=2e-5 * np.abs(want).max(),
                                           err_msg=f"call {s} {ref}")
                continue
            for part, have in (("rowsum", got.sum(1)), ("colsum", got.sum(0)),
                               ("pick", got.reshape(-1)[g["pick_" + ref.replace(".", "_")]])):
                want = c[k + "_" + part]
                np.testing.assert_allclose(have, want, rtol=1e-4, atol=2e-5 * np.abs(want).max(),
                                           err_msg=f"call {s} {ref} {part}")
    slab.zero_grad()
    m.Lt_history.zero_()
    m.Lt_count.zero_()
