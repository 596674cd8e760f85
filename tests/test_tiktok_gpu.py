"""Config 5 — GenRecV1 at the TikTok shape (9,319 users x 6,710 items, image 128-d,
text 768-d; gmr/synthetic.py "tiktok") with the fp16 MFMA scoring GEMM (csrc/score16.hip), judged the
way SURVEY.md section 7 hard part 6 says this config is judged: on Recall/NDCG@20, not index equality.

The reference scores in fp32 (models/genrecv1.py:417-427, torch.matmul at :426) and has no fp16 path,
so parity of the fp16 leg is UNPINNED by reference fixtures; the bar is the fp32 scoring of the SAME
model (whose own parity with the reference is pinned at the tiny shape, test_genrec_gpu.py):
  * after one GenRecV1Trainer epoch at this shape (diffusion + rebuild + BPR, so scores carry
    signal), the valid split is ranked with fp32 and with fp16 scoring;
  * Recall@20 and NDCG@20 (unrounded) agree within 1e-3 absolute;
  * the top-50 lists overlap >= 0.98 on average and the top-20 are identical as sets for >= 95 % of
    users: fp16 rounds each 64-d input to 11 significant bits, which reorders only near ties.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tiktok():
    from gmr.configurator import Config
    from gmr.dataloader import EvalDataLoader, TrainDataLoader
    from gmr.quick_start import popularity_groups
    from gmr.synthetic import make_dataset
    from gmr.utils import get_model, get_trainer, init_seed
    cfg = Config("GenRecV1", "tiktok", {"synthetic": "tiktok", "save_recommended_topk": False, "epochs": 1})
    ds = make_dataset(cfg, "tiktok", seed=0)
    tr, va, te = ds.split()
    pop, warm, _, _ = popularity_groups(cfg, tr)
    cfg["pop_items"], cfg["warm_users"] = pop, warm
    tl = TrainDataLoader(cfg, tr, batch_size=cfg["train_batch_size"], shuffle=True)
    vl = EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=cfg["eval_batch_size"])
    init_seed(999)
    model = get_model("GenRecV1")(cfg, tl)
    trainer = get_trainer("GenRecV1")(cfg, model)
    assert (model.n_users, model.n_items) == (9319, 6710)
    loss, _ = trainer._train_epoch(tl, 0)
    assert np.isfinite(loss)
    return {"model": model, "trainer": trainer, "vl": vl}


def _rank(t, dtype):
    t["model"].scoring_dtype = dtype
    try:
        out = t["trainer"].topk_all(t["vl"], 50).clone()
        sums = t["trainer"].evaluator.device_sums(out, t["vl"]).cpu().numpy().reshape(4, 8) / out.shape[0]
    finally:
        t["model"].scoring_dtype = "fp32"
    return out.cpu().numpy(), sums


def test_tiktok_fp16_scoring_recall_ndcg_vs_fp32(tiktok):
    t32, m32 = _rank(tiktok, "fp32")
    t16, m16 = _rank(tiktok, "fp16")
    n = t32.shape[0]
    assert n > 5000
    # rows 0 / 1 of the sums = recall / ndcg; column 2 = @20 (topk [5, 10, 20, 50])
    for j, name in ((0, "recall@20"), (1, "ndcg@20")):
        assert abs(m16[j, 2] - m32[j, 2]) <= 1e-3, (name, m16[j, 2], m32[j, 2])
        assert m32[j, 2] > 0, name
    over50 = np.mean([len(set(a) & set(b)) / 50.0 for a, b in zip(t16, t32)])
    same20 = np.mean([set(a[:20]) == set(b[:20]) for a, b in zip(t16, t32)])
    assert over50 >= 0.98, over50
    assert same20 >= 0.95, same20
