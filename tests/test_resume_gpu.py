"""checkpoint / resume including the generated graphs.

The reference saves {config, epoch, state_dict, optimizer, best_valid_score} on a best-valid
update (common/trainer.py:334-335, 345-366) but never resumes (start_epoch = 0, :97) and does not
save DiffMM's generated UI matrices (models/diffmm.py:263-274).  Here a checkpoint also holds the
UI graphs, the denoiser optimisers and the positions of the device random streams, so:
  save after epoch e -> fresh model + trainer -> resume -> epoch e+1
must give exactly (bit for bit: same kernels, same draws) what the uninterrupted run gives.
The checkpoint is read back with torch.load(weights_only=True): it holds tensors and plain data.
"""
import numpy as np
import pytest
import torch

from test_diffmm_gpu import tiny_config

pytestmark = pytest.mark.gpu


def _run(golden, tmp_path, keep_rate=1.0):
    from gmr.dataloader import TrainDataLoader
    from gmr.dataset import RecDataset
    from gmr.diffmm import DiffMM
    from gmr.trainer import DiffMMTrainer
    from gmr.utils import init_seed
    g = golden("diffmm_tiny")
    U, I = int(g["U"]), int(g["I"])
    cfg = tiny_config(checkpoint_dir=str(tmp_path), keep_rate=keep_rate)
    ds = RecDataset.from_arrays(cfg, g["train_rows"], g["train_cols"], np.zeros(len(g["train_rows"])), U, I,
                                g["v_feat"], g["t_feat"])

    def fresh():
        init_seed(999)
        tl = TrainDataLoader(cfg, ds, batch_size=40)
        m = DiffMM(cfg, tl)
        return tl, m, DiffMMTrainer(cfg, m)

    # uninterrupted: epochs 0, 1, 2
    tl, m, tr = fresh()
    tr._train_data = tl
    losses = []
    for e in range(3):
        losses.append(tr._train_epoch(tl, e)[0])
        if e == 0:
            tr._save_checkpoint(0)
    want = {"rec": m.rec_slab.data.cpu().numpy(), "den": m.denoise_model_image.slab.data.cpu().numpy(),
            "den_t": m.denoise_model_text.slab.data.cpu().numpy(),
            "adam_v": tr.optimizer.state[0]["exp_avg_sq"].cpu().numpy()}
    # resumed: load epoch 0's checkpoint into a fresh model, train epochs 1 and 2
    tl2, m2, tr2 = fresh()
    path = tmp_path / "DiffMM-baby.pth"
    tr2.resume_checkpoint(str(path), train_data=tl2)
    assert tr2.start_epoch == 1
    got_losses = [tr2._train_epoch(tl2, e)[0] for e in (1, 2)]
    assert got_losses == losses[1:]
    np.testing.assert_array_equal(m2.rec_slab.data.cpu().numpy(), want["rec"])
    np.testing.assert_array_equal(m2.denoise_model_image.slab.data.cpu().numpy(), want["den"])
    np.testing.assert_array_equal(m2.denoise_model_text.slab.data.cpu().numpy(), want["den_t"])
    np.testing.assert_array_equal(tr2.optimizer.state[0]["exp_avg_sq"].cpu().numpy(), want["adam_v"])
    ck = torch.load(str(path), map_location="cpu", weights_only=True)
    for k in ("config", "epoch", "state_dict", "optimizer", "best_valid_score"):
        assert k in ck                                   # the reference's keys (trainer.py:355-361)
    assert "image_UI_matrix" in ck["generated_graphs"]
    return ck


def test_resume_continues_the_same_run(golden, tmp_path):
    _run(golden, tmp_path)


def test_resume_with_dropped_graphs(golden, tmp_path):
    ck = _run(golden, tmp_path, keep_rate=0.5)
    assert "image_UI_matrix_T" in ck["generated_graphs"]


def test_resume_diffrec_importance_state(golden, tmp_path):
    """DiffRec's importance-sampling state (Lt_history / Lt_count, diffrec.py:279-286) and its Philox
    step travel with the checkpoint: the resumed epochs equal the uninterrupted ones bit for bit."""
    from gmr.trainer import Trainer
    from gmr.utils import init_seed
    from test_diffrec_gpu import build_diffrec
    g = golden("diffrec_tiny")

    def fresh():
        init_seed(999)
        m, cfg, ds, tl = build_diffrec(g, checkpoint_dir=str(tmp_path))
        return tl, m, Trainer(cfg, m)

    tl, m, tr = fresh()
    tr._train_data = tl
    losses = []
    for e in range(4):
        losses.append(tr._train_epoch(tl, e)[0])
        if e == 1:
            tr._save_checkpoint(1)
    assert int(m.Lt_count.sum()) > 0
    want = (m.model.slab.data.cpu().numpy(), m.Lt_history.cpu().numpy(), m.Lt_count.cpu().numpy(), m._step)
    tl2, m2, tr2 = fresh()
    tr2.resume_checkpoint(str(tmp_path / "DiffRec-baby.pth"), train_data=tl2)
    assert tr2.start_epoch == 2
    assert [tr2._train_epoch(tl2, e)[0] for e in (2, 3)] == losses[2:]
    np.testing.assert_array_equal(m2.model.slab.data.cpu().numpy(), want[0])
    np.testing.assert_array_equal(m2.Lt_history.cpu().numpy(), want[1])
    np.testing.assert_array_equal(m2.Lt_count.cpu().numpy(), want[2])
    assert m2._step == want[3]
