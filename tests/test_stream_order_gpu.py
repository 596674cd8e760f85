"""Stream-ordering guards.

The DiffMM rec step runs on three streams (the two InfoNCE terms and the text projection beside the main
chain), the diffusion phase runs each denoiser's chain on its own stream, and the trainer replays the rec step
from a host tape.  A missing join shows up only when timing changes, so these tests change it on purpose:
gmr.kernels.Streams.PERTURB queues a ~300 us sleep kernel at every fork onto one side stream, either on that
side stream (its work starts late: a main-stream read of its results without a join reads a poisoned buffer) or
on the forking stream (the side work runs ahead of everything issued after the fork).  Every work buffer and the
gradient slab are filled with NaN before each run, so a stale read cannot return the previous run's values.
Each perturbed step must equal the unperturbed one bit for bit (same kernels, same sums).
Reference: models/diffmm.py:129-258 (the step), common/trainer.py:144-208 and 491-527 (the loops).
"""
import numpy as np
import pytest
import torch

from test_diffmm_gpu import build_model, tiny_config

pytestmark = pytest.mark.gpu

DEV = "cuda"
CASES = [(w, i) for w in ("side", "main") for i in (0, 1)]


def _poison(m):
    for k, t in m._w.items():  # (part_cl: the side-stream SpMM's hub scratch, whose counters must stay zero)
        if isinstance(t, torch.Tensor) and t.is_floating_point() and k != "part_cl":
            t.fill_(float("nan"))
    m.rec_slab.grad.fill_(float("nan"))
    m.reset_step_buffers()


def _rec(m, g):
    t = lambda k: torch.as_tensor(g[k].astype(np.int32)).to(DEV)  # noqa: E731
    _poison(m)
    loss = m.rec_step(t("bpr_users"), t("bpr_pos"), t("bpr_neg"))
    torch.cuda.synchronize()
    # every gradient segment (the slab's alignment padding between segments is never written)
    return loss.clone(), torch.cat([m.rec_slab.gview(n).reshape(-1) for n in m.rec_slab.offsets])


@pytest.mark.parametrize("where,side", CASES)
def test_rec_step_bit_identical_under_stream_delays(golden, where, side):
    from gmr import kernels as K
    g = golden("diffmm_tiny")
    m = build_model(g)
    m._work(int(g["bpr_users"].size))
    loss0, grad0 = _rec(m, g)
    assert torch.isfinite(grad0).all() and torch.isfinite(loss0).all()
    K.Streams.PERTURB = (where, side, 300)
    try:
        loss1, grad1 = _rec(m, g)
    finally:
        K.Streams.PERTURB = None
    assert torch.equal(loss0, loss1)
    assert torch.equal(grad0, grad1), f"rec-step gradient changed with a delay on the {where} of side stream {side}"


def _trainer(golden, **over):
    from gmr.dataloader import TrainDataLoader
    from gmr.dataset import RecDataset
    from gmr.diffmm import DiffMM
    from gmr.trainer import DiffMMTrainer
    from gmr.utils import init_seed
    g = golden("diffmm_tiny")
    U, I = int(g["U"]), int(g["I"])
    cfg = tiny_config(**over)
    ds = RecDataset.from_arrays(cfg, g["train_rows"], g["train_cols"], np.zeros(len(g["train_rows"])), U, I,
                                g["v_feat"], g["t_feat"])
    init_seed(999)
    tl = TrainDataLoader(cfg, ds, batch_size=40)
    m = DiffMM(cfg, tl)
    tr = DiffMMTrainer(cfg, m)
    tr._train_data = tl
    return tl, m, tr


def _state(m, tr):
    torch.cuda.synchronize()
    return {"rec": m.rec_slab.data.cpu().numpy(), "den": m.denoise_model_image.slab.data.cpu().numpy(),
            "den_t": m.denoise_model_text.slab.data.cpu().numpy(),
            "adam_v": tr.optimizer.state[0]["exp_avg_sq"].cpu().numpy(), "dloss": tr._dloss.cpu().numpy()}


def _epochs(golden, n=2, perturb=None, tape=True, indep=True, over=None):
    from gmr import kernels as K
    from gmr import trainer as T
    tl, m, tr = _trainer(golden, **(over or {}))
    tr._use_tape = tape
    old = T.INDEP_DENOISERS
    T.INDEP_DENOISERS = indep
    K.Streams.PERTURB = perturb
    try:
        losses = [tr._train_epoch(tl, e)[0] for e in range(n)]
    finally:
        K.Streams.PERTURB = None
        T.INDEP_DENOISERS = old
    return losses, _state(m, tr), tr


def _same(a, b):
    la, sa, _ = a
    lb, sb, _ = b
    assert la == lb
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)


def test_taped_epochs_equal_eager_epochs(golden):
    """Two DiffMM epochs (diffusion phase, graph rebuild, BPR phase with rec steps replayed from the host tape,
    re-recorded after the second rebuild) equal the same epochs issued step by step from Python."""
    taped = _epochs(golden, tape=True)
    assert taped[2]._tape is not None and len(taped[2]._tape[1]) > 20
    _same(taped, _epochs(golden, tape=False))


def test_taped_epochs_with_edge_dropping(golden):
    """keep_rate < 1: the rebuilt UI graphs and their transposes change every epoch, so the tape is re-recorded."""
    _same(_epochs(golden, tape=True, over={"keep_rate": 0.5}), _epochs(golden, tape=False, over={"keep_rate": 0.5}))


def test_independent_denoiser_chains_equal_joined_steps(golden):
    """GMR_INDEP_DENOISERS (each denoiser's steps and Adam updates on its own stream, one join per phase) gives
    the per-step-joined phase's denoiser slabs and diffusion losses bit for bit."""
    _same(_epochs(golden, n=1, indep=True), _epochs(golden, n=1, indep=False))


@pytest.mark.parametrize("where,side", CASES)
def test_epochs_bit_identical_under_stream_delays(golden, where, side):
    """Whole epochs (denoiser streams, rebuild sweep on a side stream, taped rec steps) with one side stream
    delayed at every fork."""
    _same(_epochs(golden, n=1), _epochs(golden, n=1, perturb=(where, side, 300)))
