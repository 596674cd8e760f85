"""HIP-graph capture and replay of the DiffMM rec step.

The step forks two side streams (contrastive terms, text projection) and joins them through
reused events; torch.cuda.CUDAGraph captures all of it.  A graph captured on one batch and
replayed on another must give the eager step's loss and gradients bit for bit (same kernels, same
fixed-order sums), and the trainer's GMR_GRAPHS path must train an epoch identically to eager.
"""
import numpy as np
import pytest
import torch

from test_diffmm_gpu import build_model

pytestmark = pytest.mark.gpu


def _batch(g, shift):
    U, I = int(g["U"]), int(g["I"])
    t = lambda k: torch.as_tensor(g[k].astype(np.int32)).cuda()  # noqa: E731
    u, p, n = t("bpr_users"), t("bpr_pos"), t("bpr_neg")
    return (u + shift) % U, p, (n + shift) % I


def test_captured_rec_step_replays_eager(golden):
    g = golden("diffmm_tiny")
    m = build_model(g)
    b0, b1 = _batch(g, 0), _batch(g, 3)
    pl0, pl1 = m._plans(*b0), m._plans(*b1)
    # eager reference on batch 1
    loss_e = m.rec_step(*b1, *pl1).clone()
    grad_e = m.rec_slab.grad.clone()
    # capture on batch 0 (static buffers), replay on batch 1
    static = [t.clone() for t in (*b0, *pl0)]
    m.rec_step(*static)  # warm lazily sized buffers outside the capture
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        loss_g = m.rec_step(*static)
    for dst, src in zip(static, (*b1, *pl1)):
        dst.copy_(src)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(loss_g.view(torch.int32), loss_e.view(torch.int32))
    assert torch.equal(m.rec_slab.grad.view(torch.int32), grad_e.view(torch.int32))


def test_trainer_epoch_with_graphs_matches_eager(golden, monkeypatch):
    from gmr.dataloader import TrainDataLoader
    from gmr.dataset import RecDataset
    from gmr.diffmm import DiffMM
    from gmr.trainer import DiffMMTrainer
    from gmr.utils import init_seed
    from test_diffmm_gpu import tiny_config
    g = golden("diffmm_tiny")
    U, I = int(g["U"]), int(g["I"])
    out = []
    for graphs in ("0", "1"):
        monkeypatch.setenv("GMR_GRAPHS", graphs)
        cfg = tiny_config()
        ds = RecDataset.from_arrays(cfg, g["train_rows"], g["train_cols"], np.zeros(len(g["train_rows"])), U, I,
                                    g["v_feat"], g["t_feat"])
        init_seed(999)
        tl = TrainDataLoader(cfg, ds, batch_size=40)
        m = DiffMM(cfg, tl)
        tr = DiffMMTrainer(cfg, m)
        assert tr._use_graphs == (graphs == "1")
        losses = [tr._train_epoch(tl, e)[0] for e in range(2)]
        out.append((losses, m.rec_slab.data.cpu().numpy()))
    assert out[0][0] == out[1][0]
    np.testing.assert_array_equal(out[0][1], out[1][1])
