"""Data-parallel sharding rules (gmr/dist.py) on CPU with the gloo backend, world_size 2.

The device kernels cannot run here, so the DP arithmetic is checked on the torch-CPU oracle:
ranks compute the DiffMM rec loss on their slice of a batch with the global-row normalisation
and regulariser share of gmr.dist.dp_scales, the gradients are summed with gmr.dist.all_reduce_,
and the result must equal the single-process full-batch gradient.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_rules():
    from gmr import dist
    for n in (0, 1, 7, 8, 19445):
        for w in (1, 2, 3, 8):
            spans = [dist.shard(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            pads = [dist.padded_shard(n, w, r) for r in range(w)]
            covered = sorted(i for lo, hi, _ in pads for i in range(lo, hi))
            assert covered == list(range(n))
    assert dist.shard_sizes(2048, 3) == [683, 683, 682]
    assert dist.shard_sizes(2, 4) == [1, 1, 0, 0]
    assert dist.dp_scales(dist.shard_sizes(974, 8)) == (974.0, 1.0 / 8)
    assert dist.dp_scales([2, 1, 0, 0]) == (3.0, 1.0 / 2)


def test_sub_batch_offsets():
    """Every reference batch (train_batch_size rows of the epoch draw) is cut into `world`
    contiguous sub-batches that tile it exactly (gmr/dataloader.py sub_batch_offsets)."""
    from types import SimpleNamespace

    from gmr import dist
    from gmr.dataloader import TrainDataLoader
    for n_inter, B in ((121_846, 2048), (100, 40), (5, 2048)):
        nb = -(-n_inter // B)
        for w in (1, 2, 3, 8):
            offs = TrainDataLoader.sub_batch_offsets(SimpleNamespace(n_inter=n_inter, batch_size=B), w)
            assert len(offs) == nb * w + 1 and offs[0] == 0 and offs[-1] == n_inter
            assert np.all(np.diff(offs) >= 0)
            for b in range(nb):
                lo, hi = b * B, min((b + 1) * B, n_inter)
                assert offs[b * w] == lo and offs[(b + 1) * w] == hi
                assert list(np.diff(offs[b * w:(b + 1) * w + 1])) == dist.shard_sizes(hi - lo, w)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "generative-multimodal-recommendation_amd")):
        sys.path.insert(0, p)
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from gmr import dist
    from oracle import graph_ref, model_ref
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "diffmm_tiny.npz"), allow_pickle=False))
    U, I = int(g["U"]), int(g["I"])
    N = U + I
    adj = model_ref.sparse_from_csr(*graph_ref.norm_adj_csr(U, I, g["train_rows"], g["train_cols"]), N)
    iadj = model_ref.sparse_from_csr(*graph_ref.ui_adj_csr(U, I, np.arange(U), g["ui_img_items"]), N)
    tadj = model_ref.sparse_from_csr(*graph_ref.ui_adj_csr(U, I, np.arange(U), g["ui_txt_items"]), N)
    feats = {"v": torch.as_tensor(g["v_feat"]), "t": torch.as_tensor(g["t_feat"])}
    names = ["uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight"]
    p = {k: torch.tensor(g["p_" + k], requires_grad=True) for k in names}
    u, po, ne = (torch.as_tensor(g[k]) for k in ("bpr_users", "bpr_pos", "bpr_neg"))
    B = len(u)
    lo, hi = dist.shard(B)
    rows = [dist.shard(B, world, r)[1] - dist.shard(B, world, r)[0] for r in range(world)]
    norm, share = dist.dp_scales(rows)
    reg = (p["uEmbeds"].norm(2).square() + p["iEmbeds"].norm(2).square()) * 1e-6
    part = model_ref.rec_loss(p, feats, adj, iadj, tadj, u[lo:hi], po[lo:hi], ne[lo:hi]) - reg
    loss = part * ((hi - lo) / norm) + share * reg
    loss.backward()
    grads = torch.cat([p[k].grad.reshape(-1) for k in names])
    # two buckets in flight at once, as the diffusion phase exchanges its two denoiser slabs
    half = grads.numel() // 2
    handles = [dist.all_reduce_start(grads[:half]), dist.all_reduce_start(grads[half:])]
    for h in handles:
        dist.wait(h)
    lv = torch.tensor([loss.item()], dtype=torch.float64)
    dist.all_reduce_(lv)
    # all-gather of a padded user shard (the graph-rebuild exchange)
    lo2, hi2, size = dist.padded_shard(U)
    full = torch.full((world * size, 3), -1, dtype=torch.int32)
    full[rank * size:rank * size + (hi2 - lo2)] = torch.arange(lo2, hi2, dtype=torch.int32)[:, None]
    dist.all_gather_rows_(full, size)
    if rank == 0:
        out_q.put((grads.numpy(), float(lv.item()), full.numpy()))
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_gradient_equals_full_batch_gloo():
    from oracle import graph_ref, model_ref
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    grads, loss, full = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "diffmm_tiny.npz"), allow_pickle=False))
    # the single-process loss/gradient of the whole batch is the reference's (golden) one
    np.testing.assert_allclose(loss, g["rec_loss"], rtol=1e-5)
    want = np.concatenate([g["g_" + k].reshape(-1) for k in
                           ["uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight"]])
    np.testing.assert_allclose(grads, want, rtol=1e-4, atol=1e-7)
    U = int(g["U"])
    lo_hi = [(lo, hi) for lo, hi, _ in (__import__("gmr.dist", fromlist=["x"]).padded_shard(U, world, r)
                                         for r in range(world))]
    size = -(-U // world)
    got = np.concatenate([full[r * size:r * size + hi - lo, 0] for r, (lo, hi) in enumerate(lo_hi)])
    assert np.array_equal(got, np.arange(U))


@pytest.mark.parametrize("mode", ["global", "local"])
@pytest.mark.parametrize("n,B,w", [(1000, 96, 3), (7, 4, 2), (4096, 2048, 8), (95, 96, 4)])
def test_step_slices_cover_every_row_once(monkeypatch, mode, n, B, w):
    """dist.step_slices: over all ranks every row lies in exactly one slice; rank_rows agrees with
    the slices; row0 is the rank's offset in the step's concatenated rows; 'global' keeps
    ceil(n / B) steps of one batch, 'local' ceil(n / B / w) steps of w whole batches."""
    from gmr import dist
    monkeypatch.setenv("GMR_DP_MODE", mode)
    seen = np.zeros(n, np.int64)
    steps = None
    for r in range(w):
        sl = list(dist.step_slices(n, B, w, r))
        steps = len(sl) if steps is None else steps
        assert len(sl) == steps
        for g, lo, hi, blo, bhi, rank_rows, row0 in sl:
            assert hi - lo == rank_rows[r] and row0 == sum(rank_rows[:r])
            assert blo <= lo <= hi <= bhi
            seen[lo:hi] += 1
    assert (seen == 1).all()
    nb = -(-n // B)
    assert steps == (nb if mode == "global" else -(-nb // w))


def _early_reduce_main(rank, world, port, out_q):
    """gmr.trainer.reduce_slab_grads with a model that all-reduces the head of one slab from inside its
    step (DiffMM's E0 gradient): rank 0 ran the step (head already in flight), rank 1 was idle in a short
    last batch and issues both reduces itself; the collectives must match and the sums be exact."""
    import sys
    from types import SimpleNamespace
    for p in (ROOT, os.path.join(ROOT, "generative-multimodal-recommendation_amd")):
        sys.path.insert(0, p)
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from gmr import dist
    from gmr.trainer import reduce_slab_grads
    s0 = SimpleNamespace(grad=torch.arange(10, dtype=torch.float32) * (rank + 1))
    s1 = SimpleNamespace(grad=torch.full((4,), float(rank + 7)))

    class Model:
        early = dist.all_reduce_start(s0.grad[:3]) if rank == 0 else None

        def early_reduce_cut(self, slab):
            return 3 if slab is s0 else None

        def take_early_reduce(self):
            h, Model.early = Model.early, None
            return h

    reduce_slab_grads(Model(), [s0, s1])
    out_q.put((rank, s0.grad.numpy().copy(), s1.grad.numpy().copy()))
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.timeout(120)
def test_reduce_slab_grads_early_head_and_idle_rank():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_early_reduce_main, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for _, g0, g1 in res:
        np.testing.assert_array_equal(g0, np.arange(10, dtype=np.float32) * 3)
        np.testing.assert_array_equal(g1, np.full(4, 15.0, np.float32))
