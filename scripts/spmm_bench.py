"""SpMM microbenchmark on the baby-shaped DiffMM graphs (HIP events, 1 process).

python scripts/spmm_bench.py [--segs 128,64,32] [--reps 50]
Times gmr_spmm_csr_f32 (graph-replayed reps) for norm_adj (no self loops) and a rebuilt UI graph (top-1 per user +
self loops) at 1, 2 and 4 column blocks, per plan segment length, checks every variant against
the first, and prints GB/s with the SURVEY.md 8(d) byte formula.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gmr import kernels as K  # noqa: E402
from gmr.configurator import Config  # noqa: E402
from gmr.dataloader import TrainDataLoader  # noqa: E402
from gmr.synthetic import make_dataset  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", default="128,1024")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--panel", action="store_true", help="also time column-panel sources (lane plans)")
    ap.add_argument("--cap", type=int, default=0, help="also time norm_adj with item degrees capped at this (hub test)")
    ap.add_argument("--graphs", default="norm_adj,ui_top1,ui_hub", help="graphs to time")
    ap.add_argument("--nbs", default="1,2,4", help="64-column blocks per product")
    args = ap.parse_args()
    segs = [int(x) for x in args.segs.split(",")]
    cfg = Config("DiffMM", "baby", {"synthetic": "baby"})
    ds = make_dataset(cfg, "baby", seed=0)
    tr, _, _ = ds.split()
    tl = TrainDataLoader(cfg, tr, batch_size=2048, shuffle=True)
    U, I = ds.user_num, ds.item_num
    N = U + I
    dev = "cuda"
    uptr = torch.as_tensor(tl.uptr_np).to(dev)
    uit = torch.as_tensor(tl.uitems_np).to(dev)
    rng = np.random.default_rng(0)
    top1 = torch.as_tensor(rng.integers(0, I, U).astype(np.int32)).to(dev)
    # a rebuilt graph after p_sample collapsed: 80 % of the users pick the same item (one hub row
    # holding ~15.6k users, the shape seen in the DiffMM step)
    t_hub = rng.integers(0, I, U).astype(np.int32)
    t_hub[rng.random(U) < 0.8] = 0
    top1_hub = torch.as_tensor(t_hub).to(dev)
    graphs = {}
    for seg in segs:
        graphs[("norm_adj", seg)] = K.bipartite_symnorm(U, I, uptr, uit, self_loops=False, deg_eps=1e-7, seg_nnz=seg)
        graphs[("ui_top1", seg)] = K.bipartite_symnorm(U, I, torch.arange(U + 1, dtype=torch.int32, device=dev), top1,
                                                       self_loops=True, deg_eps=0.0, seg_nnz=seg)
        graphs[("ui_hub", seg)] = K.bipartite_symnorm(U, I, torch.arange(U + 1, dtype=torch.int32, device=dev),
                                                      top1_hub, self_loops=True, deg_eps=0.0, seg_nnz=seg)
    names = [n for n in ("norm_adj", "ui_top1", "ui_hub") if n in args.graphs.split(",")]
    if args.cap:
        # hub test: the same users and items, each item keeping only its first `cap` users
        up, ui = tl.uptr_np, tl.uitems_np
        seen = np.zeros(I, np.int64)
        keep_rows = []
        for u in range(U):
            its = ui[up[u]:up[u + 1]]
            k = []
            for i in its:
                if seen[i] < args.cap:
                    seen[i] += 1
                    k.append(i)
            keep_rows.append(np.array(k, np.int32))
        cptr = np.zeros(U + 1, np.int32)
        cptr[1:] = np.cumsum([len(k) for k in keep_rows])
        cit = np.concatenate(keep_rows).astype(np.int32)
        for seg in segs:
            graphs[("adj_cap", seg)] = K.bipartite_symnorm(U, I, torch.as_tensor(cptr).to(dev), torch.as_tensor(cit).to(dev),
                                                          self_loops=False, deg_eps=1e-7, seg_nnz=seg)
        names.append("adj_cap")
        deg = np.bincount(tl.uitems_np, minlength=I)
        print(f"item degree max {deg.max()} p99 {np.percentile(deg, 99):.0f}; capped nnz {2 * len(cit)} of {2 * len(ui)}")
    X = torch.randn(N, 256, device=dev)
    t = torch.empty_like(X)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(args.reps):
        t.copy_(X)
    e.record()
    torch.cuda.synchronize()
    us = 1e3 * s.elapsed_time(e) / args.reps
    print(f"copy N x 256 fp32: {us:.1f} us, {2 * X.numel() * 4 / us / 1e3:.0f} GB/s")
    print(f"{'graph':10s} {'nnz':>7s} {'nb':>2s} {'seg':>4s} {'us':>8s} {'GB/s':>7s} {'frac':>6s} max|diff|")
    for name in names:
        for nb in [int(x) for x in args.nbs.split(",")]:
            ref = None
            for seg in segs:
                g = graphs[(name, seg)]
                Y = torch.empty(N, 64 * nb, device=dev)
                blocks = [(X[:, 64 * b:64 * b + 64],) for b in range(nb)]
                for _ in range(3):
                    g.spmm(Y, blocks)
                torch.cuda.synchronize()
                # the reps are replayed from a HIP graph: back-to-back launches without the Python
                # call overhead, which is longer than these kernels
                cg = torch.cuda.CUDAGraph()
                with torch.cuda.graph(cg):
                    for _ in range(args.reps):
                        g.spmm(Y, blocks)
                cg.replay()
                torch.cuda.synchronize()
                s.record()
                cg.replay()
                e.record()
                torch.cuda.synchronize()
                us = 1e3 * s.elapsed_time(e) / args.reps
                d = 64 * nb
                byts = 8.0 * g.nnz + 4.0 * (N + 1) + 4.0 * d * N * 2
                gbs = byts / us / 1e3
                if ref is None:
                    ref = Y.clone()
                diff = (Y - ref).abs().max().item()
                print(f"{name:10s} {g.nnz:7d} {nb:2d} {seg:4d} {us:8.2f} {gbs:7.0f} {gbs / 8000:6.3f} {diff:.2e}")
                if args.panel and (seg & K.SPMM_LANE_PLAN):
                    # the same product from a column-panel copy of X (gmr_spmm_panel_f32)
                    W = 32 if nb == 4 else 16
                    S = 64 * nb // W
                    Xp = X[:, :64 * nb].reshape(N, S, W).permute(1, 0, 2).contiguous()
                    Y2 = torch.empty_like(Y)
                    cg2 = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(cg2):
                        for _ in range(args.reps):
                            K.spmm_panel(g, Y2, Xp, nb)
                    cg2.replay()
                    torch.cuda.synchronize()
                    s.record()
                    cg2.replay()
                    e.record()
                    torch.cuda.synchronize()
                    us = 1e3 * s.elapsed_time(e) / args.reps
                    gbs = byts / us / 1e3
                    same = bool(torch.equal(Y2.view(torch.int32), Y.view(torch.int32)))
                    print(f"{name + '/panel':10s} {g.nnz:7d} {nb:2d} {seg:4d} {us:8.2f} {gbs:7.0f} {gbs / 8000:6.3f} "
                          f"bit-identical={same}")


if __name__ == "__main__":
    main()
