"""Launch-shape sweep of the side-split SpMM (csrc/spmm_side.hip) on the baby-shaped DiffMM graphs.

python scripts/spmm_side_sweep.py [--reps 100]
For task sizes T, workgroups per XCD and entries in flight, times norm_adj / a rebuilt UI graph /
a collapsed UI graph (one item row holding 80 % of the users) at d = 64, 128, 256 (graph-replayed
back-to-back launches, HIP events), next to the lane plan; prints us and the SURVEY 8(d) fraction."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gmr import _lib  # noqa: E402
from gmr import kernels as K  # noqa: E402
from gmr.configurator import Config  # noqa: E402
from gmr.dataloader import TrainDataLoader  # noqa: E402
from gmr.synthetic import make_dataset  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return 1e3 * s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--Ts", default="16,32")
    ap.add_argument("--wpx", default="64,128,256")
    ap.add_argument("--tws", default="16,32")
    ap.add_argument("--ebs", default="16")
    args = ap.parse_args()
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
    t_hub = rng.integers(0, I, U).astype(np.int32)
    t_hub[rng.random(U) < 0.8] = 0
    ar = torch.arange(U + 1, dtype=torch.int32, device=dev)
    graphs = {"norm_adj": K.bipartite_symnorm(U, I, uptr, uit, False, 1e-7, seg_nnz=K.SPMM_NORM_ADJ),
              "ui_top1": K.bipartite_symnorm(U, I, ar, torch.as_tensor(rng.integers(0, I, U).astype(np.int32)).to(dev),
                                             True, 0.0),
              "ui_hub": K.bipartite_symnorm(U, I, ar, torch.as_tensor(t_hub).to(dev), True, 0.0)}
    X = torch.randn(N, 256, device=dev)
    lib = _lib.load()
    print(f"{'graph':9s} {'d':>3s} {'plan':>18s} {'us':>8s} {'frac':>6s}")
    for name, g in graphs.items():
        for nb in (1, 2, 4):
            d = 64 * nb
            byts = 8.0 * g.nnz + 4.0 * (N + 1) + 8.0 * d * N
            Y = torch.empty(N, d, device=dev)
            blocks = [(X[:, 64 * b:64 * (b + 1)],) for b in range(nb)]
            side = g.side
            g.side = None
            us = timed(lambda: g.spmm(Y, blocks), args.reps)
            ref = Y.clone()
            g.side = side
            print(f"{name:9s} {d:3d} {'lane':>18s} {us:8.2f} {byts / us / 1e3 / 8000:6.3f}", flush=True)
            for T, TW in ((int(x), int(y)) for x in args.Ts.split(",") for y in args.tws.split(",")):
                g.build_side_plan(U, T | (TW << 16))
                for wpx in (int(x) for x in args.wpx.split(",")):
                    for eb in (int(x) for x in args.ebs.split(",")):
                        _lib.call("gmr_spmm_side_tune", wpx, eb)
                        us = timed(lambda: g.spmm(Y, blocks), args.reps)
                        err = float(((Y - ref).abs() / (ref.abs() + 1e-3)).max())
                        tag = f"T{T}/{TW} w{wpx} eb{eb}"
                        print(f"{name:9s} {d:3d} {tag:>18s} {us:8.2f} {byts / us / 1e3 / 8000:6.3f} {err:.1e}",
                              flush=True)
    lib.gmr_spmm_side_tune(64, 16)


if __name__ == "__main__":
    main()
