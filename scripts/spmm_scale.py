"""SpMM roofline fraction vs graph size: is the lane-plan SpMM latency/launch-bound at baby size?

python scripts/spmm_scale.py [--scales 1,2,4,8,16,32] [--reps 50]
Builds norm_adj of baby-shaped synthetic bipartite graphs scaled by f (f x 19,445 users,
f x 7,050 items, f x 160,792 interactions; per-user degree 5 + Poisson, Zipf(0.8) item popularity
as gmr/synthetic.py, drawn vectorised and de-duplicated per user), times the default DiffMM
norm_adj product (lane plan, d = 128 and 256, HIP-graph replay) and prints the SURVEY 8(d)
algorithmic bytes, GB/s and the fraction of the 8 TB/s HBM roofline.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gmr import kernels as K  # noqa: E402


def interactions(U, I, n, seed):
    rng = np.random.default_rng(seed)
    deg = np.minimum(np.maximum(5, 5 + rng.poisson(max(n / U - 5.0, 0.0), size=U)), I)
    perm = rng.permutation(I)
    pop = np.empty(I)
    pop[perm] = 1.0 / np.arange(1, I + 1) ** 0.8
    pop /= pop.sum()
    users = np.repeat(np.arange(U, dtype=np.int64), deg)
    items = rng.choice(I, size=users.size, p=pop)
    key = np.unique(users * I + items)  # sorted by user, then item; duplicates dropped
    u, it = key // I, key % I
    uptr = np.zeros(U + 1, np.int64)
    np.add.at(uptr, u + 1, 1)
    return np.cumsum(uptr).astype(np.int32), it.astype(np.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scales", default="1,2,4,8,16,32")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--nbs", default="2,4")
    args = ap.parse_args()
    dev = "cuda"
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print(f"{'scale':>5s} {'users':>8s} {'items':>8s} {'nnz':>9s} {'d':>4s} {'us':>9s} {'MB':>8s} {'GB/s':>7s} {'frac':>6s}")
    for f in [int(x) for x in args.scales.split(",")]:
        U, I, n = 19445 * f, 7050 * f, 160792 * f
        uptr, uit = interactions(U, I, n, seed=f)
        g = K.bipartite_symnorm(U, I, torch.as_tensor(uptr).to(dev), torch.as_tensor(uit).to(dev),
                                self_loops=False, deg_eps=1e-7, seg_nnz=K.SPMM_NORM_ADJ)
        N = U + I
        X = torch.randn(N, 256, device=dev)
        for nb in [int(x) for x in args.nbs.split(",")]:
            Y = torch.empty(N, 64 * nb, device=dev)
            blocks = [(X[:, 64 * b:64 * b + 64],) for b in range(nb)]
            for _ in range(3):
                g.spmm(Y, blocks)
            torch.cuda.synchronize()
            reps = max(5, args.reps // f)
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg):
                for _ in range(reps):
                    g.spmm(Y, blocks)
            cg.replay()
            torch.cuda.synchronize()
            s.record()
            cg.replay()
            e.record()
            torch.cuda.synchronize()
            us = 1e3 * s.elapsed_time(e) / reps
            d = 64 * nb
            byts = 8.0 * g.nnz + 4.0 * (N + 1) + 4.0 * d * N * 2
            gbs = byts / us / 1e3
            print(f"{f:5d} {U:8d} {I:8d} {g.nnz:9d} {d:4d} {us:9.2f} {byts / 1e6:8.1f} {gbs:7.0f} {gbs / 8000:6.3f}",
                  flush=True)
        del g, X, Y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
