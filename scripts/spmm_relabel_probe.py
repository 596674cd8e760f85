"""Does relabelling users / items for gather locality speed up the side-split SpMM?

python scripts/spmm_relabel_probe.py [--reps 200]

Builds the baby norm_adj (SURVEY 8d synthetic data) under several id orders - identity, reverse
Cuthill-McKee of the bipartite graph (users and items each ranked by their RCM position), BFS from the most
popular item, item popularity (descending) with users ordered by their most popular item, and a random
relabelling as a control - and times the side-split product (the product default) at d = 64, 128 and 256
with HIP events on the current stream.  Each order's result is checked against the identity order's
(permuted back, fp64 tolerance).  Prints us per call and the fraction of the 8(d) roofline.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402
from scipy.sparse.csgraph import breadth_first_order, reverse_cuthill_mckee  # noqa: E402

from gmr import kernels as K  # noqa: E402
from gmr.configurator import Config  # noqa: E402
from gmr.dataloader import TrainDataLoader  # noqa: E402
from gmr.synthetic import make_dataset  # noqa: E402


def orders(U, I, up, ui):
    rows = np.repeat(np.arange(U), np.diff(up))
    A = sp.coo_matrix((np.ones(len(ui)), (rows, ui)), shape=(U, I)).tocsr()
    B = sp.bmat([[None, A], [A.T, None]]).tocsr()
    out = {"identity": (np.arange(U), np.arange(I))}

    def split(perm):
        pos = np.empty(U + I, np.int64)
        pos[perm] = np.arange(U + I)
        return np.argsort(pos[:U], kind="stable"), np.argsort(pos[U:], kind="stable")
    out["rcm"] = split(reverse_cuthill_mckee(B, symmetric_mode=True))
    deg_i = np.bincount(ui, minlength=I)
    start = U + int(np.argmax(deg_i))
    bfs = breadth_first_order(B, start, directed=False, return_predecessors=False)
    rest = np.setdiff1d(np.arange(U + I), bfs)
    out["bfs"] = split(np.concatenate([bfs, rest]))
    item_order = np.argsort(-deg_i, kind="stable")
    rank = np.empty(I, np.int64)
    rank[item_order] = np.arange(I)
    best = np.array([rank[ui[up[u]:up[u + 1]]].min() if up[u + 1] > up[u] else I for u in range(U)])
    out["popularity"] = (np.argsort(best, kind="stable"), item_order)
    rng = np.random.default_rng(1)
    out["random"] = (rng.permutation(U), rng.permutation(I))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    cfg = Config("DiffMM", "baby", {"synthetic": "baby"})
    ds = make_dataset(cfg, "baby", seed=0)
    tr, _, _ = ds.split()
    tl = TrainDataLoader(cfg, tr, batch_size=2048, shuffle=True)
    U, I = ds.user_num, ds.item_num
    N = U + I
    up, ui = tl.uptr_np.astype(np.int64), tl.uitems_np.astype(np.int64)
    dev = "cuda"
    X = torch.randn(N, 256, device=dev)
    ref = {}
    for name, (uo, io) in orders(U, I, up, ui).items():
        # new ids: user uo[j] -> j, item io[j] -> j
        unew = np.empty(U, np.int64)
        unew[uo] = np.arange(U)
        inew = np.empty(I, np.int64)
        inew[io] = np.arange(I)
        lists = [np.sort(inew[ui[up[u]:up[u + 1]]]) for u in uo]
        nptr = np.concatenate([[0], np.cumsum([len(x) for x in lists])]).astype(np.int32)
        nit = np.concatenate(lists).astype(np.int32)
        g = K.bipartite_symnorm(U, I, torch.as_tensor(nptr).to(dev), torch.as_tensor(nit).to(dev), self_loops=False,
                                deg_eps=1e-7)
        perm = torch.as_tensor(np.concatenate([uo, U + io])).to(dev)  # new row j holds old row perm[j]
        Xp = X[perm].contiguous()
        line = [name]
        for nb in (1, 2, 4):
            y = torch.empty((N, 64 * nb), device=dev)
            blocks = [(Xp[:, 64 * b:64 * (b + 1)],) for b in range(nb)]
            g.spmm(y, blocks)
            torch.cuda.synchronize()
            back = torch.empty_like(y)
            back[perm] = y
            if name == "identity":
                ref[nb] = back.clone()
            else:
                err = (back - ref[nb]).abs().max().item() / max(ref[nb].abs().max().item(), 1e-30)
                assert err < 1e-5, (name, nb, err)
            for _ in range(10):
                g.spmm(y, blocks)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                g.spmm(y, blocks)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            d = 64 * nb
            byts = 8 * g.nnz + 4 * (N + 1) + 4 * d * N + 4 * d * N
            line.append(f"d={d}: {us:6.2f} us ({byts / us / 1e6 / 8.0:.3f})")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
