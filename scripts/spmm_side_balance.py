"""Per-side critical path of the side-split SpMM: the baby graphs timed whole and with the item side's
tasks removed from the plan (its XCDs idle), so each side's time alone shows whether one side's
XCDs finish late.  python scripts/spmm_side_balance.py [--reps 100]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gmr import kernels as K  # noqa: E402
from gmr.configurator import Config  # noqa: E402
from gmr.dataloader import TrainDataLoader  # noqa: E402
from gmr.synthetic import make_dataset  # noqa: E402
from spmm_side_sweep import timed  # noqa: E402

H_TASK, H_NT0, H_NT1, H_EMPTY, H_NE0, H_NE1, H_WAVE, H_NW0, H_NW1 = 4, 5, 6, 7, 8, 9, 16, 17, 18


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
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
    ar = torch.arange(U + 1, dtype=torch.int32, device=dev)
    graphs = {"norm_adj": K.bipartite_symnorm(U, I, uptr, uit, False, 1e-7, seg_nnz=K.SPMM_NORM_ADJ),
              "ui_top1": K.bipartite_symnorm(U, I, ar, torch.as_tensor(rng.integers(0, I, U).astype(np.int32)).to(dev),
                                             True, 0.0)}
    X = torch.randn(N, 256, device=dev)
    for name, g in graphs.items():
        plan, split = g.side
        h = plan[:32].cpu().numpy()
        print(f"{name}: nnz {g.nnz} tasks {h[H_NT0]}/{h[H_NT1]} wave tasks {h[H_NW0]}/{h[H_NW1]} "
              f"empty {h[H_NE0]}/{h[H_NE1]}", flush=True)
        for nb in (1, 2, 4):
            Y = torch.empty(N, 64 * nb, device=dev)
            blocks = [(X[:, 64 * b:64 * (b + 1)],) for b in range(nb)]
            full = timed(lambda: g.spmm(Y, blocks), args.reps)
            saved = plan[:32].clone()
            plan[H_NT1] = 0
            plan[H_NE1] = 0
            plan[H_NW1] = 0
            side0 = timed(lambda: g.spmm(Y, blocks), args.reps)
            plan[:32].copy_(saved)
            # item side alone: the user side's counts zeroed and the item side's tables re-based to index 0
            plan[H_TASK] = int(saved[H_TASK]) + 4 * int(saved[H_NT0])
            plan[H_NT0] = 0
            plan[H_WAVE] = int(saved[H_WAVE]) + 4 * int(saved[H_NW0])
            plan[H_NW0] = 0
            plan[H_EMPTY] = int(saved[H_EMPTY]) + int(saved[H_NE0])
            plan[H_NE0] = 0
            side1 = timed(lambda: g.spmm(Y, blocks), args.reps)
            plan[:32].copy_(saved)
            print(f"  d={64 * nb:3d} whole {full:7.2f} us   user side alone {side0:7.2f} us   item side alone "
                  f"{side1:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
