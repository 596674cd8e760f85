"""Measured per-rank work of DiffMM data parallelism at world size W, on ONE GPU.

python scripts/dp_shard_probe.py [--worlds 1,2,4,8] [--epochs 3] [--shape baby] [--mode global|local]

RCCL cannot run two ranks on one GPU (profiles/r04_rccl_same_device_probe.log), so this runs rank 0 of a
W-rank job ALONE: gmr.dist answers world() = W, rank() = 0, and its collectives are elided (all-reduces are
no-ops; all-gathers copy the local shard into every other rank's slot, so the rebuilt graphs stay valid).
Every kernel rank 0 would run - its diffusion slices, its p_sample user shard, its BPR sub-batches over the
replicated full-graph forward/backward, its Adam steps - runs for real, so the phase times are rank 0's
compute time per epoch under the reference's global batch (or GMR_DP_MODE=local).  The collectives the
elided calls stand for are counted (bytes and calls per epoch) and printed, so DESIGN §6 adds their cost
from a stated bandwidth model.  Numbers (loss values) are NOT meaningful here, only times.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from gmr import dist  # noqa: E402

COUNT = {}


def _count(kind, t):
    n, b = COUNT.get(kind, (0, 0))
    COUNT[kind] = (n + 1, b + t.numel() * t.element_size())


def shadow(W):
    """Turn gmr.dist into rank 0 of W with the collectives elided (and counted)."""
    dist.is_dist = lambda: W > 1
    dist.world = lambda: W
    dist.rank = lambda: 0

    def all_reduce_(t):
        _count("all_reduce", t)
        return t

    def all_reduce_start(t):
        _count("all_reduce", t)
        return None

    def all_gather_rows_(full, size):
        _count("all_gather", full)
        for q in range(1, W):
            n = min(size, full.shape[0] - q * size)
            if n > 0:
                full[q * size:q * size + n].copy_(full[:n])
        return full

    def gather_step_rows(local, rank_rows):
        m = max(max(rank_rows), 1)
        full = local.new_zeros((W * m,) + tuple(local.shape[1:]))
        if rank_rows[0]:
            full[:rank_rows[0]].copy_(local[:rank_rows[0]])
        all_gather_rows_(full, m)
        return torch.cat([full[q * m:q * m + rank_rows[q]] for q in range(W)])

    dist.all_reduce_ = all_reduce_
    dist.all_reduce_start = all_reduce_start
    dist.wait = lambda h: None
    dist.all_gather_rows_ = all_gather_rows_
    dist.gather_step_rows = gather_step_rows
    dist.barrier = lambda: None
    dist.max_scalar = lambda x, device: x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--shape", default="baby")
    ap.add_argument("--mode", default="global", choices=["global", "local"])
    a = ap.parse_args()
    os.environ["GMR_DP_MODE"] = a.mode
    os.environ["GMR_PHASE_TIMES"] = "1"
    for W in [int(x) for x in a.worlds.split(",")]:
        shadow(W)
        args = argparse.Namespace(model="diffmm", shape=a.shape, scoring_dtype=None)
        cfg, ds, tr, tl, vl, model, trainer = bench.setup(args)
        trainer._train_epoch(tl, 0)  # warm: kernels loaded, UI graphs built, workspaces sized
        torch.cuda.synchronize()
        COUNT.clear()
        ph = []
        t0 = time.perf_counter()
        for e in range(a.epochs):
            trainer._train_epoch(tl, e + 1)
            ph.append(trainer.phase_ms)
        torch.cuda.synchronize()
        wall = 1e3 * (time.perf_counter() - t0) / a.epochs
        mean = [sum(p[i] for p in ph) / len(ph) for i in range(3)]
        coll = ", ".join(f"{k}: {n / a.epochs:.0f} calls, {b / a.epochs / 1e6:.1f} MB" for k, (n, b) in
                         sorted(COUNT.items()))
        print(f"{a.shape} {a.mode} W={W} rank0: epoch {wall:.2f} ms = diffusion {mean[0]:.2f} + rebuild {mean[1]:.2f}"
              f" + bpr {mean[2]:.2f} ms; per epoch elided collectives: {coll or 'none'}", flush=True)
        del trainer, model, tl, vl
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
