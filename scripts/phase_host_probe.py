"""Host-bound or GPU-bound, per epoch phase: wall time, host issue time and GPU time of each phase.

python scripts/phase_host_probe.py [--model genrecv1|diffmm] [--reps 3]

For each phase (diffusion, rebuild, BPR) after a warm epoch:
  wall   the phase between two device synchronisations (what the epoch pays);
  host   the phase issued while a ~150 ms GPU blocker (repeated GEMMs) is still running: the host's own
         issue cost (a phase with an internal synchronisation waits for the blocker - flagged);
  gpu    HIP events around that second run: with the launches queued ahead there are no host gaps, so
         this is the phase's GPU-bound time.
wall ~ host > gpu means the phase is host-bound (launch overhead); wall ~ gpu > host means GPU-bound.
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
from gmr import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="genrecv1")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    args = argparse.Namespace(model=a.model, shape="tiktok" if a.model == "genrecv1" else "baby", scoring_dtype=None)
    cfg, ds, tr, tl, vl, model, trainer = bench.setup(args)
    trainer._train_epoch(tl, 0)
    torch.cuda.synchronize()
    from gmr import dist
    rebuild = trainer.rebuild if hasattr(trainer, "rebuild") else model.rebuild_ui_graphs
    st = {}

    def prep_bpr():  # the epoch draw copies its batch offsets to the host: outside the timed region
        model.train()
        st["d"] = tl.epoch()
        torch.cuda.synchronize()

    def bpr():  # Trainer._train_epoch's loop without its final loss read-back
        for b, rank_rows, u, p, ng, pb, pc in tl.batches(st["d"]):
            norm, share = dist.dp_scales(rank_rows)
            trainer._rec_step(u, p, ng, pb, pc, norm, share, 0)
            trainer.optimizer.step()

    phases = (("diffusion", None, lambda: trainer.diffusion_phase(1)), ("rebuild", None, rebuild),
              ("bpr", prep_bpr, bpr))
    X = torch.randn(4096, 4096, device="cuda")
    Y = torch.empty_like(X)

    def blocker(n):
        for _ in range(n):
            K.gemm(X, X, Y, trans_b=True)

    blocker(2)
    torch.cuda.synchronize()
    t = time.perf_counter()
    blocker(10)
    torch.cuda.synchronize()
    nb = max(1, int(0.15 / ((time.perf_counter() - t) / 10)))
    for rep in range(a.reps):
        for name, prep, fn in phases:
            if prep:
                prep()
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            wall = time.perf_counter() - t
            if prep:
                prep()
            blocker(nb)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            t = time.perf_counter()
            fn()
            host = time.perf_counter() - t
            e1.record()
            pending = not e0.query()
            torch.cuda.synchronize()
            print(f"rep {rep} {a.model} {name:9s} wall {1e3 * wall:8.2f} ms  host {1e3 * host:8.2f} ms  "
                  f"gpu {e0.elapsed_time(e1):8.2f} ms  (blocker still running after the issue: {pending})", flush=True)


if __name__ == "__main__":
    main()
