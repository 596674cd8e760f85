"""Is the DiffMM BPR step host-bound?  Separates the host's issue cost from the GPU's own time per step.

python scripts/host_vs_gpu_probe.py [--steps 5]

1. a ~40 ms GPU blocker (repeated GEMMs) is queued first, so the GPU is busy while the host issues;
2. the host then issues --steps rec_steps (with their loader batches pre-built): the wall time of that
   loop is the pure host cost per step (nothing it launches can run yet);
3. HIP events queued before and after those steps time them on the GPU once the blocker drains: with
   every launch already queued there are no host gaps, so that is the GPU-bound time per step.
host cost > GPU time per step means the step is host-bound (the GPU idles between launches).
--tape: the steps are replayed from a host tape recorded on the first batch (gmr/tape.py, the trainer's
default issue path since round 6) instead of issued eagerly from Python.
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--model", default="diffmm")
    ap.add_argument("--tape", action="store_true")
    a = ap.parse_args()
    args = argparse.Namespace(model=a.model, shape="baby" if a.model != "genrecv1" else "tiktok", scoring_dtype=None)
    cfg, ds, tr, tl, vl, model, trainer = bench.setup(args)
    trainer._train_epoch(tl, 0)  # builds the UI graphs, warms every kernel
    torch.cuda.synchronize()
    d = tl.epoch()
    batches = list(tl.batches(d))[:a.steps]
    tape = None
    if a.tape:
        from gmr.tape import Tape
        _, _, u, p, ng, pb, pc = batches[0]
        acc = torch.zeros(1, device="cuda")
        tape = Tape((u, p, ng, pb, pc))
        with tape.recording():
            model.rec_step(u, p, ng, pb, pc, acc=acc)
        torch.cuda.synchronize()
    X = torch.randn(4096, 4096, device="cuda")
    Y = torch.empty_like(X)

    def blocker(n):
        for _ in range(n):
            K.gemm(X, X, Y, trans_b=True)

    # calibrate the blocker
    blocker(2)
    torch.cuda.synchronize()
    t = time.perf_counter()
    blocker(10)
    torch.cuda.synchronize()
    per = (time.perf_counter() - t) / 10
    nb = max(1, int(0.04 / per))
    for rep in range(3):
        torch.cuda.synchronize()
        blocker(nb)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        for _, _, u, p, ng, pb, pc in batches:
            if tape is not None:
                tape.replay((u, p, ng, pb, pc))
            else:
                model.rec_step(u, p, ng, pb, pc)
        t_host = time.perf_counter() - t0
        e1.record()
        pending = not e1.query()
        torch.cuda.synchronize()
        gpu_ms = e0.elapsed_time(e1)
        print(f"{'tape' if tape is not None else 'eager'} rep {rep}: host issue {1e3 * t_host / len(batches):.3f} ms/step, GPU {gpu_ms / len(batches):.3f} "
              f"ms/step (blocker still running when the host finished: {pending})", flush=True)


if __name__ == "__main__":
    main()
