"""Host-side cost of the DiffMM BPR step: wall time of issuing N rec_steps without synchronising
vs with, and a cProfile of the issuing loop (top entries by total time).

python scripts/host_profile.py [--steps 30]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    args = argparse.Namespace(model="diffmm", shape="baby", scoring_dtype=None)
    cfg, ds, tr, tl, vl, model, trainer = bench.setup(args)
    trainer._train_epoch(tl, 0)  # builds the UI graphs, warms every kernel
    torch.cuda.synchronize()
    d = tl.epoch()
    batches = list(tl.batches(d))[:a.steps]

    def run():
        for _, _, u, p, ng, pb, pc in batches:
            model.rec_step(u, p, ng, pb, pc)

    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"{len(batches)} rec_steps: host issue {1e3 * t_issue / len(batches):.3f} ms/step, "
          f"issue+drain {1e3 * t_all / len(batches):.3f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    run()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
