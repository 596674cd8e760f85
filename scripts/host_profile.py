"""Host-side profile (cProfile) of one warm epoch: where the host issue time goes (Python wrappers vs the
ctypes calls into libgmr_hip.so, which include the HIP launch).

python scripts/host_profile.py [--model genrecv1|diffmm] [--top 45]
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
    ap.add_argument("--model", default="genrecv1")
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    args = argparse.Namespace(model=a.model, shape="tiktok" if a.model == "genrecv1" else "baby", scoring_dtype=None)
    cfg, ds, tr, tl, vl, model, trainer = bench.setup(args)
    trainer._train_epoch(tl, 0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    trainer._train_epoch(tl, 1)
    torch.cuda.synchronize()
    print(f"epoch (no profiler) {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    trainer._train_epoch(tl, 2)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(a.top)
    st.sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
