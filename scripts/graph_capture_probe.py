"""Diagnose HIP-graph capture of the DiffMM rec step (faulthandler prints the Python stack if the
capture or the replay crashes).  python scripts/graph_capture_probe.py"""
import argparse
import faulthandler
import os
import sys

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = argparse.Namespace(model="diffmm", shape="baby", scoring_dtype=None)
    cfg, ds, tr, tl, vl, model, trainer = bench.setup(args)
    trainer._train_epoch(tl, 0)
    torch.cuda.synchronize()
    d = tl.epoch()
    _, _, u, p, ng, pb, pc = list(tl.batches(d))[0]
    static = [t.clone() for t in (u, p, ng, pb, pc)]
    model.rec_step(*static)  # warm every lazily sized buffer outside the capture
    torch.cuda.synchronize()
    print("eager ok", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss = model.rec_step(*static)
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("replayed, loss", float(loss.item()), flush=True)


if __name__ == "__main__":
    main()
