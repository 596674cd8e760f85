"""Where does an epoch phase synchronise with the host?  torch's sync debug mode (warn) reports every
torch-initiated device synchronisation (.item(), .cpu(), blocking copies) with its Python stack.

python scripts/sync_probe.py [--model genrecv1|diffmm]
"""
import argparse
import os
import sys
import traceback
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="genrecv1")
    a = ap.parse_args()
    args = argparse.Namespace(model=a.model, shape="tiktok" if a.model == "genrecv1" else "baby", scoring_dtype=None)
    cfg, ds, tr, tl, vl, model, trainer = bench.setup(args)
    trainer._train_epoch(tl, 0)
    torch.cuda.synchronize()
    rebuild = trainer.rebuild if hasattr(trainer, "rebuild") else model.rebuild_ui_graphs
    seen = {}

    def hook(message, category, filename, lineno, file=None, line=None):
        st = "".join(traceback.format_stack(limit=8)[:-1])
        if st not in seen:
            seen[st] = message
            print(f"--- sync: {message}\n{st}", flush=True)

    warnings.showwarning = hook
    for name, fn in (("diffusion", lambda: trainer.diffusion_phase(1)), ("rebuild", rebuild)):
        print(f"=== {name}", flush=True)
        torch.cuda.set_sync_debug_mode(1)
        fn()
        torch.cuda.set_sync_debug_mode(0)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
