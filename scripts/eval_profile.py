"""Time full-rank eval passes of the bench workload (after one training epoch) and print the
per-pass wall time; run under rocprofv3 --kernel-trace --stats for the per-kernel split.
python scripts/eval_profile.py [--model diffmm] [--passes 10] [--fused 0|1]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--model", default="diffmm")
ap.add_argument("--passes", type=int, default=10)
ap.add_argument("--fused", default="1")
a = ap.parse_args()
os.environ["GMR_EVAL_FUSED"] = a.fused
import torch  # noqa: E402

import bench  # noqa: E402

args = argparse.Namespace(model=a.model, shape=bench.DEFAULT_SHAPE[a.model], scoring_dtype=None)
cfg, ds, tr, tl, vl, model, trainer = bench.setup(args)
trainer._train_epoch(tl, 0)
trainer.evaluate(vl)
torch.cuda.synchronize()
ts = []
for _ in range(a.passes):
    t0 = time.time()
    trainer.evaluate(vl)
    ts.append(time.time() - t0)
print(f"{a.model} fused={a.fused} users={vl.pr_end} pass ms: min {1e3 * min(ts):.3f} median "
      f"{1e3 * sorted(ts)[len(ts) // 2]:.3f} -> {vl.pr_end / min(ts) / 1e6:.2f}M users/s", flush=True)
