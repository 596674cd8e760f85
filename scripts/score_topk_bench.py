"""Fused eval microbenchmark (gmr_score_topk_f32) at an eval pass's shape: 19,445 users x 7,050 items,
d = 64, k = 50, each row masked at ~6 sorted train items (baby-like).  Prints us per pass (HIP events
over 20 launches) and the index agreement with torch (fp32 GEMM + mask + topk) outside near ties.

python scripts/score_topk_bench.py [--users 19445] [--items 7050] [--dim 64] [--reps 20]
Under rocprofv3 --pmc the launches are the counters' sample."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

from gmr import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=19445)
    ap.add_argument("--items", type=int, default=7050)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    n, I, d, k = a.users, a.items, a.dim, 50
    g = torch.Generator().manual_seed(0)
    usr = (torch.randn(n, d, generator=g) * 0.3).cuda()
    itm = (torch.randn(I, d, generator=g) * 0.3).cuda()
    per = torch.randint(1, 12, (n,), generator=g)
    cols = [torch.unique(torch.randint(0, I, (int(c),), generator=g)) for c in per]
    mptr = torch.zeros(n + 1, dtype=torch.int64)
    mptr[1:] = torch.cumsum(torch.tensor([c.numel() for c in cols]), 0)
    mcols = torch.cat(cols).to(torch.int32).cuda()
    mptr = mptr.cuda()
    out = torch.empty(n, k, dtype=torch.int32, device="cuda")
    val = torch.empty(n, k, device="cuda")
    K.score_topk(usr, itm, None, mptr, mcols, k, out, val)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        K.score_topk(usr, itm, None, mptr, mcols, k, out, val)
    e.record()
    torch.cuda.synchronize()
    us = 1e3 * s.elapsed_time(e) / a.reps
    # check against torch on the first 2048 rows
    m = min(n, 2048)
    sc = usr[:m].double() @ itm.double().T
    rows = torch.repeat_interleave(torch.arange(m, device="cuda"), (mptr[1:m + 1] - mptr[:m]))
    sc[rows, mcols[:int(mptr[m])].long()] = -1e10
    ref = torch.topk(sc, k, dim=1)
    got = out[:m].long()
    diff = got != ref.indices
    sg = torch.gather(sc, 1, got)
    tie = (sg - ref.values).abs() <= 1e-6 * ref.values.abs().clamp_min(1e-3)
    bad = int((diff & ~tie).sum())
    print(f"score_topk n={n} I={I} d={d} k={k}: {us:8.1f} us per pass, {n / us:6.2f} M users/s, "
          f"{2.0 * n * I * d / us / 1e6:6.1f} TF/s; positions differing outside 1e-6 ties: {bad}", flush=True)
    if bad:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
