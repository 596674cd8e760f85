"""Top-K (k = 50) per-row timing on eval-shaped score matrices (HIP-graph replayed, 1 process).

python scripts/topk_bench.py   -> us per 4096-row batch at I = 7050 (baby) and 18357 (sports)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

from gmr import kernels as K  # noqa: E402


def main():
    torch.manual_seed(0)
    for I in (7050, 18357):
        E = 4096
        ub, it = torch.randn(E, 64, device="cuda") * 0.1, torch.randn(I, 64, device="cuda") * 0.1
        sc = torch.empty(E, (I + 3) // 4 * 4, device="cuda")[:, :I]
        K.gemm(ub, it, sc, trans_b=True)
        out = torch.empty(E, 50, dtype=torch.int32, device="cuda")
        K.topk_rows(sc, 50, out)
        ref = torch.topk(sc, 50, dim=1).indices.to(torch.int32)
        same = (out == ref).float().mean().item()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(10):
                K.topk_rows(sc, 50, out)
        g.replay()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        us = 1e3 * s.elapsed_time(e) / 10
        print(f"I={I:6d} E={E}: {us:8.1f} us per batch, {E / us:6.2f} M rows/s, "
              f"{E * I * 4 / us / 1e3:7.0f} GB/s of scores, index agreement with torch.topk {same:.4f}")


if __name__ == "__main__":
    main()
