"""K8 fused InfoNCE microbenchmark at the DiffMM baby shapes (B = 2048 gathered rows against the
user table, 19,445 rows, and the item table, 7,050 rows; d = 64), graph-replayed, HIP events.

python scripts/contrast_bench.py [--reps 20]   (GMR_CL_WG_ROWS / GMR_CL_WG_TABLE tune the grid)
Prints us per call and the MFMA rate over 3 x 2 B n d flops (logits in each pass + the two
products)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

from gmr import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    B = 2048
    for n in (19445, 7050):
        CLN = torch.nn.functional.normalize(torch.randn(n, 128, generator=g), dim=1).to(dev)
        CLN[:, 64:] = torch.nn.functional.normalize(CLN[:, 64:], dim=1)
        CLN[:, :64] = torch.nn.functional.normalize(CLN[:, :64], dim=1)
        nodes = torch.randint(0, n, (B,), generator=g, dtype=torch.int32).to(dev)
        P = CLN[nodes.long(), :64].contiguous()
        loss = torch.empty(B, device=dev)
        contrib = torch.empty(B, 128, device=dev)
        dT = torch.empty(n, 64, device=dev)
        ws = K.contrast_workspace(B, n, dev, f"bench{n}")

        def call():
            K.contrast_fused(P, CLN[:, 64:], CLN, nodes, 0, 10.0, 0.01, loss, contrib, dT, ws)

        for _ in range(3):
            call()
        torch.cuda.synchronize()
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg):
            for _ in range(args.reps):
                call()
        cg.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        cg.replay()
        e.record()
        torch.cuda.synchronize()
        us = 1e3 * s.elapsed_time(e) / args.reps
        fl = 3 * 2.0 * B * n * 64 + 2.0 * B * n * 64  # rows pass: S + U; table pass: S + dT
        print(f"n={n:6d}: {us:8.1f} us/call  {fl / us / 1e6:6.1f} TF/s  loss[0]={loss[0].item():.6f} "
              f"dT.sum={dT.double().sum().item():.6e}")


if __name__ == "__main__":
    main()
