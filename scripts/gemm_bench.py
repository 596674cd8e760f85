"""Per-shape timing of gmr_gemm_f32 on the DiffMM-baby GEMM shapes (HIP events, 1 process).

python scripts/gemm_bench.py [--tiles 0,64,128] [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

from gmr import kernels as K  # noqa: E402

MF_FLAG = {32: 1 << 25, 16: 1 << 24, 6: 1 << 26}  # GMR_GEMM_MFMA32 / MFMA16 / X6 (split bf16) (include/gmr.h)

# name, M, N, K, trans_a, trans_b, calls per epoch
SHAPES = [
    ("square4096 (NT)", 4096, 4096, 4096, 0, 1, 0),
    ("square8192 (NT)", 8192, 8192, 8192, 0, 1, 0),
    ("psample_h19k (NT)", 19445, 1000, 7050, 0, 1, 10),
    ("psample_out19k (NT)", 19445, 7050, 1000, 0, 1, 10),
    ("psample_h (NT)", 8192, 1000, 7050, 0, 1, 20),
    ("psample_out (NT)", 8192, 7050, 1000, 0, 1, 20),
    # p_sample output layer with the in-place posterior epilogue (as models/diffmm.py p_sample runs it)
    ("psample_post (NT,epi)", 8192, 7050, 1000, 0, 1, 20),
    ("psample_post3061 (NT,epi)", 3061, 7050, 1000, 0, 1, 10),
    ("train_h (NT)", 2048, 1000, 7050, 0, 1, 20),
    ("train_out (NT)", 2048, 7050, 1000, 0, 1, 20),
    ("dh (NN)", 2048, 1000, 7050, 0, 0, 20),
    ("dW2 (TN)", 7050, 1000, 2048, 1, 0, 20),
    ("dW1 (TN)", 1000, 7050, 2048, 1, 0, 20),
    ("proj_v (NN,N=64)", 7050, 64, 4096, 0, 0, 60),
    ("proj_v_grad (TN,N=64)", 4096, 64, 7050, 1, 0, 60),
    ("proj_t (NN,N=64)", 7050, 64, 384, 0, 0, 60),
    ("proj_t_grad (TN,N=64)", 384, 64, 7050, 1, 0, 60),
    ("cl_logits_u (NT,K=64)", 2048, 19445, 64, 0, 1, 60),
    ("cl_dtab_u (TN,N=64)", 19445, 64, 2048, 1, 0, 60),
    ("cl_dp1_u (NN,N=64)", 2048, 64, 19445, 0, 0, 60),
    ("dout+=G f^T (NT,K=64)", 2048, 7050, 64, 0, 1, 40),
    ("train_Z (NN,N=64)", 2048, 64, 7050, 0, 0, 40),
    # GenRecV1 ModalDenoiseTransformer (B = 2048, D = 512, I = 6710 TikTok); calls per epoch ~ 5 batches
    ("tf_lin (NT)", 2048, 512, 512, 0, 1, 5 * 6 * 4 * 6),
    ("tf_dX (NN)", 2048, 512, 512, 0, 0, 5 * 6 * 4),
    ("tf_dW (TN)", 512, 512, 2048, 1, 0, 5 * 6 * 4),
    ("tf_in (NT)", 2048, 512, 6710, 0, 1, 5 * 11),
    ("tf_out (NT)", 2048, 6710, 256, 0, 1, 5 * 11),
    ("tf_dg (NN)", 2048, 256, 6710, 0, 0, 5),
    ("tf_dWout (TN)", 6710, 256, 2048, 1, 0, 5),
    ("tf_dWin (TN)", 512, 6710, 2048, 1, 0, 5),
]


def run(args):
    torch.manual_seed(0)
    dev = "cuda"
    tot_ms = 0.0
    print(f"{'shape':26s} {'tile':>4s} {'us':>9s} {'TF/s':>7s} {'ms/epoch':>9s}")
    for name, M, N, Kd, ta, tb, calls in SHAPES:
        if args.only and not any(o in name for o in args.only.split(",")):
            continue
        r4 = lambda n: (n + 3) // 4 * 4  # noqa: E731  (the model's buffers pad rows to 16 bytes)
        A = torch.randn((Kd, r4(M)) if ta else (M, r4(Kd)), device=dev)[:, :(M if ta else Kd)]
        B = torch.randn((N, r4(Kd)) if tb else (Kd, r4(N)), device=dev)[:, :(Kd if tb else N)]
        C = torch.empty((M, r4(N)), device=dev)[:, :N]
        kw = {}
        if "epi" in name:
            bias = torch.randn(N, device=dev)
            kw = dict(epi=K.EPI_POSTERIOR, bias=bias, aux=C, slope=0.9, beta=0.1)
        best = None
        for tile0 in args.tiles:
          for mf in args.mfma:
           tile = tile0 | (MF_FLAG[mf] if (tile0 or mf == 6) else 0)
           if args.acc and not kw:
               K.gemm(A, B, C, trans_a=bool(ta), trans_b=bool(tb), tile=tile)
               a64 = (A.t() if ta else A).double()
               b64 = (B.t() if tb else B).double()
               ref = a64 @ b64
               scale = a64.abs() @ b64.abs()
               err = ((C.double() - ref).abs() / scale).max().item()
               print(f"{name:26s} {tile0:7d} m{mf} max |C - C64| / (|A||B|) = {err:.3e}", flush=True)
           for split in args.splits:
            for _ in range(3):
                K.gemm(A, B, C, trans_a=bool(ta), trans_b=bool(tb), tile=tile, split_k=split, **kw)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                K.gemm(A, B, C, trans_a=bool(ta), trans_b=bool(tb), tile=tile, split_k=split, **kw)
            e.record()
            torch.cuda.synchronize()
            us = 1e3 * s.elapsed_time(e) / args.reps
            tf = 2.0 * M * N * Kd / (us * 1e-6) / 1e12
            print(f"{name:26s} {tile0:7d} m{mf} s{split:<2d} {us:9.1f} {tf:7.1f} {us * calls / 1e3:9.2f}", flush=True)
            best = us if best is None else min(best, us)
        tot_ms += best * calls / 1e3
    print(f"total GEMM ms/epoch (best tile per shape): {tot_ms:.1f}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="0,64,128,256,256128,128256")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--splits", default="0")
    ap.add_argument("--only", default="", help="substring filter on shape names")
    ap.add_argument("--mfma", default="32", help="MFMA shapes to try: 32 (32x32x2), 16 (16x16x4), 6 (split-bf16)")
    ap.add_argument("--acc", action="store_true", help="also print the error vs an fp64 product")
    a = ap.parse_args()
    a.tiles = [int(t) for t in a.tiles.split(",")]
    a.splits = [int(t) for t in a.splits.split(",")]
    a.mfma = [int(t) for t in a.mfma.split(",")]
    run(a)
