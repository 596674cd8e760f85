"""Library calibration for the split-bf16 GEMM's roofline: torch.matmul (hipBLASLt /
rocBLAS) in bf16 and fp32 at the shapes of the epoch's dominant products, beside gmr's split-bf16
kernel on the same fp32 operands.  The bf16 column is what the library's tuned kernels reach on the
matrix cores at that shape; six such products is the split's work.

python scripts/blas_calib.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

from gmr import kernels as K  # noqa: E402

SHAPES = [(19445, 7050, 1000), (19445, 1000, 7050), (2048, 1000, 7050), (2048, 7050, 1000), (8192, 8192, 8192)]


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    torch.manual_seed(0)
    for M, N, Kd in SHAPES:
        a = torch.randn(M, Kd, device="cuda")
        b = torch.randn(N, Kd, device="cuda")
        c = torch.empty(M, N, device="cuda")
        fl = 2.0 * M * N * Kd
        ab, bb = a.bfloat16(), b.bfloat16()
        t_bf = timed(lambda: torch.matmul(ab, bb.T))
        t_32 = timed(lambda: torch.matmul(a, b.T))
        t_x6 = timed(lambda: K.gemm(a, b, c, trans_b=True))
        print(f"{M:6d} x {N:6d} x {Kd:6d}: torch bf16 {fl / t_bf / 1e12:7.1f} TF/s ({1e6 * t_bf:8.1f} us), "
              f"torch fp32 {fl / t_32 / 1e12:6.1f} TF/s, gmr split-bf16 {fl / t_x6 / 1e12:6.1f} TF/s "
              f"({1e6 * t_x6:8.1f} us) = {6 * fl / t_x6 / 1e12:7.1f} TF/s of bf16 products", flush=True)


if __name__ == "__main__":
    main()
