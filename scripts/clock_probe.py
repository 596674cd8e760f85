"""Sample the GPU shader clock while the fp32 MFMA GEMM runs back to back (DVFS check).

python scripts/clock_probe.py [--seconds 6]
Runs gmr_gemm_f32 on 8192^3 (and the 2048 x 7050 x 1000 denoiser shape) in a loop on the GPU while
a child process polls amd-smi / rocm-smi; prints the achieved TF/s and the sampled clocks.
"""
import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

from gmr import kernels as K  # noqa: E402


def sampler(seconds, out):
    cmds = [["amd-smi", "metric", "-g", "0", "--clock"], ["rocm-smi", "-d", "0", "--showclocks"]]
    script = "; ".join(f"({' '.join(c)}) 2>&1" for c in cmds)
    return subprocess.Popen(["bash", "-c", f"for i in $(seq 1 {int(seconds * 2)}); do {script}; sleep 0.5; done"],
                            stdout=out, stderr=subprocess.STDOUT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    a = ap.parse_args()
    for (M, N, Kd, tb) in ((8192, 8192, 8192, True), (2048, 7050, 1000, True)):
        A = torch.randn(M, Kd, device="cuda")
        B = torch.randn((N, Kd) if tb else (Kd, N), device="cuda")
        C = torch.empty(M, N, device="cuda")
        K.gemm(A, B, C, trans_b=tb)
        torch.cuda.synchronize()
        log = open(os.path.join(ROOT, "gpurun_out", f"clock_{M}x{N}x{Kd}.txt"), "w")
        p = sampler(a.seconds, log)
        t0 = time.time()
        n = 0
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        while time.time() - t0 < a.seconds:
            for _ in range(10):
                K.gemm(A, B, C, trans_b=tb)
            n += 10
            torch.cuda.synchronize()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / n
        p.wait()
        log.close()
        print(f"{M}x{N}x{Kd}: {n} launches, {ms * 1e3:.1f} us each, {2.0 * M * N * Kd / ms / 1e9:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
