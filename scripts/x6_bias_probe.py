"""Rounding bias of the GEMM kernels on the denoiser's output-layer product (round 6 gc-row diagnosis).

python scripts/x6_bias_probe.py
out = h @ W2^T with h = tanh-like rows (M x 1000) and W2 ~ N(0, 2 / (1000 + I)) (I x 1000), the shape of
models/diffmm.py:355-358's output layer: C on the split-bf16 kernel (gmr_gemm_f32 default plan) and on the
fp32-input MFMA (GMR_GEMM_F32), against fp64 on the host.  Reports the error's mean (bias), its rms, and the
mean relative to the rms: an unbiased kernel has |mean| << rms; a kernel whose accumulation rounds toward zero
(or any directed rounding) shows |mean| of the order of the rms, and such an error adds up linearly in a
downstream product over the items (the gc term's Z = out @ feats)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gmr import kernels as K  # noqa: E402


def main():
    rng = np.random.default_rng(0)
    M, Hd, I = 256, 1000, 7050
    h = np.tanh(rng.standard_normal((M, Hd)) * 0.7).astype(np.float32)
    w = (rng.standard_normal((I, Hd)) * np.sqrt(2.0 / (Hd + I))).astype(np.float32)
    c64 = h.astype(np.float64) @ w.astype(np.float64).T
    feats = rng.standard_normal((I, 64)).astype(np.float32)
    z64 = c64 @ feats.astype(np.float64)
    hd, wd = torch.as_tensor(h).cuda(), torch.as_tensor(w).cuda()
    for name, tile in (("split-bf16 (default plan)", 0), ("fp32-input MFMA", 1 << 27)):
        c = torch.empty((M, (I + 3) // 4 * 4), device="cuda")[:, :I]
        K.gemm(hd, wd, c, trans_b=True, tile=tile)
        torch.cuda.synchronize()
        e = c.double().cpu().numpy() - c64
        ez = e @ feats.astype(np.float64)
        print(f"{name:26s} err mean {e.mean():+.3e} rms {np.sqrt((e ** 2).mean()):.3e} mean/rms "
              f"{e.mean() / np.sqrt((e ** 2).mean()):+.3f} | C rms {np.sqrt((c64 ** 2).mean()):.3e} | "
              f"Z = C @ feats row-norm rel err max {np.max(np.linalg.norm(ez, axis=1) / np.linalg.norm(z64, axis=1)):.3e}")


if __name__ == "__main__":
    main()
