#!/bin/bash
# r04q: k-means planted-cluster test alone, after the decoder tests, and a determinism probe
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_genrec_gpu.py -k kmeans > gpurun_out/r04q_a.log 2>&1; echo "alone rc=$?"; grep -E "PASSED|FAILED|^E " gpurun_out/r04q_a.log | head -8
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_decoder_gpu.py tests/test_genrec_gpu.py -k "decoder or kmeans" > gpurun_out/r04q_b.log 2>&1; echo "after decoder rc=$?"; grep -E "PASSED|FAILED|^E " gpurun_out/r04q_b.log | head -14
timeout -k 10 200 python -u - > gpurun_out/r04q_c.log 2>&1 <<'PY'
import sys, numpy as np, torch
sys.path.insert(0, "generative-multimodal-recommendation_amd"); sys.path.insert(0, "tests")
from gmr.kmeans import kmeans_labels
g = dict(np.load("tests/golden/genrecv1_tiny.npz", allow_pickle=False))
keys = [k for k in g if "km_" in k]
print("keys", keys)
from gmr import kernels as K
for N in (1, 3, 4):
    Y = torch.randn(700, 16, device="cuda"); C = torch.randn(N, 16, device="cuda")
    out = torch.empty(700, 4, device="cuda")[:, :N]
    K.gemm(Y, C, out, trans_b=True)
    print("gemm N", N, "max err", float((out - Y @ C.T).abs().max()), flush=True)
X = torch.as_tensor(g[[k for k in keys if "feat" in k][0]]).cuda()
true = g[[k for k in keys if "true" in k][0]]
for s in (11, 11, 12, 13):
    lab = kmeans_labels(X, 4, seed=s).cpu().numpy()
    print("seed", s, "pairs", sorted(set(zip(lab.tolist(), true.tolist()))), flush=True)
print("X", X.shape, float(X.abs().max()))
PY
echo "probe rc=$?"; cat gpurun_out/r04q_c.log | tail -8
