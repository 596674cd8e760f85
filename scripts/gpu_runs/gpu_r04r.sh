#!/bin/bash
# r04r: k-means step-by-step against numpy on the tiny fixture's planted clusters
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u - > gpurun_out/r04r.log 2>&1 <<'PY'
import sys, numpy as np, torch
sys.path.insert(0, "generative-multimodal-recommendation_amd")
from gmr import _lib, kernels as K
from gmr.kernels import ptr, stream
g = dict(np.load("tests/golden/genrecv1_tiny.npz", allow_pickle=False))
Xn = g["r_km_feat"]; n, d = Xn.shape
X = torch.as_tensor(Xn).cuda()
ld = (d + 3) // 4 * 4
Y = torch.empty((n, ld), device="cuda")[:, :d]; mean = torch.empty(d, device="cuda"); scale = torch.empty(d, device="cuda"); xsq = torch.empty(n, device="cuda")
_lib.call("gmr_kmeans_standardize", n, d, ptr(X), K._ld(X), ptr(mean), ptr(scale), ptr(Y), ld, ptr(xsq), stream())
Yn = (Xn - Xn.mean(0)) / Xn.std(0)
print("Y err", float(np.abs(Y.cpu().numpy() - Yn).max()), "xsq err", float(np.abs(xsq.cpu().numpy() - (Yn**2).sum(1)).max()))
C = torch.zeros((4, ld), device="cuda")[:, :d]; csq = torch.zeros(4, device="cuda")
pick = torch.zeros(1, dtype=torch.int32, device="cuda")
_lib.call("gmr_kmeans_pp_pick", n, None, 11, 0, ptr(pick), stream())
_lib.call("gmr_kmeans_take_center", d, ptr(Y), ld, ptr(pick), ptr(C), ld, 0, ptr(xsq), ptr(csq), stream())
p0 = int(pick.item()); print("pick0", p0, "C0 err", float(np.abs(C[0].cpu().numpy() - Yn[p0]).max()), "csq0", float(csq[0]), float((Yn[p0]**2).sum()))
dots = torch.empty((n, 4), device="cuda")[:, :1]
K.gemm(Y, C[0:1], dots, trans_b=True)
print("dots err", float(np.abs(dots.cpu().numpy()[:, 0] - Yn @ Yn[p0]).max()))
mind = torch.empty(n, device="cuda")
_lib.call("gmr_kmeans_min_dist", n, ptr(xsq), ptr(dots), ptr(csq), 0, ptr(mind), 1, stream())
dn = ((Yn - Yn[p0]) ** 2).sum(1)
print("mind err", float(np.abs(mind.cpu().numpy() - dn).max()), "mind sum", float(mind.sum()), float(dn.sum()))
for t in range(3):
    _lib.call("gmr_kmeans_pp_pick", n, ptr(mind), 11, 1024 + 16 + t, ptr(pick), stream())
    pk = int(pick.item()); print("cand", t, pk, "true", int(g["r_km_true"][pk]), "dist", float(dn[pk]))
from gmr.kmeans import kmeans_labels
lab = kmeans_labels(X, 4, seed=11).cpu().numpy()
print("labels", lab.tolist()); print("true", g["r_km_true"].tolist())
PY
echo "rc=$?"; cat gpurun_out/r04r.log
