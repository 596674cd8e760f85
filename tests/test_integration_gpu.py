"""INTEGRATION.md's ctypes binding block, executed as written against torch ops on the GPU:
the stub a reference maintainer would add must work verbatim."""
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _load_stub():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = re.search(r"```python\n(# GenMMRec/src/common/gmr_bind.py.*?)```", text, re.S).group(1)
    lib = os.path.join(ROOT, "generative-multimodal-recommendation_amd", "gmr", "libgmr_hip.so")
    block = block.replace('"/path/to/gmr/libgmr_hip.so"', repr(lib))
    ns = {}
    exec(compile(block, "INTEGRATION.md", "exec"), ns)
    return ns


def test_integration_stub_spmm_and_topk():
    ns = _load_stub()
    rng = np.random.default_rng(3)
    n = 500
    rows = rng.integers(0, n, 4000)
    cols = rng.integers(0, n, 4000)
    rows = np.concatenate([rows, np.zeros(700, np.int64)])  # one hub row (> 128 nnz: partial path)
    cols = np.concatenate([cols, rng.integers(0, n, 700)])
    vals = rng.standard_normal(len(rows)).astype(np.float32)
    adj = torch.sparse_coo_tensor(torch.as_tensor(np.stack([rows, cols])), torch.as_tensor(vals), (n, n)).coalesce()
    x = torch.randn(n, 64)
    want = torch.sparse.mm(adj.double(), x.double()).float()
    g = ns["CSR"](adj.cuda())
    got = g.mm(x.cuda()).cpu()
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5)
    s = torch.randn(37, 1000)
    s[:, 5] = s[:, 9]  # exact ties resolve to the lower index
    idx = ns["topk"](s.cuda(), 20).cpu()
    order = np.lexsort((np.arange(1000)[None, :].repeat(37, 0), -s.numpy()), axis=1)[:, :20]
    assert np.array_equal(idx.numpy(), order)
