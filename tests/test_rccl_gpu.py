"""The RCCL data-parallel code path on hardware (RCCL never executed).

RCCL refuses two ranks on one GPU (profiles/r04_rccl_same_device_probe.log), so the multi-rank tests run on
gloo.  This runs the same code on RCCL with ONE rank: a spawned process initialises the process group with the
`nccl` backend (RCCL) and `device_id` exactly as bench.py does, and gmr.dist is told the job is distributed
(is_dist() = True at world size 1), so every collective the DP path issues goes through RCCL: the rec step's
asynchronous E0 all-reduce on RCCL's stream and the Trainer's remainder reduce + wait (reduce_slab_grads), the
synchronous all-reduces of losses and denoiser gradients, the nccl branch of all_gather_rows_ (all_gather_
into_tensor), gather_step_rows and max_scalar.  A one-rank SUM all-reduce returns its input, so the results
must equal the single-process (no process group) run bit for bit (tests/test_dist_gpu.py's cases, tiny golden
shape).
"""
import os

import numpy as np
import pytest
import torch

from test_dist_gpu import ROOT, _case, _free_port

pytestmark = pytest.mark.gpu


def _rccl_worker(port, q):
    import sys
    for pth in (ROOT, os.path.join(ROOT, "generative-multimodal-recommendation_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, pth)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch.distributed as tdist
    torch.cuda.set_device(0)
    tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                             device_id=torch.device("cuda", 0))
    try:
        from gmr import dist
        assert tdist.get_backend() == "nccl"
        dist.is_dist = lambda: True  # one rank, every DP collective on RCCL
        res = _case()
        # the remaining collectives of the DP path
        full = torch.arange(12, dtype=torch.int32, device="cuda").view(6, 2).clone()
        dist.all_gather_rows_(full, 6)
        res["gather"] = full.cpu().numpy()
        rows = torch.randn(5, 64, device="cuda")
        res["step_rows_eq"] = np.array([torch.equal(dist.gather_step_rows(rows, [5]), rows)])
        res["max"] = np.array([dist.max_scalar(3.5, "cuda")])
        torch.cuda.synchronize()
        q.put(res)
    finally:
        tdist.destroy_process_group()


@pytest.mark.timeout(240)
def test_rccl_one_rank_dp_path_equals_single_process():
    import torch.multiprocessing as mp
    single = _case()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    pr.start()
    res = q.get(timeout=200)
    pr.join(timeout=60)
    assert pr.exitcode == 0
    for k, v in single.items():
        np.testing.assert_array_equal(res[k], v, err_msg=k)
    np.testing.assert_array_equal(res["gather"], np.arange(12, dtype=np.int32).reshape(6, 2))
    assert res["step_rows_eq"][0] and res["max"][0] == 3.5
