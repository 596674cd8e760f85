"""Can RCCL run two ranks on ONE GPU (the 1-GPU box)?  Spawns 2 processes on cuda:0 with the nccl backend,
all-reduces a small tensor and all-gathers another; prints the result or the error of each rank.
usage: python scripts/rccl_same_device_probe.py [port]"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=2, device_id=torch.device("cuda", 0))
        t = torch.full((4,), float(rank + 1), device="cuda")
        dist.all_reduce(t)
        g = torch.empty(2 * 3, device="cuda")
        dist.all_gather_into_tensor(g, torch.full((3,), float(rank), device="cuda"))
        torch.cuda.synchronize()
        print(f"rank {rank}: all_reduce {t.tolist()} all_gather {g.tolist()}", flush=True)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - report whatever RCCL says
        print(f"rank {rank}: {type(e).__name__}: {e}", flush=True)


if __name__ == "__main__":
    mp.spawn(worker, args=(int(sys.argv[1]) if len(sys.argv) > 1 else 29611,), nprocs=2, join=True)
