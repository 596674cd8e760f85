"""Entry point — same CLI surface as the reference's src/main.py (--model/-m, --dataset/-d).

    python main.py --model DiffMM --dataset baby [--synthetic baby] [--epochs N]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from gmr.quick_start import quick_start  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", "-m", type=str, default="DiffMM", help="name of models")
    ap.add_argument("--dataset", "-d", type=str, default="baby", help="name of datasets")
    ap.add_argument("--synthetic", type=str, default=None, help="generate an Amazon-shaped dataset in memory")
    ap.add_argument("--epochs", type=int, default=None)
    args, _ = ap.parse_known_args()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:  # launched by torch.distributed.run: one rank per GPU
        import torch
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))  # RCCL
    cfg = {}
    if args.synthetic:
        cfg["synthetic"] = args.synthetic
    if args.epochs is not None:
        cfg["epochs"] = args.epochs
    quick_start(model=args.model, dataset=args.dataset, config_dict=cfg, save_model=True)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch
        torch.distributed.destroy_process_group()
