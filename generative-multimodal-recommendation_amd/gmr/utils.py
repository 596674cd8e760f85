"""Registry, seeding, early stopping — mirror utils/utils.py of the reference (:28-111, :118-125)."""
import datetime
import importlib
import random

import numpy as np
import torch

# model name -> module of this package (reference: importlib of models.<name.lower()>, utils.py:28-41)
_MODELS = {"DiffMM": "diffmm", "DiffRec": "diffrec", "VBPR": "vbpr", "GenRecV1": "genrecv1"}


def get_local_time():
    return datetime.datetime.now().strftime("%b-%d-%Y-%H-%M-%S")


def get_model(model_name):
    if model_name not in _MODELS:
        raise ValueError(f"model {model_name} is not on the MI355X hot path; available: {sorted(_MODELS)}")
    mod = importlib.import_module(f"{__package__}.{_MODELS[model_name]}")
    return getattr(mod, model_name)


def get_trainer(model_name=None):
    """DiffMM -> DiffMMTrainer, GenRecV1 -> GenRecV1Trainer, anything else -> Trainer (utils.py:44-58)."""
    mod = importlib.import_module(f"{__package__}.trainer")
    if model_name == "DiffMM":
        return mod.DiffMMTrainer
    if model_name == "GenRecV1":
        return mod.GenRecV1Trainer
    return mod.Trainer


def init_seed(seed):
    random.seed(seed)
    np.random.seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
    torch.manual_seed(seed)


def early_stopping(value, best, cur_step, max_step, bigger=True):
    stop_flag = False
    update_flag = False
    better = value > best if bigger else value < best
    if better:
        cur_step = 0
        best = value
        update_flag = True
    else:
        cur_step += 1
        if cur_step > max_step:
            stop_flag = True
    return best, cur_step, stop_flag, update_flag


def dict2str(result_dict):
    return "".join(str(k) + ": " + "%.04f" % v + "    " for k, v in result_dict.items())
