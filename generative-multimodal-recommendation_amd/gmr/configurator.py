"""Layered YAML configuration — mirrors utils/configurator.py of the reference.

Order: configs/overall.yaml -> configs/dataset/<dataset>.yaml -> configs/model/<model>.yaml
(-> configs/mg.yaml when mg) -> config_dict.  Missing keys read as None
(reference utils/configurator.py:125-129).  The configs directory is taken from the current
working directory when it has one (as the reference does, :72-76), else from this package.
"""
import os
import re

import yaml

_PKG_CONFIGS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs")


def _yaml_loader():
    # accept 1e-4 style floats (PyYAML's default resolver needs a dot) — configurator.py:93-105
    loader = yaml.SafeLoader

    class L(loader):
        pass

    L.add_implicit_resolver(
        "tag:yaml.org,2002:float",
        re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
            |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
            |\.[0-9_]+(?:[eE][-+][0-9]+)?
            |[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+\.[0-9_]*
            |[-+]?\.(?:inf|Inf|INF)
            |\.(?:nan|NaN|NAN))$""", re.X),
        list("-+0123456789."))
    return L


class Config:
    def __init__(self, model=None, dataset=None, config_dict=None, mg=False, config_dir=None):
        config_dict = dict(config_dict or {})
        config_dict["model"] = model
        config_dict["dataset"] = dataset
        self.config_dir = config_dir or self._find_dir()
        self.final_config_dict = self._load(config_dict, mg)
        self.final_config_dict.update(config_dict)
        self._set_defaults()
        self._init_device()

    @staticmethod
    def _find_dir():
        cwd = os.path.join(os.getcwd(), "configs")
        if os.path.isfile(os.path.join(cwd, "overall.yaml")):
            return cwd
        return _PKG_CONFIGS

    def _load(self, config_dict, mg):
        files = [os.path.join(self.config_dir, "overall.yaml"),
                 os.path.join(self.config_dir, "dataset", f"{config_dict['dataset']}.yaml"),
                 os.path.join(self.config_dir, "model", f"{config_dict['model']}.yaml")]
        if mg:
            files.append(os.path.join(self.config_dir, "mg.yaml"))
        out, hyper = {}, []
        for f in files:
            if os.path.isfile(f):
                with open(f, encoding="utf-8") as fh:
                    data = yaml.load(fh.read(), Loader=_yaml_loader()) or {}
                if data.get("hyper_parameters"):
                    hyper.extend(data["hyper_parameters"])
                out.update(data)
        out["hyper_parameters"] = hyper
        return out

    def _set_defaults(self):
        vm = (self.final_config_dict.get("valid_metric") or "Recall@20").split("@")[0]
        self.final_config_dict["valid_metric_bigger"] = vm.lower() not in ("rmse", "mae", "logloss")
        if "seed" not in self.final_config_dict["hyper_parameters"]:
            self.final_config_dict["hyper_parameters"] += ["seed"]

    def _init_device(self):
        import torch
        use_gpu = self.final_config_dict.get("use_gpu", True)
        self.final_config_dict["device"] = torch.device("cuda" if (use_gpu and torch.cuda.is_available()) else "cpu")

    def __setitem__(self, key, value):
        if not isinstance(key, str):
            raise TypeError("index must be a str.")
        self.final_config_dict[key] = value

    def __getitem__(self, item):
        return self.final_config_dict.get(item, None)

    def __contains__(self, key):
        if not isinstance(key, str):
            raise TypeError("index must be a str.")
        return key in self.final_config_dict

    def get(self, key, default=None):
        v = self.final_config_dict.get(key, None)
        return default if v is None else v

    def __str__(self):
        return "\n" + "\n".join(f"{k}={v}" for k, v in self.final_config_dict.items()) + "\n\n"

    __repr__ = __str__
