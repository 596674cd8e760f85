"""Flat parameter slabs and the fused Adam that updates them.

A model's parameters live in one contiguous fp32 device buffer (16-byte aligned segments,
optionally with a padded leading dimension so the GEMM can use float4 loads); every
nn.Parameter is a view into it and every .grad a view into a twin gradient slab.  One
gmr_adam_f32 launch then updates a whole model (reference: torch.optim.Adam over
model.parameters(), common/trainer.py:125-142).
"""
import math

import torch
import torch.nn as nn

from . import kernels as K

ALIGN = 64  # floats


class Slab:
    def __init__(self, specs, device):
        """specs: list of (name, shape, ld) — ld = padded row stride for 2-D params or None."""
        self.offsets, self.layout = {}, {}
        off = 0
        for name, shape, ld in specs:
            if len(shape) == 2:
                rows, cols = shape
                ld = ld or cols
                size = (rows - 1) * ld + cols if rows else 0
            else:
                ld = None
                size = int(math.prod(shape))
            self.offsets[name] = off
            self.layout[name] = (tuple(shape), ld)
            off += (size + ALIGN - 1) // ALIGN * ALIGN
        self.numel = max(off, ALIGN)
        self.data = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=device)

    def _view(self, buf, name):
        shape, ld = self.layout[name]
        off = self.offsets[name]
        if len(shape) == 2:
            return buf.as_strided(shape, (ld, 1), off)
        return buf[off:off + int(math.prod(shape))].view(shape)

    # views are cached per name (GenRecV1's step reads ~8,000 parameter views per epoch and is host-issue-bound;
    # building one costs ~2 us); a cached view is dropped when its buffer is no longer the slab's
    def view(self, name):
        c = self.__dict__.setdefault("_vcache", {})
        v = c.get(name)
        if v is None or v[0] is not self.data:
            v = c[name] = (self.data, self._view(self.data, name))
        return v[1]

    def gview(self, name):
        c = self.__dict__.setdefault("_gcache", {})
        v = c.get(name)
        if v is None or v[0] is not self.grad:
            v = c[name] = (self.grad, self._view(self.grad, name))
        return v[1]

    def parameter(self, name):
        p = nn.Parameter(self.view(name))
        p.grad = self.gview(name)
        return p

    def load(self, name, value):
        self.view(name).copy_(value)

    def zero_grad(self):
        K.zero_(self.grad)


class FlatAdam:
    """torch.optim.Adam semantics (single-tensor path) over one or more slabs."""

    def __init__(self, slabs, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.slabs = list(slabs)
        self.base_lr = lr
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.state = [{"step": 0, "exp_avg": torch.zeros_like(s.data), "exp_avg_sq": torch.zeros_like(s.data)}
                      for s in self.slabs]
        self.param_groups = [{"lr": lr, "betas": betas, "eps": eps, "weight_decay": weight_decay}]

    def zero_grad(self):
        for s in self.slabs:
            s.zero_grad()

    def step(self):
        for s, st in zip(self.slabs, self.state):
            st["step"] += 1
            K.adam(s.data, s.grad, st["exp_avg"], st["exp_avg_sq"], self.lr, self.betas[0], self.betas[1], self.eps,
                   self.weight_decay, st["step"])

    def set_lr_factor(self, f):
        self.lr = self.base_lr * f
        self.param_groups[0]["lr"] = self.lr

    def state_dict(self):
        return {"state": [{k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in st.items()}
                          for st in self.state], "param_groups": self.param_groups}

    def load_state_dict(self, sd):
        if len(sd["state"]) != len(self.state):
            raise ValueError("optimizer state holds a different number of slabs")
        if sd.get("param_groups"):
            self.lr = float(sd["param_groups"][0]["lr"])
            self.param_groups[0]["lr"] = self.lr
        for st, src in zip(self.state, sd["state"]):
            st["step"] = src["step"]
            st["exp_avg"].copy_(src["exp_avg"])
            st["exp_avg_sq"].copy_(src["exp_avg_sq"])
