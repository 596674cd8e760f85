"""Host tape (gmr/tape.py) on CPU: argument conversion, per-batch pointer re-basing and the recorder hook of
_lib.call, driven through ctypes callbacks that stand in for C-ABI entry points (no GPU needed)."""
import ctypes

import pytest
import torch

from gmr import _lib
from gmr.tape import Tape, TapeUnsupported

PROTO = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p)


def _fn(log):
    def body(n, p, x, arr):
        log.append((n, p, round(x, 6), arr))
        return 0
    f = PROTO(body)
    f.argtypes = list(PROTO._argtypes_)
    return f


def test_replay_rebases_input_pointers(monkeypatch):
    log = []
    fn = _fn(log)
    monkeypatch.setitem(_lib._fns, "fake_entry", (fn, 4))
    monkeypatch.setattr(_lib, "_lib", object())  # call() needs no library for a cached entry
    a = torch.arange(8, dtype=torch.int32)
    b = torch.arange(8, dtype=torch.int32)
    fixed = torch.zeros(4)
    tape = Tape([a, b])
    with tape.recording():
        _lib.call("fake_entry", 3, ctypes.c_void_p(a.data_ptr() + 8), 0.5, ctypes.c_void_p(fixed.data_ptr()))
        _lib.call("fake_entry", 4, b.data_ptr(), 1.5, None)
    assert len(tape) == 2 and len(tape.patches) == 2 and _lib.recorder is None
    a2, b2 = a.clone(), b.clone()
    log.clear()
    tape.replay([a2, b2])
    assert log == [(3, a2.data_ptr() + 8, 0.5, fixed.data_ptr()), (4, b2.data_ptr(), 1.5, None)]
    with pytest.raises(ValueError):
        tape.replay([a2[:4], b2])


def test_input_pointer_inside_host_array_is_refused(monkeypatch):
    fn = _fn([])
    monkeypatch.setitem(_lib._fns, "fake_entry", (fn, 4))
    monkeypatch.setattr(_lib, "_lib", object())
    a = torch.arange(8, dtype=torch.int32)
    tape = Tape([a])
    arr = (ctypes.c_void_p * 2)(a.data_ptr(), 0)
    with pytest.raises(TapeUnsupported):
        with tape.recording():
            _lib.call("fake_entry", 1, None, 0.0, arr)
    assert _lib.recorder is None
