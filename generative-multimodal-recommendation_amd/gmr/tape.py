"""Host-issue tape: record the C-ABI calls of one step, replay them without the Python layer.

The DiffMM rec step (calculate_loss + backward, models/diffmm.py:203-258, issued once per BPR batch by
common/trainer.py:144-208) is ~48 kernel launches and ~17 stream forks issued from Python; the per-call
Python work (argument marshalling, plan lookups, views) costs about as much host time as the whole step costs
on the GPU, so the GPU waits on the host between dependent launches (profiles/r05o_graph_step_probe.txt,
profiles/r05zw_rec_step_trace.txt).  A HIP graph removes the host cost but its replay lost the eager step's
three-stream overlap.  A tape keeps the eager step exactly - the same entry points with the same arguments on
the same streams, in the same order - and only drops the Python around them: while recording, every
`_lib.call` is executed and its arguments are converted once to their ctypes parameter objects; a replay calls
the functions with those objects.  Pointers into the step's per-batch inputs (the users / pos / neg rows and
the two scatter plans, which move through the epoch's device arrays batch by batch) are found while recording
and re-based on every replay; everything else a step touches (work buffers, slabs, graphs, workspaces, the
stream handles) is fixed for as long as the tape's key holds (the trainer re-records after a graph rebuild or
when the batch shape changes).
"""
import ctypes

from . import _lib


class TapeUnsupported(RuntimeError):
    """The recorded step passed an input pointer where the tape cannot re-base it (inside a host array)."""


def _value(a):
    if isinstance(a, ctypes.c_void_p):
        return a.value
    if isinstance(a, int) and not isinstance(a, bool):
        return a
    return None


def _param(t, a):
    """The argument as an instance of its declared ctypes type (ctypes takes those without conversion); host
    arrays, byref() objects and None pass as they are."""
    if a is None or isinstance(a, t):
        return a
    if t is ctypes.c_void_p:
        return ctypes.c_void_p(a) if isinstance(a, int) else a
    return t(a)


class Tape:
    """Record with `with tape.recording(): body()` (the body runs for real), then `tape.replay(inputs)` with the
    same number of input tensors of the same sizes (their data pointers may differ)."""

    def __init__(self, inputs):
        self.calls = []     # (name, fn, [ctypes parameter objects], keep-alive originals)
        self.patches = []   # (call index, argument index, input index, byte offset)
        self._ranges = [(t.data_ptr(), t.numel() * t.element_size()) for t in inputs]
        self._sizes = [r[1] for r in self._ranges]

    def _input_of(self, v):
        for k, (base, size) in enumerate(self._ranges):
            if base <= v < base + max(size, 1):
                return k, v - base
        return None

    def note(self, name, fn, args):
        params = []
        ci = len(self.calls)
        for ai, (t, a) in enumerate(zip(fn.argtypes, args)):
            v = _value(a) if t is ctypes.c_void_p else None
            hit = self._input_of(v) if v else None
            if hit is not None:
                self.patches.append((ci, ai, hit[0], hit[1]))
            elif isinstance(a, ctypes.Array) and issubclass(a._type_, (ctypes.c_void_p,)):
                if any(e and self._input_of(e) for e in a):
                    raise TapeUnsupported(f"{name}: a per-batch input pointer inside a host array")
            params.append(_param(t, a))
        self.calls.append((name, fn, params, args))

    class _Rec:
        def __init__(self, tape):
            self.tape = tape

        def __enter__(self):
            if _lib.recorder is not None:
                raise RuntimeError("a tape is already recording")
            _lib.recorder = self.tape
            return self.tape

        def __exit__(self, *a):
            _lib.recorder = None
            return False

    def recording(self):
        return Tape._Rec(self)

    def replay(self, inputs):
        if [t.numel() * t.element_size() for t in inputs] != self._sizes:
            raise ValueError("tape replay: input sizes differ from the recorded step's")
        calls = self.calls
        if self.patches:
            bases = [t.data_ptr() for t in inputs]
            for ci, ai, k, off in self.patches:
                calls[ci][2][ai] = ctypes.c_void_p(bases[k] + off)
        for name, fn, params, _ in calls:
            rc = fn(*params)
            if rc != 0:
                _lib.check(rc, name)

    def __len__(self):
        return len(self.calls)
