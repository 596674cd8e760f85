"""Thin tensor-level wrappers over the C-ABI (include/gmr.h).

Every function takes torch tensors that already live on the GPU, passes raw device
pointers + the current torch HIP stream to libgmr_hip.so, and raises on error.  Torch is
used here only for memory and streams.
"""
import ctypes
import os

import torch

from . import _lib

EPI_NONE, EPI_BIAS, EPI_BIAS_TANH, EPI_LEAKY, EPI_POSTERIOR, EPI_DTANH, EPI_ROWSCALE_AUX, EPI_BIAS_RELU, EPI_DRELU = range(9)
EPI_LEAKY_NORM = 9  # leaky + row normalisation in the split-K reduce: aux = normalised rows, rv1 = norms (written)
EPI_SCALE_BIAS = 10  # slope * (acc + bias): the posterior with c2 = 0, no aux read

_ws = {}

# ---------------------------------------------------------------- live per-kernel timing (bench.py)
_probe = None
_probe_every = 1
_probe_count = 0


def probe_begin(tags, every=1):
    """Record HIP events around the launches whose tag is in `tags` (on the launching stream); with
    every > 1 a hashed 1-in-`every` sample keeps the probe's own cost out of the timed region."""
    global _probe, _probe_every, _probe_count
    _probe = {t: [] for t in tags}
    _probe_every, _probe_count = max(1, int(every)), 0


def probe_end():
    global _probe
    p, _probe = _probe, None
    return p


class _Probe:
    def __init__(self, tag, meta):
        global _probe_count
        self.rec = _probe.get(tag) if _probe is not None else None
        if self.rec is not None and torch.cuda.is_current_stream_capturing():
            self.rec = None  # launches captured into a HIP graph are not individually timed
        if self.rec is not None and _probe_every > 1:
            _probe_count += 1  # hashed 1-in-`every` selection: no aliasing with the launch pattern
            if (((_probe_count * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF) >> 40) % _probe_every:
                self.rec = None
        self.meta = meta

    def __enter__(self):
        if self.rec is not None:
            self.s = torch.cuda.Event(enable_timing=True)
            self.e = torch.cuda.Event(enable_timing=True)
            self.s.record()

    def __exit__(self, *a):
        if self.rec is not None:
            self.e.record()
            self.rec.append((self.s, self.e, self.meta))


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def stream():
    """The current torch HIP stream as a ctypes pointer.  Called for every launch (~56 per DiffMM
    rec step, whose host issue time is close to its GPU time), so it takes torch's raw C accessor
    rather than building a torch.cuda.Stream object (a third of the step's host time)."""
    if _raw_stream is not None and _cur_device is not None:
        return ctypes.c_void_p(_raw_stream(_cur_device()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


_get_stream = getattr(torch._C, "_cuda_getCurrentStream", None)
_set_stream = getattr(torch._C, "_cuda_setStream", None)


class Streams:
    """Fork/join helper over a few side streams: work issued inside `with st.on(i):` runs on side
    stream i after everything already issued on the current stream; st.join(i) makes the current
    stream wait for it.  The fork/join is one C-ABI call on raw stream handles (gmr_stream_fork)
    and the current stream is switched with torch's raw setter: the DiffMM rec step forks ~17
    times per step and is host-issue-bound, so torch Stream/Event objects are kept off this path
    (torch.cuda.stream() is the fallback when this torch build lacks the raw setters).
    SERIAL (GMR_SERIAL=1, profiling): side work runs on the current stream, so every kernel's
    duration is its own and not stretched by a concurrent one."""

    SERIAL = False

    PRIORITY = int(os.environ.get("GMR_SIDE_PRIO", "0"))  # torch stream priority of the side streams (-1: high)

    # stream-ordering probe (tests/test_stream_order_gpu.py): None, or (where, i, us) - at every fork onto side
    # stream i a ~us-microsecond sleep kernel is queued on that side stream ("side": its work starts late, so a
    # main-stream read of it without a join sees stale data) or on the forking stream ("main": the side work runs
    # ahead of everything the forking stream issues next).  A correctly joined step gives the same bits either way.
    PERTURB = None

    def __init__(self, n):
        self.side = [torch.cuda.Stream(priority=Streams.PRIORITY) for _ in range(n)]
        self._raw = [ctypes.c_void_p(s.cuda_stream) for s in self.side]
        self._ids = [(s.stream_id, s.device_index, s.device_type) for s in self.side]
        self._dev = torch.cuda.current_device()
        lib = _lib.load()
        self._ev = []
        for _ in range(2 * n):
            e = ctypes.c_void_p()
            _lib.check(lib.gmr_event_create(ctypes.cast(ctypes.pointer(e), ctypes.c_void_p)), "gmr_event_create")
            self._ev.append(e)

    def on(self, i):
        return _OnSide(self, i)

    def join(self, *idx):
        if Streams.SERIAL:
            return
        cur = stream()
        for i in idx:
            _lib.call("gmr_stream_fork", self._raw[i], cur, self._ev[2 * i + 1])

    def close(self):
        """Release the fork/join events (after the device has drained the streams' work)."""
        ev, self._ev = getattr(self, "_ev", []), []
        if ev and _lib is not None:
            torch.cuda.synchronize(self._dev)
            lib = _lib.load()
            for e in ev:
                lib.gmr_event_destroy(e)

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter shutdown: the runtime may be gone)
            pass


Streams.SERIAL = os.environ.get("GMR_SERIAL", "0") == "1"


class _OnSide:
    __slots__ = ("st", "i", "prev", "ctx")

    def __init__(self, st, i):
        self.st, self.i = st, i

    def __enter__(self):
        st, i = self.st, self.i
        if Streams.SERIAL:
            self.prev = None
            return None
        if _cur_device is not None and _cur_device() != st._dev:
            raise RuntimeError(f"Streams built on device {st._dev} used while device {_cur_device()} is current")
        _lib.call("gmr_stream_fork", stream(), st._raw[i], st._ev[2 * i])
        pb = Streams.PERTURB
        if pb is not None and pb[1] == i:
            _lib.call("gmr_delay", int(pb[2]), st._raw[i] if pb[0] == "side" else stream())
        if _get_stream is None or _set_stream is None:
            self.prev = None
            self.ctx = torch.cuda.stream(st.side[i])
            self.ctx.__enter__()
            return st.side[i]
        self.ctx = None
        self.prev = _get_stream(st._dev)
        sid, dev, dt = st._ids[i]
        _set_stream(stream_id=sid, device_index=dev, device_type=dt)
        return st.side[i]

    def __exit__(self, *a):
        if self.prev is None:
            if not Streams.SERIAL and self.ctx is not None:
                self.ctx.__exit__(*a)
            return False
        sid, dev, dt = self.prev
        _set_stream(stream_id=sid, device_index=dev, device_type=dt)
        return False


def ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("gmr kernels take device tensors only (no CPU fallback)")
    return ctypes.c_void_p(t.data_ptr())


def _ld(t):
    if t.dim() == 1:
        return t.shape[0]
    if t.stride(-1) != 1:
        raise ValueError("inner dimension must be contiguous")
    return t.stride(0)


def workspace(nfloats, device, tag="gemm"):
    """Cached scratch per (tag, device, stream): kernels running concurrently on different
    streams never share one."""
    key = (tag, device, _raw_stream(_cur_device()) if _raw_stream is not None and _cur_device is not None
           else torch.cuda.current_stream().cuda_stream)
    w = _ws.get(key)
    if w is None or w.numel() < nfloats:
        # zeroed: a GEMM split-K workspace starts with tile counters that must be zero
        # (GMR_GEMM_COUNTER_WORDS, include/gmr.h); every call leaves them zero
        w = torch.zeros(max(nfloats, 1 << 20), dtype=torch.float32, device=device)
        _ws[key] = w
    return w


def zero_(t):
    if not t.is_contiguous():
        raise ValueError("zero_ needs a contiguous tensor")
    _lib.call("gmr_zero", ptr(t), t.numel() * t.element_size(), stream())
    return t


# ----------------------------------------------------------------------------- GEMM
_gemm_kinds = {}
# tile flags OR-ed into every gemm() call (tests: GMR_GEMM_F32 = 1 << 27 runs a whole path on the fp32-input MFMA)
GEMM_TILE_FLAGS = 0


def _gemm_tag(A, B, trans_a, trans_b, M, N, K, tile, split_k):
    """Probe class of a GEMM launch: "gemm_x6" when the plan takes the split-bf16 kernel
    (gmr_gemm_kernel_kind == 6), else "gemm" (fp32-input MFMA)."""
    aligned = int(A.data_ptr() % 16 == 0 and B.data_ptr() % 16 == 0 and _ld(A) % 4 == 0 and _ld(B) % 4 == 0)
    key = (int(trans_a), int(trans_b), M, N, K, tile, split_k, aligned)
    kind = _gemm_kinds.get(key)
    if kind is None:
        kind = _gemm_kinds[key] = int(_lib.load().gmr_gemm_kernel_kind(*key))
    return "gemm_x6" if kind == 6 else "gemm"


# gemm() call plans by (shapes, leading dimensions, dtypes, flags): the shape checks and the workspace size
# are worked out once per call site.  GenRecV1 issues ~2,400 GEMMs per epoch and is host-issue-bound, so the
# per-call Python work (~13 us before this cache) is kept to the pointer reads and the one ctypes call.
_gemm_plans = {}


def _gemm_plan(A, B, C, trans_a, trans_b, tile, split_k):
    M, N = C.shape
    K = A.shape[0] if trans_a else A.shape[1]
    if (A.shape[1] if trans_a else A.shape[0]) != M:
        raise ValueError(f"A shape {tuple(A.shape)} does not give M={M}")
    if (B.shape[1] if trans_b else B.shape[0]) != K or (B.shape[0] if trans_b else B.shape[1]) != N:
        raise ValueError(f"B shape {tuple(B.shape)} does not match K={K}, N={N}")
    for t in (A, B, C):
        if t.dtype != torch.float32:
            raise TypeError("gemm is fp32")
        if not t.is_cuda:
            raise ValueError("gmr kernels take device tensors only (no CPU fallback)")
    tile |= GEMM_TILE_FLAGS
    need = int(_lib.load().gmr_gemm_workspace_floats(int(trans_a), int(trans_b), M, N, K, tile, split_k))
    return M, N, K, tile, need, _ld(A), _ld(B), _ld(C)


def gemm(A, B, C, trans_a=False, trans_b=False, alpha=1.0, beta=0.0, epi=EPI_NONE, bias=None, bias_row=None,
         ld_bias=0, aux=None, rv1=None, rv2=None, slope=0.0, tile=0, split_k=0):
    """C = epi(alpha * op(A) @ op(B) ...), see include/gmr.h gmr_gemm_f32."""
    key = (A.shape, A.stride(), B.shape, B.stride(), C.shape, C.stride(), A.dtype, B.dtype, C.dtype, A.device,
           trans_a, trans_b, tile, split_k, GEMM_TILE_FLAGS)
    pl = _gemm_plans.get(key)
    if pl is None:
        pl = _gemm_plans[key] = _gemm_plan(A, B, C, trans_a, trans_b, tile, split_k)
    M, N, K, tile, need, lda, ldb, ldc = pl
    ws = workspace(need, C.device) if need > 0 else None  # split-K partials only when this call splits
    args = (int(trans_a), int(trans_b), M, N, K, float(alpha), A.data_ptr(), lda, B.data_ptr(), ldb, float(beta),
            C.data_ptr(), ldc, epi, ptr(bias), ptr(bias_row), ld_bias, ptr(aux), _ld(aux) if aux is not None else 0,
            ptr(rv1), ptr(rv2), float(slope), tile, split_k, ws.data_ptr() if ws is not None else None,
            ws.numel() if ws is not None else 0, stream())
    if _probe is None:
        _lib.call("gmr_gemm_f32", *args)
    else:
        with _Probe(_gemm_tag(A, B, trans_a, trans_b, M, N, K, tile, split_k), (M, N, K, int(trans_a), int(trans_b), epi)):
            _lib.call("gmr_gemm_f32", *args)
    return C


class Planes:
    """A plane set (include/gmr.h gmr_split3_planes): an fp32 matrix of `rows` x `cols` held as three bf16
    planes [3][rows][ld] (x = hi + mid + lo exactly), ld = cols rounded up to 32, pad columns zero.  The
    item-table form of the split-bf16 fused eval (gmr_score_topk_x6)."""

    def __init__(self, rows, cols, device):
        self.rows, self.cols = int(rows), int(cols)
        self.ld = (self.cols + 31) // 32 * 32
        self.t = torch.zeros((3, self.rows, self.ld), dtype=torch.int16, device=device)  # pad columns stay 0
        self.ps = self.rows * self.ld

    def ptr(self):
        return ctypes.c_void_p(self.t.data_ptr())

    def load(self, src):
        """Planes of the fp32 matrix src (its rows -> the first src.shape[0] rows; cols columns, unit column
        stride)."""
        if src.shape[0] > self.rows or src.shape[1] != self.cols or src.dtype != torch.float32 or src.stride(1) != 1:
            raise ValueError("split3: src must be an fp32 (<= rows) x cols matrix with unit column stride")
        _lib.call("gmr_split3_planes", src.shape[0], self.cols, ptr(src), src.stride(0), self.ptr(), self.ld, self.ps,
                  stream())
        return self

    def to_float(self):
        """hi + mid + lo as an fp32 rows x cols tensor (tests)."""
        p = self.t[:, :, :self.cols].to(torch.int32) << 16
        f = p.view(torch.float32) if p.is_contiguous() else p.contiguous().view(torch.float32)
        return (f[0] + f[1]) + f[2]


# ----------------------------------------------------------------------------- SpMM
# SpMM plan: 64..448 = segment plan (wave per <= seg_nnz segment), 512..8192 = blocked plan,
# SPMM_LANE_PLAN | L = lane plan (XCD column slices, lane group per row)
# (see include/gmr.h).  The lane plan with L = 32 measured fastest on the DiffMM graphs
# (scripts/spmm_bench.py, profiles/r01_spmm_lane_bench.txt).
# GMR_SPMM_CLASSES=1: lane plans of bipartite graphs schedule the item rows before the user rows
# (gmr_spmm_plan_build_split).  Off by default: −2…3 % per product alone, but the BPR phase ran
# 1.4 ms slower with it (profiles/r02v_spmm_classes_ab.txt)
SPMM_CLASSES = os.environ.get("GMR_SPMM_CLASSES", "0") == "1"
SPMM_NO_SPLIT_ROWS = 1
SPMM_HUB_FIXUP = 2  # lane plan with split hub rows: the launch adds their segment partials (include/gmr.h)
SPMM_LANE_PLAN = 1 << 16  # | L (32, 64, 128): lane plan (include/gmr.h)
SPMM_PACKED = 1 << 17  # | SPMM_LANE_PLAN | 32: packed lane plan (col/val of short rows in plan order)
SPMM_SEG_NNZ = SPMM_LANE_PLAN | 32
# the fixed norm_adj (built once, 7 of the 11 products of a DiffMM step) runs the plain lane plan:
# since hub rows are cut into 1,024-entry segments the packed plan (bit-identical sums, 4-7 %
# faster in round 1, profiles/r01g_spmm_packed_bench.txt) is 5-8 % slower at d = 64 / 128 and
# 3 % faster only at d = 256 (profiles/r02i_spmm_nt.txt); it stays a tested alternative
SPMM_NORM_ADJ = SPMM_LANE_PLAN | 32
SPMM_CHUNK = 1 << 18  # chunk plan: whole-row tasks of <= 128 entries, one gather round per wave (include/gmr.h)
# side-split plans (csrc/spmm_side.hip) for square matrices with a side split (the bipartite graph-conv
# adjacencies): each XCD serves one (side, 32-column slice), lane groups stream <= SPMM_SIDE_T-entry
# tasks, hub rows combine in-launch.  GMR_SPMM_SIDE=0 keeps every product on the lane plans (A/B)
SPMM_SIDE = os.environ.get("GMR_SPMM_SIDE", "1") == "1"
# short-row task entries: 16 for every graph (round-3 sweeps with 8 / 12 / 16 / 32 / 64-entry tasks,
# profiles/r03o_sweep.txt, r03p_sweep.txt: 16 is best or tied at d <= 128); GMR_SPMM_SIDE_T overrides
SPMM_SIDE_T = int(os.environ.get("GMR_SPMM_SIDE_T", "0"))
# degree-class plan for the short rows (GMR_SIDE_CLASSES, include/gmr.h); GMR_SPMM_DC=0: the task plan
SPMM_SIDE_CLASSES = 1 << 24
SPMM_DC = os.environ.get("GMR_SPMM_DC", "1") == "1"
SPMM_SIDE_TW = int(os.environ.get("GMR_SPMM_SIDE_TW", "32"))


class CSR:
    """Device CSR (int32 rowptr/col, fp32 val) of an n x n matrix with its SpMM work plan."""

    def __init__(self, rowptr, col, val, n_cols=None, seg_nnz=None, symmetric=True, class_split=0, side=False):
        seg_nnz = SPMM_SEG_NNZ if seg_nnz is None else seg_nnz
        self.rowptr, self.col, self.val = rowptr, col, val
        self.n_rows = rowptr.numel() - 1
        self.n_cols = self.n_rows if n_cols is None else n_cols
        self.nnz = col.numel()
        self.seg_nnz = seg_nnz
        self.symmetric = symmetric
        dev = rowptr.device
        words = _lib.load().gmr_spmm_plan_words(self.n_rows, self.nnz, seg_nnz)
        self.plan = torch.empty(words, dtype=torch.int32, device=dev)
        prow = _lib.load().gmr_spmm_partial_rows(self.n_rows, self.nnz, seg_nnz)
        self.partial = torch.zeros((prow, 256), dtype=torch.float32, device=dev)
        cs = class_split if (SPMM_CLASSES and seg_nnz & SPMM_LANE_PLAN and not seg_nnz & SPMM_PACKED) else 0
        self.class_split = class_split
        self.side = None
        _lib.call("gmr_spmm_plan_build_split", ptr(rowptr), self.n_rows, self.nnz, seg_nnz, cs, ptr(self.plan),
                  stream())
        if seg_nnz & SPMM_PACKED or seg_nnz == SPMM_CHUNK:  # col/val are final here (built before wrapping)
            _lib.call("gmr_spmm_plan_pack", ptr(rowptr), ptr(col), ptr(val), self.n_rows, self.nnz, seg_nnz,
                      ptr(self.plan), stream())
        hdr = (ctypes.c_int32 * 4)()
        _lib.call("gmr_spmm_plan_info", ptr(self.plan), hdr, stream())  # one sync per graph build
        self.plan_header = tuple(hdr)
        # segment plan without split rows: the combine pass is skipped; lane plan with split hubs: fixup pass
        self.flags = SPMM_NO_SPLIT_ROWS if (seg_nnz < 512 and hdr[1] == 0) else 0
        if seg_nnz & SPMM_LANE_PLAN and hdr[2] >> 1:
            self.flags |= SPMM_HUB_FIXUP
        if side and SPMM_SIDE and class_split > 0 and self.n_cols == self.n_rows and self.nnz > 0:
            self.build_side_plan(class_split)

    def build_side_plan(self, split, T=None, classes=None):
        """Side-split plan (gmr_spmm_side_*): built on the host from a host copy of rowptr (one
        device sync per graph build), entries packed on the device; self.partial becomes the plan's
        scratch (zeroed: its hub counters re-arm themselves after every launch)."""
        import numpy as np
        lib = _lib.load()
        if T is None:
            T = SPMM_SIDE_T or 16  # 16-entry tasks: norm_adj d = 64 / 128 -10 % vs 32 (profiles/r03o_sweep.txt)
        T = int(T)
        if not (T >> 16) & 0xFF:
            T |= SPMM_SIDE_TW << 16
        # the degree-class plan for the graph-conv adjacency (norm_adj, d = 128: 17.5 -> 15.5 us, d = 64 11.3 ->
        # 11.1, profiles/r04i_spmm_classes_probe.txt); the rebuilt UI graphs (about two entries per row) keep
        # the task plan (+2..5 % with classes there)
        short = self.nnz < 4 * self.n_rows
        if (SPMM_DC and not short if classes is None else classes) and T & 0xFFFF == 16:
            T |= SPMM_SIDE_CLASSES
        rp = np.ascontiguousarray(self.rowptr.cpu().numpy().astype(np.int32))
        rpp = rp.ctypes.data_as(ctypes.c_void_p)
        words = int(lib.gmr_spmm_side_plan_words(rpp, self.n_rows, int(split), int(T)))
        if words <= 0:
            raise RuntimeError("gmr_spmm_side_plan_words failed")
        host = np.zeros(words, np.int32)
        _lib.call("gmr_spmm_side_plan_build", rpp, self.n_rows, int(split), int(T), host.ctypes.data_as(ctypes.c_void_p),
                  words)
        dev = self.rowptr.device
        plan = torch.from_numpy(host).to(dev)
        _lib.call("gmr_spmm_side_pack", ptr(self.rowptr), ptr(self.col), ptr(self.val), self.n_rows, self.nnz,
                  int(host[14]), ptr(plan), stream())
        _lib.call("gmr_spmm_side_pack_classes", ptr(self.rowptr), ptr(self.col), ptr(self.val),
                  host.ctypes.data_as(ctypes.c_void_p), ptr(plan), stream())
        self.side_classes = bool(host[20])
        nsc = int(lib.gmr_spmm_side_scratch_floats(host.ctypes.data_as(ctypes.c_void_p)))
        self.side = (plan, int(split))
        # workgroups per XCD by product width (profiles/r03b_sweep.txt): the short-task UI graphs and
        # the 64-column products fill the XCDs with 128, the wider norm_adj products with 256
        short = self.nnz < 4 * self.n_rows
        self.side_wpx = {1: 128, 2: 128, 4: 128 if short else 256}
        self.side_hdr = tuple(int(x) for x in host[:27])  # csrc/spmm_side.hip H_MAGIC .. H_NSE
        self.partial = torch.zeros(max(nsc, self.partial.numel()), dtype=torch.float32, device=dev)

    def spmm(self, out, blocks, split=None, alpha=1.0, beta=0.0, partial=None):
        """out = alpha * A @ X + beta * out; X = column blocks [(lo, hi), ...] of 64 columns each.

        Source row s of a block reads lo[s] if s < split else hi[s - split] (hi may be None
        when split is None, i.e. lo covers all rows).  `partial` overrides the hub-row scratch
        (two products of one matrix running concurrently on different streams)."""
        nb = len(blocks)
        if nb not in (1, 2, 4):
            raise ValueError("1, 2 or 4 blocks of 64 columns")
        if out.shape[0] != self.n_rows or out.shape[1] != 64 * nb:
            raise ValueError(f"out shape {tuple(out.shape)} != ({self.n_rows}, {64 * nb})")
        PArr = ctypes.c_void_p * 4
        LArr = ctypes.c_int64 * 4
        lo = PArr(*[b[0].data_ptr() for b in blocks] + [0] * (4 - nb))
        ldl = LArr(*[_ld(b[0]) for b in blocks] + [0] * (4 - nb))
        if split is None:
            split = self.n_cols
            hi, ldh = lo, ldl
        else:
            hi = PArr(*[b[1].data_ptr() for b in blocks] + [0] * (4 - nb))
            ldh = LArr(*[_ld(b[1]) for b in blocks] + [0] * (4 - nb))
        for b in blocks:
            if b[0].shape[1] != 64 or (split != self.n_cols and b[1].shape[1] != 64):
                raise ValueError("each block is 64 columns wide")
        if self.side is not None:
            ys = PArr(*[out[:, 64 * b:64 * (b + 1)].data_ptr() for b in range(nb)] + [0] * (4 - nb))
            ldy = LArr(*[_ld(out)] * nb + [0] * (4 - nb))
            self._side_call(nb, lo, ldl, hi, ldh, split, alpha, beta, ys, ldy, partial)
            return out
        with _Probe("spmm", (self.nnz, self.n_rows, self.n_cols, nb, beta != 0.0)):
            _lib.call("gmr_spmm_csr_f32", ptr(self.rowptr), ptr(self.col), ptr(self.val), self.n_rows, self.nnz,
                      ptr(self.plan), self.seg_nnz, ptr(self.partial if partial is None else partial), nb, lo, ldl,
                      hi, ldh, split, float(alpha),
                      float(beta), ptr(out), _ld(out), self.flags, stream())
        return out


def _side_call(self, nb, lo, ldl, hi, ldh, split, alpha, beta, ys, ldy, partial):
    """gmr_spmm_side_f32 with host arrays of block pointers / strides (CSR.spmm, spmm_multi, spmm_jobs)."""
    with _Probe("spmm", (self.nnz, self.n_rows, self.n_cols, nb, beta != 0.0)):
        _lib.call("gmr_spmm_side_f32", ptr(self.side[0]), nb, lo, ldl, hi, ldh, int(split), float(alpha), float(beta),
                  ys, ldy, ptr(self.partial if partial is None else partial), self.side_wpx[nb], stream())


CSR._side_call = _side_call


def spmm_side2(a, outs, blocks, z, split=None, alpha=1.0, beta=1.0, only_side=-1, partial=None):
    """outs[b] = alpha * A @ X_b + beta * z[b] on a side-split plan (gmr_spmm_side2_f32): X_b = blocks[b] (a (lo,)
    or (lo, hi) split source as in CSR.spmm), z[b] an n_rows x 64 view (the beta term's source, may differ from
    outs[b]); only_side 0 / 1 computes only the rows below / from the split (the others are left untouched)."""
    if a.side is None:
        raise ValueError("spmm_side2 needs a side-split plan")
    nb = len(blocks)
    if nb not in (1, 2, 4) or len(outs) != nb or len(z) != nb:
        raise ValueError("1, 2 or 4 blocks, one output and one z view each")
    for o in list(outs) + list(z):
        if o.shape != (a.n_rows, 64):
            raise ValueError(f"output / z block shape {tuple(o.shape)} != ({a.n_rows}, 64)")
    PArr, LArr = ctypes.c_void_p * 4, ctypes.c_int64 * 4
    lo = PArr(*[b[0].data_ptr() for b in blocks] + [0] * (4 - nb))
    ldl = LArr(*[_ld(b[0]) for b in blocks] + [0] * (4 - nb))
    if split is None:
        split, hi, ldh = a.n_cols, lo, ldl
    else:
        hi = PArr(*[b[1].data_ptr() for b in blocks] + [0] * (4 - nb))
        ldh = LArr(*[_ld(b[1]) for b in blocks] + [0] * (4 - nb))
    ys = PArr(*[o.data_ptr() for o in outs] + [0] * (4 - nb))
    ldy = LArr(*[_ld(o) for o in outs] + [0] * (4 - nb))
    zs = PArr(*[o.data_ptr() for o in z] + [0] * (4 - nb))
    ldz = LArr(*[_ld(o) for o in z] + [0] * (4 - nb))
    key = (a.nnz, a.n_rows, a.n_cols, nb, beta != 0.0)
    if only_side >= 0:  # one side of a bipartite product: its rows, half the entries, the other side's X rows
        sp = a.side[1]
        rows = sp if only_side == 0 else a.n_rows - sp
        key = (a.nnz // 2, rows, a.n_rows - rows, nb, beta != 0.0)
    with _Probe("spmm", key):
        _lib.call("gmr_spmm_side2_f32", ptr(a.side[0]), nb, lo, ldl, hi, ldh, int(split), float(alpha), float(beta), zs,
                  ldz, ys, ldy, int(only_side), ptr(a.partial if partial is None else partial), a.side_wpx[nb],
                  stream())
    return outs


def score_f16(a, b, out):
    """out = fp16(a) @ fp16(b)^T with fp32 accumulation (gmr_score_f16; a: E x 64, b: I x 64)."""
    E, d = a.shape
    n = b.shape[0]
    if d != 64 or b.shape[1] != 64 or out.shape != (E, n):
        raise ValueError("score_f16: a (E, 64), b (I, 64), out (E, I)")
    _lib.call("gmr_score_f16", E, n, d, ptr(a), _ld(a), ptr(b), _ld(b), ptr(out), _ld(out), stream())
    return out


def spmm_multi(a, outs, blocks, split=None, alpha=1.0, beta=0.0, partial=None):
    """One lane-plan launch for independent products of `a`: block b (64 columns, a (lo, hi) split
    source as in CSR.spmm) lands in outs[b] (an n_rows x 64 view).  gmr_spmm_multi_f32."""
    nb = len(blocks)
    if nb not in (1, 2, 4) or len(outs) != nb:
        raise ValueError("1, 2 or 4 blocks, one output each")
    for o in outs:
        if o.shape != (a.n_rows, 64):
            raise ValueError(f"output block shape {tuple(o.shape)} != ({a.n_rows}, 64)")
    PArr, LArr = ctypes.c_void_p * 4, ctypes.c_int64 * 4
    lo = PArr(*[b[0].data_ptr() for b in blocks] + [0] * (4 - nb))
    ldl = LArr(*[_ld(b[0]) for b in blocks] + [0] * (4 - nb))
    if split is None:
        split, hi, ldh = a.n_cols, lo, ldl
    else:
        hi = PArr(*[b[1].data_ptr() for b in blocks] + [0] * (4 - nb))
        ldh = LArr(*[_ld(b[1]) for b in blocks] + [0] * (4 - nb))
    ys = PArr(*[o.data_ptr() for o in outs] + [0] * (4 - nb))
    ldy = LArr(*[_ld(o) for o in outs] + [0] * (4 - nb))
    if a.side is not None:
        a._side_call(nb, lo, ldl, hi, ldh, split, alpha, beta, ys, ldy, partial)
        return outs
    with _Probe("spmm", (a.nnz, a.n_rows, a.n_cols, nb, beta != 0.0)):
        _lib.call("gmr_spmm_multi_f32", ptr(a.col), ptr(a.val), a.n_rows, a.nnz, ptr(a.plan), a.seg_nnz, nb, lo, ldl,
                  hi, ldh, split, float(alpha), float(beta), ys, ldy, ptr(a.partial if partial is None else partial),
                  a.flags, stream())
    return outs


# side-plan products of a jobs call in one launch (gmr_spmm_side_jobs_f32; GMR_SPMM_SIDE_JOBS=0: one per job)
SIDE_JOBS = os.environ.get("GMR_SPMM_SIDE_JOBS", "1") != "0"


def _side_jobs(jobs, alpha, beta):
    """Side-plan products [(a, outs, blocks, split, partial), ...] of one width in one gmr_spmm_side_jobs_f32."""
    n, nb = len(jobs), len(jobs[0][2])
    PA, LA = ctypes.c_void_p * (4 * n), ctypes.c_int64 * (4 * n)
    plans, scr = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)()
    lo, hi, ys = PA(), PA(), PA()
    ldl, ldh, ldy = LA(), LA(), LA()
    splits = (ctypes.c_int64 * n)()
    key = []
    for q, (a, outs, blocks, split, partial) in enumerate(jobs):
        if isinstance(outs, torch.Tensor):
            outs = [outs[:, 64 * b:64 * (b + 1)] for b in range(nb)]
        if len(outs) != nb or any(o.shape != (a.n_rows, 64) for o in outs):
            raise ValueError("one n_rows x 64 output per block")
        plans[q] = a.side[0].data_ptr()
        scr[q] = (a.partial if partial is None else partial).data_ptr()
        splits[q] = a.n_cols if split is None else int(split)
        for b in range(nb):
            lo[4 * q + b], ldl[4 * q + b] = blocks[b][0].data_ptr(), _ld(blocks[b][0])
            src_hi = blocks[b][1] if split is not None else blocks[b][0]
            hi[4 * q + b], ldh[4 * q + b] = src_hi.data_ptr(), _ld(src_hi)
            ys[4 * q + b], ldy[4 * q + b] = outs[b].data_ptr(), _ld(outs[b])
        key.append((a.nnz, a.n_rows, a.n_cols, nb, beta != 0.0))
    with _Probe("spmm", ("side_jobs",) + tuple(key)):
        _lib.call("gmr_spmm_side_jobs_f32", n, plans, scr, nb, lo, ldl, hi, ldh, splits, float(alpha), float(beta), ys,
                  ldy, jobs[0][0].side_wpx[nb], stream())


def spmm_jobs(jobs, alpha=1.0, beta=0.0):
    """One launch for up to 4 independent lane-plan products (gmr_spmm_jobs_f32).

    jobs: [(a, outs, blocks, split, partial), ...] with a CSR, outs a list of n_rows x 64 output
    views (one per block) or one n_rows x 64*nb tensor, blocks / split as in CSR.spmm, and partial
    the hub-row scratch (None: a.partial).  Each job's sums equal its CSR.spmm call's."""
    n = len(jobs)
    if not 1 <= n <= 4:
        raise ValueError("1 to 4 jobs")
    if any(j[0].side is not None for j in jobs):
        # side-plan products of one width go out as one multi-job launch (gmr_spmm_side_jobs_f32; SIDE_JOBS=0:
        # one launch each, in job order); lane-plan products as a lane multi-job launch
        lane = [j for j in jobs if j[0].side is None]
        side = [j for j in jobs if j[0].side is not None]
        if SIDE_JOBS and len(side) > 1 and len({len(j[2]) for j in side}) == 1 and \
                len({j[0].side_wpx[len(j[2])] for j in side}) == 1:
            _side_jobs(side, alpha, beta)
        else:
            for a, outs, blocks, split, partial in side:
                if isinstance(outs, torch.Tensor):
                    outs = [outs[:, 64 * b:64 * (b + 1)] for b in range(len(blocks))]
                spmm_multi(a, outs, blocks, split=split, alpha=alpha, beta=beta, partial=partial)
        if lane:
            spmm_jobs(lane, alpha=alpha, beta=beta)
        return
    arr = (_lib.SpmmJob * n)()
    for q, (a, outs, blocks, split, partial) in enumerate(jobs):
        nb = len(blocks)
        if nb not in (1, 2, 4):
            raise ValueError("1, 2 or 4 blocks of 64 columns")
        if isinstance(outs, torch.Tensor):
            if outs.shape != (a.n_rows, 64 * nb):
                raise ValueError(f"out shape {tuple(outs.shape)} != ({a.n_rows}, {64 * nb})")
            outs = [outs[:, 64 * b:64 * (b + 1)] for b in range(nb)]
        if len(outs) != nb or any(o.shape != (a.n_rows, 64) for o in outs):
            raise ValueError("one n_rows x 64 output per block")
        for b in blocks:
            if b[0].shape[1] != 64 or (split is not None and b[1].shape[1] != 64):
                raise ValueError("each block is 64 columns wide")
        j = arr[q]
        j.col, j.val, j.plan = ptr(a.col), ptr(a.val), ptr(a.plan)
        j.partial = ptr(a.partial if partial is None else partial)
        j.n_rows, j.nnz, j.seg_nnz, j.n_blocks, j.flags = a.n_rows, a.nnz, a.seg_nnz, nb, a.flags
        for b in range(nb):
            j.x_lo[b], j.ld_lo[b] = blocks[b][0].data_ptr(), _ld(blocks[b][0])
            if split is not None:
                j.x_hi[b], j.ld_hi[b] = blocks[b][1].data_ptr(), _ld(blocks[b][1])
            j.y[b], j.ld_y[b] = outs[b].data_ptr(), _ld(outs[b])
        j.split = a.n_cols if split is None else split
        j.alpha, j.beta = float(alpha), float(beta)
    key = tuple((a.nnz, a.n_rows, a.n_cols, len(bl), beta != 0.0) for a, _, bl, _, _ in jobs)
    with _Probe("spmm", ("jobs",) + key):
        _lib.call("gmr_spmm_jobs_f32", n, ctypes.cast(arr, ctypes.c_void_p), stream())


def spmm_panel(a, out, x_panel, nb, alpha=1.0, beta=0.0, partial=None):
    """out = alpha * A @ X + beta * out with X given in column-panel layout (S, n, W), see
    include/gmr.h gmr_spmm_panel_f32 (lane plans only)."""
    W = 32 if nb == 4 else 16
    if x_panel.shape != (64 * nb // W, a.n_cols, W) or not x_panel.is_contiguous():
        raise ValueError(f"x_panel must be a contiguous ({64 * nb // W}, {a.n_cols}, {W}) panel stack")
    if out.shape[0] != a.n_rows or out.shape[1] != 64 * nb:
        raise ValueError("out shape")
    with _Probe("spmm", (a.nnz, a.n_rows, a.n_cols, nb, beta != 0.0)):
        _lib.call("gmr_spmm_panel_f32", ptr(a.col), ptr(a.val), a.n_rows, a.nnz, ptr(a.plan), a.seg_nnz, nb,
                  ptr(x_panel), a.n_cols, float(alpha), float(beta), ptr(out), _ld(out),
                  ptr(a.partial if partial is None else partial), a.flags, stream())
    return out


def bipartite_symnorm(n_users, n_items, user_ptr, user_items, self_loops, deg_eps, seg_nnz=None):
    """Build the normalised (U+I)^2 bipartite adjacency on the device (graph.hip); its lane plan
    lists the item rows before the user rows (row classes, gmr_spmm_plan_build_split)."""
    lib = _lib.load()
    dev = user_ptr.device
    n_ui = user_items.numel()
    nnz = lib.gmr_bipartite_nnz(n_users, n_items, n_ui, int(self_loops))
    N = n_users + n_items
    rowptr = torch.empty(N + 1, dtype=torch.int32, device=dev)
    col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    val = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
    ws = torch.empty(lib.gmr_bipartite_workspace_ints(n_users, n_items), dtype=torch.int32, device=dev)
    _lib.call("gmr_bipartite_symnorm_build", n_users, n_items, ptr(user_ptr), ptr(user_items), n_ui,
              int(self_loops), float(deg_eps), ptr(ws), ptr(rowptr), ptr(col), ptr(val), stream())
    return CSR(rowptr, col[:nnz], val[:nnz], seg_nnz=seg_nnz, class_split=n_users, side=True)


def topk_to_user_csr(topk, user_ptr, user_items):
    U, k = topk.shape
    _lib.call("gmr_topk_to_user_csr", U, k, ptr(topk), _ld(topk), ptr(user_ptr), ptr(user_items), stream())


# ----------------------------------------------------------------------------- rows / reductions
def normalize_rows(x, y, nrm=None):
    n, cols = x.shape
    _lib.call("gmr_normalize_rows_f32", n, cols, ptr(x), _ld(x), ptr(y), _ld(y), ptr(nrm), stream())
    return y


def normalize_rows_bwd(y, nrm, dy, dx, slope=1.0, accumulate=False):
    n, cols = y.shape
    _lib.call("gmr_normalize_rows_bwd_f32", n, cols, ptr(y), _ld(y), ptr(nrm), ptr(dy), _ld(dy), ptr(dx), _ld(dx),
              float(slope), int(accumulate), stream())
    return dx


def topk_rows(scores, k, out_idx, out_val=None):
    n, m = scores.shape
    _lib.call("gmr_topk_rows_f32", n, m, ptr(scores), _ld(scores), int(k), ptr(out_idx), _ld(out_idx), ptr(out_val),
              stream())
    return out_idx


# GMR_EVAL_X6=1: the fused eval scores d = 64 embeddings on the bf16 matrix cores from exact three-way splits
# (gmr_score_topk_x6; the item table split once per table version).  Opt-in: the kernel is bound by its
# selection bookkeeping, not the score products (694 us fp32 vs 712 us split per 19,445-user pass,
# profiles/r04l_topk.txt), so the default keeps the fp32 MFMA scores
EVAL_X6 = os.environ.get("GMR_EVAL_X6", "0") != "0"
_item_planes = {}


def _planes_of(itm):
    """Plane set of the item table, cached per (storage, version, shape): one split per eval pass."""
    key = (itm.data_ptr(), itm._version, tuple(itm.shape), _ld(itm), itm.device)
    hit = _item_planes.get("key")
    if hit is not None and hit[0] == key:
        return hit[1]
    pl = Planes(itm.shape[0], itm.shape[1], itm.device).load(itm)
    _item_planes["key"] = (key, pl)
    return pl


def score_topk(usr, itm, users, mask_ptr, mask_cols, k, out_idx, out_val=None, fill=-1e10):
    """Fused eval (gmr_score_topk_f32 / _x6): top-k of usr[users] . itm^T with each row's train positives
    (mask_cols[mask_ptr[r]:mask_ptr[r+1]], sorted) set to fill; no rows x items score buffer."""
    n = users.numel() if users is not None else out_idx.shape[0]
    if out_idx.shape[0] < n or mask_ptr.numel() < n + 1 or mask_ptr.dtype != torch.int64:
        raise ValueError("score_topk: out_idx / mask_ptr (int64, n + 1) too small for the rows")
    if n == 0:  # an empty rank shard: nothing to score (the C-ABI rejects n_rows < 1)
        return out_idx
    if EVAL_X6 and itm.shape[1] == 64 and usr.shape[1] == 64:
        pl = _planes_of(itm)
        _lib.call("gmr_score_topk_x6", n, ptr(users), ptr(usr), _ld(usr), itm.shape[0], pl.ptr(), pl.ld, pl.ps, 64,
                  ptr(mask_ptr), ptr(mask_cols), float(fill), int(k), ptr(out_idx), _ld(out_idx), ptr(out_val),
                  stream())
        return out_idx
    _lib.call("gmr_score_topk_f32", n, ptr(users), ptr(usr), _ld(usr), itm.shape[0], ptr(itm), _ld(itm), itm.shape[1],
              ptr(mask_ptr), ptr(mask_cols), float(fill), int(k), ptr(out_idx), _ld(out_idx), ptr(out_val), stream())
    return out_idx


def mask_scores(scores, rows, cols, fill=-1e10):
    _lib.call("gmr_mask_scores_f32", rows.numel(), ptr(rows), ptr(cols), ptr(scores), _ld(scores), float(fill),
              stream())


def contrast_workspace(B, n, device, tag):
    return workspace(int(_lib.load().gmr_contrast_workspace_floats(B, n)), device, tag=tag)


def contrast_fused(P, T, CLN, nodes, node_off, inv_temp, coef, loss, contrib, dT, ws):
    """K8 fused InfoNCE (include/gmr.h gmr_contrast_fused_f32): loss rows, dP rows into contrib and
    the dense table gradient dT, without the B x n logits.  P = None: the batch rows are read in place,
    P_i = CLN[node_off + nodes[i], :64] (the pipelined split-bf16 passes only)."""
    B, n = (P.shape[0] if P is not None else nodes.numel()), T.shape[0]
    with _Probe("infonce", (B, n)):
        _lib.call("gmr_contrast_fused_f32", B, n, ptr(P), _ld(P) if P is not None else _ld(CLN), ptr(T), _ld(T),
                  ptr(CLN), ptr(nodes), node_off,
                  float(inv_temp), float(coef), ptr(loss), ptr(contrib), _ld(contrib), ptr(dT), _ld(dT), ptr(ws),
                  ws.numel(), stream())


def colsum(x, out, group=None, n_groups=1, accumulate=False):
    rows, cols = x.shape
    if group is None and cols <= 2048 and rows >= 1024:  # few column blocks: split the rows too
        ws = workspace(32 * cols, x.device, tag="colsum")
        _lib.call("gmr_colsum_split_f32", rows, cols, ptr(x), _ld(x), ptr(out), int(accumulate), ptr(ws), ws.numel(),
                  stream())
        return out
    _lib.call("gmr_colsum_f32", rows, cols, ptr(x), _ld(x), ptr(group), n_groups, ptr(out), int(accumulate),
              stream())
    return out


def gather_rows(src, idx, out, off=0):
    B = idx.numel()
    _lib.call("gmr_gather_rows_f32", B, out.shape[1], ptr(src), _ld(src), ptr(idx), off, ptr(out), _ld(out),
              stream())
    return out


def adam(param, grad, m, v, lr, beta1, beta2, eps, weight_decay, step):
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    _lib.call("gmr_adam_f32", param.numel(), ptr(param), ptr(grad), ptr(m), ptr(v), float(beta1), float(beta2),
              float(eps), float(weight_decay), float(lr / bc1), float(bc2 ** 0.5), stream())


def eval_metrics(topk, pos_ptr, pos_items, ks, partials, out_sums):
    n, K = topk.shape
    ks_t = ks
    _lib.call("gmr_eval_metrics", n, ptr(topk), _ld(topk), K, ptr(pos_ptr), ptr(pos_items), ks_t.numel(), ptr(ks_t),
              ptr(partials), ptr(out_sums), stream())


# ----------------------------------------------------------------------------- GenRecV1 graphs
def user_item_csr(n_users, n_items, user_ptr, user_items):
    """R (U x I, binary) as a CSR over the train user CSR (models/genrecv1.py:128-131)."""
    val = torch.ones(max(user_items.numel(), 1), dtype=torch.float32, device=user_ptr.device)[:user_items.numel()]
    return CSR(user_ptr, user_items, val, n_cols=n_items, symmetric=False)


def csr_transpose(a):
    """A^T as a CSR (columns ascending per row), for the backward of non-symmetric SpMMs."""
    dev = a.rowptr.device
    nc = a.n_cols
    trp = torch.empty(nc + 1, dtype=torch.int32, device=dev)
    n = max(a.nnz, 1)
    tcol = torch.empty(n, dtype=torch.int32, device=dev)
    tval = torch.empty(n, dtype=torch.float32, device=dev)
    scol = torch.empty(n, dtype=torch.int32, device=dev)
    sval = torch.empty(n, dtype=torch.float32, device=dev)
    ws = torch.empty(2 * nc, dtype=torch.int32, device=dev)
    _lib.call("gmr_csr_transpose", a.n_rows, nc, a.nnz, ptr(a.rowptr), ptr(a.col), ptr(a.val), ptr(ws), ptr(trp),
              ptr(tcol), ptr(tval), ptr(scol), ptr(sval), stream())
    return CSR(trp, tcol[:a.nnz], tval[:a.nnz], n_cols=a.n_rows, symmetric=False,
               class_split=a.class_split if a.n_rows == a.n_cols else 0, side=a.side is not None)


def csr_drop_edges(a, keep_rate, seed=0, step=0, keep=None, transposed=False):
    """SpAdjDropEdge (models/genrecv1.py:443-457): each entry kept iff floor(u + keep_rate) >= 1,
    kept values / keep_rate.  keep: optional 0/1 bytes per entry (CSR order) replacing the draws.
    transposed (structurally symmetric a only): the transpose of the dropped matrix, from the same
    draws.  One host sync reads the kept count."""
    dev = a.rowptr.device
    orp = torch.empty(a.n_rows + 1, dtype=torch.int32, device=dev)
    ws = torch.empty(a.n_rows, dtype=torch.int32, device=dev)
    _lib.call("gmr_csr_drop_count", a.n_rows, ptr(a.rowptr), ptr(a.col), int(transposed), ptr(keep), float(keep_rate),
              int(seed), int(step), ptr(ws), ptr(orp), stream())
    nnz = int(orp[-1].item())
    ocol = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    oval = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
    _lib.call("gmr_csr_drop_write", a.n_rows, ptr(a.rowptr), ptr(a.col), ptr(a.val), int(transposed), ptr(keep),
              float(keep_rate), int(seed), int(step), ptr(orp), ptr(ocol), ptr(oval), stream())
    return CSR(orp, ocol[:nnz], oval[:nnz], n_cols=a.n_cols, symmetric=False, class_split=a.class_split,
               side=a.side is not None)


def knn_graph(feat, k):
    """_build_knn_adj (common/trainer.py:682-687 -> utils/utils.py:184-197): cosine similarity on the
    MFMA GEMM, per-row top-k, 'sym' normalisation.  Returns the I x I CSR."""
    n, d = feat.shape
    dev = feat.device
    fn = torch.empty((n, d), dtype=torch.float32, device=dev)
    normalize_rows(feat, fn)
    sim = torch.empty((n, (n + 3) // 4 * 4), dtype=torch.float32, device=dev)[:, :n]
    gemm(fn, fn, sim, trans_b=True)
    ti = torch.empty((n, k), dtype=torch.int32, device=dev)
    tv = torch.empty((n, k), dtype=torch.float32, device=dev)
    topk_rows(sim, k, ti, tv)
    del sim
    rp = torch.empty(n + 1, dtype=torch.int32, device=dev)
    col = torch.empty(n * k, dtype=torch.int32, device=dev)
    val = torch.empty(n * k, dtype=torch.float32, device=dev)
    dis = torch.empty(n, dtype=torch.float32, device=dev)
    _lib.call("gmr_knn_symnorm_csr", n, k, ptr(ti), k, ptr(tv), k, ptr(dis), ptr(rp), ptr(col), ptr(val), stream())
    return CSR(rp, col, val, n_cols=n, symmetric=False)
