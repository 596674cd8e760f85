"""Data parallelism across the GPUs of one node: one process per GPU, torch.distributed over RCCL
(backend "nccl" is RCCL on ROCm, riding xGMI).  The reference has no distributed code (SURVEY.md
F2); this module holds the sharding rules used by the trainers:

  * diffusion phase  — each batch of train_batch_size users of the epoch permutation is split
    over the ranks (contiguous slices); denoiser gradients are all-reduced (SUM of per-rank sums
    normalised by the batch's row count) before the identical Adam steps;
  * graph rebuild    — users are split in contiguous shards (GenRecV1: whole batch chunks dealt
    round-robin); each rank p_samples its users and the int32 top-k lists are exchanged; every
    rank builds the identical CSR;
  * BPR phase        — each train_batch_size batch of the epoch draw is split over the ranks;
    the rec gradients are all-reduced (the regulariser is counted once);
  * evaluation       — eval users are sharded; the top-K index rows are all-gathered.
The global batch is the reference's train_batch_size at every world size, so the number of
optimiser steps per epoch, and the trajectory up to fp32 reassociation of the sums, are the
single-process ones (the per-GPU batch shrinks as B / world: strong scaling).  DiffMM and DiffRec
key every device draw by (global step, global row), so their draws are also the single-process
ones at any world size.  GenRecV1 does the same: its diffusion draws (t, flips, dropout masks) are
keyed by (global step, global row), the value-only InfoNCE of its diffusion loss (genrecv1.py:577-582)
takes the whole step's rows as keys (gather_step_rows), and its rebuild deals whole train_batch_size
chunks of users round-robin over the ranks, each chunk drawing what it draws in one process
(tests/test_dist_gpu.py).

Opt-in GMR_DP_MODE=local ("partition users across the GPUs", BASELINE north star): every rank
takes whole train_batch_size batches (rank r takes batch g * world + r of global step g), so one
global step is world batches = the single-process step with a world x train_batch_size batch; the
epoch takes 1 / world of the optimiser steps.  This changes the reference's schedule and is
reported under its own label by bench.py, never as the default.
Everything here also runs on CPU tensors with the gloo backend (tests/test_dist_cpu.py).
"""
import os

import torch
import torch.distributed as tdist


def is_dist():
    return tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1


def dp_mode():
    """'global' (default: the reference's batch split over the ranks) or 'local' (GMR_DP_MODE=local)."""
    return "local" if os.environ.get("GMR_DP_MODE", "global") == "local" else "global"


def local_batches():
    """True when ranks take whole batches (GMR_DP_MODE=local with more than one rank)."""
    return dp_mode() == "local" and world() > 1


def step_slices(n, B, w=None, r=None):
    """The global optimiser steps over n rows in batches of B, for rank r of w: yields
    (g, lo, hi, blo, bhi, rank_rows, row0) — this rank's rows [lo, hi), the batch they belong to
    [blo, bhi) (the whole global batch in 'global' mode, the rank's own batch in 'local' mode), the
    rows every rank holds in step g, and this rank's offset inside the step's concatenated rows
    (the key of its per-row random draws)."""
    w = world() if w is None else w
    r = rank() if r is None else r
    nb = -(-n // B)
    if dp_mode() == "local" and w > 1:
        for g in range(-(-nb // w)):
            sizes = [max(0, min(n, (g * w + q + 1) * B) - min(n, (g * w + q) * B)) for q in range(w)]
            blo = min(n, (g * w + r) * B)
            bhi = blo + sizes[r]
            yield g, blo, bhi, blo, bhi, sizes, sum(sizes[:r])
        return
    for g in range(nb):
        blo, bhi = g * B, min(n, (g + 1) * B)
        a, b = shard(bhi - blo, w, r)
        yield g, blo + a, blo + b, blo, bhi, shard_sizes(bhi - blo, w), a


def world():
    return tdist.get_world_size() if is_dist() else 1


def rank():
    return tdist.get_rank() if is_dist() else 0


def shard(n, w=None, r=None):
    """Contiguous [lo, hi) slice of n items for rank r of w (first n % w ranks get one more)."""
    w = world() if w is None else w
    r = rank() if r is None else r
    q, rem = divmod(n, w)
    lo = r * q + min(r, rem)
    return lo, lo + q + (1 if r < rem else 0)


def padded_shard(n, w=None, r=None):
    """Equal-size shards (ceil(n / w)) for all-gathers: returns (lo, hi, size) with hi clipped to n."""
    w = world() if w is None else w
    r = rank() if r is None else r
    s = -(-n // w)
    lo = min(n, r * s)
    return lo, min(n, lo + s), s


def shard_sizes(n, w=None):
    """Rows of each rank's contiguous shard of an n-row batch."""
    w = world() if w is None else w
    return [shard(n, w, r)[1] - shard(n, w, r)[0] for r in range(w)]


def dp_scales(rows):
    """(norm_rows, reg_share) for one global step whose ranks hold `rows` rows each (0 = idle rank):
    every active rank divides its batch sums by the global row count and adds 1/active of the
    regulariser, so the SUM all-reduce equals the gradient of the global-batch loss."""
    active = sum(1 for x in rows if x > 0)
    return float(sum(rows)), (1.0 / active if active else 0.0)


def all_reduce_(t):
    if is_dist():
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM)
    return t


def all_reduce_start(t):
    """SUM all-reduce issued without blocking the compute stream (RCCL runs it on its own stream);
    returns a handle for wait(), or None outside a process group.  `t` must not be touched until
    then: the diffusion phase overlaps one denoiser's gradient exchange with the other's step."""
    if is_dist():
        return tdist.all_reduce(t, op=tdist.ReduceOp.SUM, async_op=True)
    return None


def wait(handle):
    """Make the current stream wait for an all_reduce_start (no host block under RCCL)."""
    if handle is not None:
        handle.wait()


def all_gather_rows_(full, size):
    """full: (world * size, ...) buffer whose rank slice [rank*size, (rank+1)*size) is filled
    locally; gathers every rank's slice in place."""
    if is_dist():
        r = rank()
        local = full[r * size:(r + 1) * size].clone()
        if tdist.get_backend() == "nccl":
            tdist.all_gather_into_tensor(full, local)
        else:  # gloo rehearsal (CPU tests, or several ranks sharing one GPU)
            parts = list(full.split(size))
            tdist.all_gather(parts, local)
            for i, p in enumerate(parts):
                full[i * size:(i + 1) * size].copy_(p)
    return full


def gather_step_rows(local, rank_rows):
    """Rows of one global step held by each rank (rank q holds rank_rows[q] rows, 0 = idle) -> the
    step's rows in rank order on every rank (one padded all-gather; idle ranks pass an empty slice)."""
    if not is_dist():
        return local
    w, r = world(), rank()
    m = max(max(rank_rows), 1)
    full = local.new_zeros((w * m,) + tuple(local.shape[1:]))
    if rank_rows[r]:
        full[r * m:r * m + rank_rows[r]].copy_(local[:rank_rows[r]])
    all_gather_rows_(full, m)
    return torch.cat([full[q * m:q * m + rank_rows[q]] for q in range(w)])


def barrier():
    if is_dist():
        tdist.barrier()


def max_scalar(x, device):
    if not is_dist():
        return x
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())
