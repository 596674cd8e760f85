"""the on-device BPR epoch sampler and diffusion batch permutation.

The reference draws each epoch on the host (utils/dataloader.py:226-275): the interactions in a
shuffled order, one negative per row drawn uniformly from the training items (`all_items`, :116)
and redrawn while it is in the user's history (:267-275); the diffusion phase iterates a
DataLoader(shuffle=True) over all users (common/trainer.py:462).  Our sampler uses its own
Philox streams, so it is checked on the properties the reference's draws have:
  * every train interaction appears exactly once per epoch (a permutation of the rows);
  * every negative is a training item outside the user's history; a user holding every item
    cannot get one (the reference would loop forever): those rows are counted, not hidden;
  * negatives are uniform over all_items (chi-square), epochs differ, and a (seed, epoch) pair
    redraws the same epoch;
  * the per-(batch, rank) scatter plans hold exactly the sorted keys of their sub-batch;
  * the user permutation of the diffusion phase is a bijection.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _loader(users, items, U, I, batch=64):
    from gmr.configurator import Config
    from gmr.dataloader import TrainDataLoader
    from gmr.dataset import RecDataset
    cfg = Config("DiffMM", "baby", {"train_batch_size": batch, "seed": [999]})
    rng = np.random.default_rng(0)
    ds = RecDataset.from_arrays(cfg, users, items, np.zeros(len(users), np.int64), U, I,
                                rng.random((I, 8), dtype=np.float32), rng.random((I, 8), dtype=np.float32))
    return TrainDataLoader(cfg, ds, batch_size=batch)


def _data(seed=0, U=300, I=200):
    rng = np.random.default_rng(seed)
    us, its = [], []
    for u in range(U):
        d = int(rng.integers(5, 30))
        us.append(np.full(d, u))
        its.append(rng.choice(I, size=d, replace=False))
    return np.concatenate(us), np.concatenate(its), U, I


def test_epoch_is_a_permutation_with_true_negatives():
    users, items, U, I = _data()
    tl = _loader(users, items, U, I)
    d = tl.epoch()
    s = d["sample"].cpu().numpy()
    assert tl.fallbacks() == 0
    got = np.sort(s[0].astype(np.int64) * I + s[1])
    want = np.sort(users.astype(np.int64) * I + items)
    assert np.array_equal(got, want)                                 # each interaction once
    hist = set((users.astype(np.int64) * I + items).tolist())
    assert not any(int(u) * I + int(n) in hist for u, n in zip(s[0], s[2]))   # negatives not in history
    assert np.isin(s[2], tl.all_items_np).all()                      # drawn from the training items
    # a second epoch reshuffles; the same (seed, epoch) redraws the same epoch
    s2 = tl.epoch()["sample"].cpu().numpy()
    assert not np.array_equal(s2, s)
    tl._epoch = 0
    s0 = tl.epoch()["sample"].cpu().numpy()
    assert np.array_equal(s0, s)


def test_negatives_uniform_over_training_items():
    users, items, U, I = _data(seed=1)
    # only users with few items, so the rejection step hardly biases the marginal
    tl = _loader(users, items, U, I)
    counts = np.zeros(I)
    for _ in range(20):
        s = tl.epoch()["sample"].cpu().numpy()
        counts += np.bincount(s[2], minlength=I)
    ai = tl.all_items_np
    c = counts[ai]
    # expected count of item j: sum over rows of 1/(|all_items| - |history|) for users not holding j
    deg = np.bincount(users, minlength=U)
    per_row = np.repeat(1.0 / (len(ai) - deg), deg)
    held = np.zeros((U, I), bool)
    held[users, items] = True
    exp = np.zeros(I)
    row_user = np.repeat(np.arange(U), deg)
    for j in ai:
        exp[j] = 20 * per_row[~held[row_user, j]].sum()
    chi2 = float(((c - exp[ai]) ** 2 / exp[ai]).sum())
    dof = len(ai) - 1
    assert chi2 < dof + 6 * np.sqrt(2 * dof), (chi2, dof)


def test_user_with_every_item_is_counted_as_fallback():
    users, items, U, I = _data(seed=2, U=40, I=30)
    full = np.arange(I)
    users = np.concatenate([users, np.full(I, U)])                   # user U holds every item
    items = np.concatenate([items, full])
    tl = _loader(users, items, U + 1, I)
    s = tl.epoch()["sample"].cpu().numpy()
    assert tl.fallbacks() == I                                       # one per row of that user
    others = s[0] != U
    hist = set((users.astype(np.int64) * I + items).tolist())
    assert not any(int(u) * I + int(n) in hist for u, n in zip(s[0][others], s[2][others]))


def test_sub_batch_plans_hold_sorted_keys():
    users, items, U, I = _data(seed=3)
    tl = _loader(users, items, U, I, batch=96)
    d = tl.epoch()
    s = d["sample"].cpu().numpy().astype(np.int64)
    for b, rank_rows, u, p, n, pb, pc in tl.batches(d):
        rows = sum(rank_rows)
        lo = b * 96
        assert rows == min(96, tl.n_inter - lo) and u.numel() == rows
        keys = np.concatenate([s[0, lo:lo + rows], s[1, lo:lo + rows] + U, s[2, lo:lo + rows] + U])
        plan = pb.cpu().numpy().view(np.uint64)
        valid = plan[plan != np.iinfo(np.uint64).max]
        assert np.array_equal(np.sort(keys), (valid >> np.uint64(32)).astype(np.int64))
        slots = (valid & np.uint64(0xFFFFFFFF)).astype(np.int64)
        assert np.array_equal(keys[slots], (valid >> np.uint64(32)).astype(np.int64))


@pytest.mark.parametrize("n", [1, 2, 7, 1000, 19445, 100003])
def test_diffusion_permutation_is_a_bijection(n):
    from gmr import _lib
    from gmr.kernels import ptr, stream
    out = torch.empty(n, dtype=torch.int32, device=DEV)
    _lib.call("gmr_permutation", n, 999, 1000, ptr(out), stream())
    a = out.cpu().numpy()
    assert np.array_equal(np.sort(a), np.arange(n))
    if n >= 1000:
        out2 = torch.empty(n, dtype=torch.int32, device=DEV)
        _lib.call("gmr_permutation", n, 999, 1001, ptr(out2), stream())
        assert not np.array_equal(out2.cpu().numpy(), a)             # the next epoch reshuffles
