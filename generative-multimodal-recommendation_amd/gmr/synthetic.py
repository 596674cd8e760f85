"""Synthetic Amazon-shaped interaction data (no dataset ships with the reference: data/README.md).

Recipe: numpy default_rng(seed); per-user degree max(5, 5 + Poisson(nnz/U - 5));
item popularity Zipf(s=0.8) over a random permutation, items drawn without replacement; split per
preprocessing/1splitting.ipynb (n < 10: n-2 train, 1 valid, 1 test; else 20 % held out, split
evenly between valid and test); image features |N(0,1)| (4096-d CNN fc7 is post-ReLU), text
features N(0,1) rows L2-normalised (384-d MiniLM).
"""
import numpy as np

SHAPES = {
    # name: (users, items, interactions, image dim, text dim)
    "baby": (19445, 7050, 160792, 4096, 384),
    "sports": (35598, 18357, 296337, 4096, 384),
    "tiny": (600, 400, 6000, 256, 64),
    # TikTok-shaped (config 5; public GenRec-V1 statistics, shape only): image 128-d, text 768-d
    "tiktok": (9319, 6710, 59541, 128, 768),
}
# feature value distributions: Amazon shapes as above; TikTok features N(0, 1)
GAUSSIAN_FEATS = {"tiktok"}


def make_interactions(n_users, n_items, n_inter, seed=0, zipf_s=0.8):
    rng = np.random.default_rng(seed)
    lam = max(n_inter / n_users - 5.0, 0.0)
    deg = np.maximum(5, 5 + rng.poisson(lam, size=n_users))
    deg = np.minimum(deg, n_items)
    perm = rng.permutation(n_items)
    pop = np.empty(n_items)
    pop[perm] = 1.0 / np.arange(1, n_items + 1) ** zipf_s
    pop /= pop.sum()
    users, items, labels = [], [], []
    for u in range(n_users):
        n = int(deg[u])
        it = rng.choice(n_items, size=n, replace=False, p=pop)
        if n < 10:
            lb = [0] * (n - 2) + [1, 2]
        else:
            nh = int(round(0.2 * n))
            nv = nh // 2
            lb = [0] * (n - nh) + [1] * nv + [2] * (nh - nv)
        users.append(np.full(n, u))
        items.append(it)
        labels.append(np.asarray(lb))
    return np.concatenate(users), np.concatenate(items), np.concatenate(labels)


def make_features(n_items, dv, dt, seed=0, gaussian=False):
    rng = np.random.default_rng(seed + 1)
    v = rng.standard_normal((n_items, dv), dtype=np.float32)
    t = rng.standard_normal((n_items, dt), dtype=np.float32)
    if not gaussian:
        v = np.abs(v)
        t /= np.linalg.norm(t, axis=1, keepdims=True)
    return v, t


def make_dataset(config, shape="baby", seed=0):
    """A RecDataset of the named shape with in-memory features."""
    from .dataset import RecDataset
    U, I, n, dv, dt = SHAPES[shape]
    u, i, lb = make_interactions(U, I, n, seed)
    v, t = make_features(I, dv, dt, seed, gaussian=shape in GAUSSIAN_FEATS)
    return RecDataset.from_arrays(config, u, i, lb, user_num=U, item_num=I, v_feat=v, t_feat=t)
