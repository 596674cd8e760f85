"""torch-CPU fp32 restatement of GenRecV1 — TEST ORACLE ONLY.

Plain functions over explicit parameter dicts (names as the reference's named_parameters with
'.' -> '_') so tests feed the same tensors to the oracle and to the HIP path.  Every random draw
(dropout keep masks, flip masks, p_sample Bernoulli outcomes, random.sample picks) is an explicit
input.  Line references are to GenMMRec/src of the reference snapshot.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from .model_ref import sparse_from_csr  # noqa: F401  (re-exported for the tests)

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
LN_EPS = 1e-5


# ----------------------------------------------------------------------------- graphs
def knn_graph_csr(feat, k):
    """_build_knn_adj + build_knn_normalized_graph(is_sparse, 'sym') — common/trainer.py:682-687,
    utils/utils.py:152-163,184-197.  sim = normalize(F) normalize(F)^T; top-k per row (values kept,
    may be negative); deg[r] = sum of row r's kept values (fp32, top-k order); w = d_r * v * d_c with
    d = deg^-1/2 (inf -> 0).  Returns CSR (columns ascending) + the raw top-k (idx, val)."""
    fn = F.normalize(torch.as_tensor(feat, dtype=torch.float32), p=2, dim=-1)
    sim = fn @ fn.t()
    val, idx = torch.topk(sim, k, dim=-1)
    n = sim.shape[0]
    deg = torch.zeros(n).index_add_(0, torch.arange(n).repeat_interleave(k), val.reshape(-1))
    d = deg.pow(-0.5)
    d[torch.isinf(d)] = 0.0
    w = d[:, None] * val * d[idx]
    rows = np.repeat(np.arange(n), k)
    cols = idx.numpy().reshape(-1)
    order = np.lexsort((cols, rows))
    rowptr = np.zeros(n + 1, np.int64)
    np.add.at(rowptr, rows + 1, 1)
    return (np.cumsum(rowptr).astype(np.int32), cols[order].astype(np.int32),
            w.numpy().reshape(-1)[order].astype(np.float32)), (idx.numpy(), val.numpy())


def drop_edges_csr(rowptr, col, val, keep, keep_rate=0.5):
    """SpAdjDropEdge — models/genrecv1.py:443-457: kept edges scaled by 1/keep_rate.
    keep: per-entry flags in CSR (row-major, columns ascending) order."""
    keep = np.asarray(keep).astype(bool)
    n = len(rowptr) - 1
    rows = np.repeat(np.arange(n), np.diff(rowptr))[keep]
    nrp = np.zeros(n + 1, np.int64)
    np.add.at(nrp, rows + 1, 1)
    v = (torch.as_tensor(val[keep]) / keep_rate).numpy()
    return np.cumsum(nrp).astype(np.int32), np.asarray(col)[keep].astype(np.int32), v.astype(np.float32)


def user_item_csr(n_users, n_items, rows, cols):
    """R = raw binary U x I interactions (models/genrecv1.py:128-131)."""
    key = np.unique(np.asarray(rows, np.int64) * n_items + np.asarray(cols, np.int64))
    u, i = key // n_items, key % n_items
    rp = np.zeros(n_users + 1, np.int64)
    np.add.at(rp, u + 1, 1)
    return np.cumsum(rp).astype(np.int32), i.astype(np.int32), np.ones(len(i), np.float32)


# ----------------------------------------------------------------------------- rec model
def batch_norm(x, w, b, state, name, train):
    """nn.BatchNorm1d (eps 1e-5, momentum 0.1): batch stats (biased var) in train mode and a
    running-stat update with the unbiased var; running stats in eval mode."""
    if train:
        mean = x.mean(0)
        var = x.var(0, unbiased=False)
        n = x.shape[0]
        with torch.no_grad():
            rm, rv = state[name]
            state[name] = ((1 - BN_MOMENTUM) * rm + BN_MOMENTUM * mean.detach(),
                           (1 - BN_MOMENTUM) * rv + BN_MOMENTUM * var.detach() * n / (n - 1))
    else:
        mean, var = state[name]
    return (x - mean) / torch.sqrt(var + BN_EPS) * w + b


def _dropout(x, mask, p=0.1):
    if mask is None:
        return x
    return x * torch.as_tensor(mask, dtype=torch.float32) / (1 - p)


def modal_feature(p, feat, mod, state, train, masks):
    """getImageFeats / getTextFeats — models/genrecv1.py:225-239 (Linear -> BN -> LeakyReLU(0.2)
    -> Dropout(0.1), twice, then res_scale * x + modal)."""
    pre = f"{mod}_residual_project_"
    x = feat @ p[pre + "0_weight"].t() + p[pre + "0_bias"]
    x = _dropout(F.leaky_relu(batch_norm(x, p[pre + "1_weight"], p[pre + "1_bias"], state, pre + "1", train), 0.2),
                 masks.get(pre + "3") if train else None)
    pre2 = f"{mod}_modal_project_"
    m = x @ p[pre2 + "0_weight"].t() + p[pre2 + "0_bias"]
    m = _dropout(F.leaky_relu(batch_norm(m, p[pre2 + "1_weight"], p[pre2 + "1_bias"], state, pre2 + "1", train), 0.2),
                 masks.get(pre2 + "3") if train else None)
    return p["res_scale"] * x + m


def gate(p, name, x, state, train):
    """_build_gate: Linear -> BN -> Sigmoid (models/genrecv1.py:155-164)."""
    z = x @ p[name + "_0_weight"].t() + p[name + "_0_bias"]
    return torch.sigmoid(batch_norm(z, p[name + "_1_weight"], p[name + "_1_bias"], state, name + "_1", train))


def forward(p, feats, graphs, state, train=True, masks=None):
    """GenRecV1.forward — models/genrecv1.py:255-353 (image + text, n_layers = 1).
    graphs: norm_adj, ui_img (dropped rebuilt UI graph), ii_img, ii_txt (kNN), R (U x I), as
    torch sparse tensors.  state: BN running stats {name: (mean, var)} (updated in train mode).
    Returns (content N x d, side N x d)."""
    masks = masks or {}
    U = p["user_embedding_weight"].shape[0]
    E = torch.cat([p["user_embedding_weight"], p["item_id_embedding_weight"]])
    c1 = torch.stack([E, torch.sparse.mm(graphs["norm_adj"], E)], 1).mean(1)
    c2 = torch.stack([E, torch.sparse.mm(graphs["ui_img"], E)], 1).mean(1)
    w = torch.softmax(torch.stack([p["origin_weight"], p["generation_weight"]]), 0)
    content = w[0] * c1 + w[1] * c2
    iE = p["item_id_embedding_weight"]
    ui = []
    for mod, gname, ii in (("image", "gate_image_modal", "ii_img"), ("text", "gate_text_modal", "ii_txt")):
        f = modal_feature(p, feats[mod], mod, state, train, masks)
        x = iE * gate(p, gname, f, state, train)
        x = torch.sparse.mm(graphs[ii], x)
        ui.append(torch.cat([torch.sparse.mm(graphs["R"], x), x]))
    img, txt = ui

    def common_score(x):
        z = x @ p["caculate_common_0_weight"].t() + p["caculate_common_0_bias"]
        z = torch.tanh(batch_norm(z, p["caculate_common_1_weight"], p["caculate_common_1_bias"], state,
                                  "caculate_common_1", train))
        return z @ p["caculate_common_3_weight"].t()

    att = torch.softmax(torch.cat([common_score(img), common_score(txt)], -1), -1)
    common = att[:, 0:1] * img + att[:, 1:2] * txt
    si, st = img - common, txt - common
    pi = gate(p, "gate_image_modal", content, state, train)
    pt = gate(p, "gate_text_modal", content, state, train)
    side = (pi * si + pt * st + common) / 4
    return content, side


def info_nce(v1, v2, temperature):
    """GenRecV1.infoNCE_loss / FlipInterestDiffusion.infoNCE_loss — models/genrecv1.py:407-414, 641-648."""
    v1, v2 = F.normalize(v1, dim=1), F.normalize(v2, dim=1)
    pos = torch.exp(torch.sum(v1 * v2, -1) / temperature)
    neg = torch.exp(v1 @ v2.t() / temperature).sum(1)
    return -torch.log(pos / neg).mean()


def calculate_loss(p, feats, graphs, state, users, pos, neg, masks=None, reg_weight=1e-5, temp=0.55,
                   ssl_reg1=0.1, ssl_reg2=0.1):
    """GenRecV1.calculate_loss — models/genrecv1.py:355-405."""
    U = p["user_embedding_weight"].shape[0]
    content, side = forward(p, feats, graphs, state, True, masks)
    usr, itm = content[:U], content[U:]
    a, pe, ne = usr[users], itm[pos], itm[neg]
    bpr = -torch.mean(F.logsigmoid((a * pe).sum(-1) - (a * ne).sum(-1)))
    reg = (p["user_embedding_weight"].norm(2).square() + p["item_id_embedding_weight"].norm(2).square()) * reg_weight
    su, si = side[:U], side[U:]
    cl1 = info_nce(si[pos], itm[pos], temp) + info_nce(su[users], usr[users], temp)
    cl2 = info_nce(usr[users], itm[pos], temp) + info_nce(usr[users], si[pos], temp)
    return bpr + reg + cl1 * ssl_reg1 + cl2 * ssl_reg2


# ----------------------------------------------------------------------------- denoiser
def time_embedding(t, emb_size=10):
    """ModalDenoiseTransformer.forward :692-696 (cos/sin of t * 10000^(-k/half))."""
    half = emb_size // 2
    freqs = torch.exp(-math.log(10000) * torch.arange(0, half, dtype=torch.float32) / half)
    temp = torch.as_tensor(t)[:, None].float() * freqs[None]
    te = torch.cat([torch.cos(temp), torch.sin(temp)], -1)
    if emb_size % 2:
        te = torch.cat([te, torch.zeros_like(te[:, :1])], -1)
    return te


def denoiser(w, x, t, n_layers, nhead=8, emb_size=10):
    """ModalDenoiseTransformer.forward — models/genrecv1.py:691-710, dropout off (eval or p = 0).
    nn.TransformerDecoderLayer (post-norm, ReLU) on a length-1 target with zero memory: self-attention
    reduces to out_proj(V), cross-attention to the constant out_proj(b_v)."""
    x = torch.as_tensor(x, dtype=torch.float32)
    te = time_embedding(t, emb_size) @ w["emb_layer_weight"].t() + w["emb_layer_bias"]
    h = torch.cat([x, te], -1) @ w["input_proj_weight"].t() + w["input_proj_bias"]
    ada = F.silu(te) @ w["adaLN_modulation_1_weight"].t() + w["adaLN_modulation_1_bias"]
    D = h.shape[1]
    shift, scale = ada[:, :D], ada[:, D:]
    h = h * (1 + scale) + shift
    for l in range(n_layers):
        pre = f"transformer_decoder_layers_{l}_"
        Wsa, bsa = w[pre + "self_attn_in_proj_weight"], w[pre + "self_attn_in_proj_bias"]
        v = h @ Wsa[2 * D:].t() + bsa[2 * D:]
        sa = v @ w[pre + "self_attn_out_proj_weight"].t() + w[pre + "self_attn_out_proj_bias"]
        h = F.layer_norm(h + sa, (D,), w[pre + "norm1_weight"], w[pre + "norm1_bias"], LN_EPS)
        bca = w[pre + "multihead_attn_in_proj_bias"][2 * D:]
        ca = bca @ w[pre + "multihead_attn_out_proj_weight"].t() + w[pre + "multihead_attn_out_proj_bias"]
        h = F.layer_norm(h + ca, (D,), w[pre + "norm2_weight"], w[pre + "norm2_bias"], LN_EPS)
        ff = F.relu(h @ w[pre + "linear1_weight"].t() + w[pre + "linear1_bias"])
        ff = ff @ w[pre + "linear2_weight"].t() + w[pre + "linear2_bias"]
        h = F.layer_norm(h + ff, (D,), w[pre + "norm3_weight"], w[pre + "norm3_bias"], LN_EPS)
    o = h @ w["output_proj_0_weight"].t() + w["output_proj_0_bias"]
    o = F.layer_norm(o, (o.shape[1],), w["output_proj_1_weight"], w["output_proj_1_bias"], LN_EPS)
    o = F.gelu(o)
    return o @ w["output_proj_3_weight"].t() + w["output_proj_3_bias"]


# ----------------------------------------------------------------------------- flip diffusion
def flip_schedule(x0, steps=5):
    """FlipInterestDiffusion.get_cum — models/genrecv1.py:480-498 (from the batch sparsity)."""
    x0 = torch.as_tensor(x0)
    s = (x0 == 0).float().mean()
    gs = 0.1 * (1 - s) + 0.001
    es = 0.005 * s + 0.0001
    gamma = torch.linspace(gs, gs * 0.1, steps)
    eps = torch.clamp(torch.linspace(es, es * 0.1, steps), max=0.01)
    return 1 - torch.cumprod(1 - gamma, 0), 1 - torch.cumprod(1 - eps, 0)


def flip_prob(x0, t, noise, gamma_cum, eps_cum, temp=1.0):
    """q_sample's flip probability — models/genrecv1.py:512-522."""
    x0 = torch.as_tensor(x0)
    a0 = gamma_cum[torch.as_tensor(t)][:, None]
    a1 = eps_cum[torch.as_tensor(t)][:, None]
    return torch.where(x0 == 0, torch.sigmoid((a0 - noise) * temp), torch.sigmoid((a1 - noise) * temp))


def flip_apply(x0, flip):
    """x_t[flip] = 1 - x_t[flip] (:523-526)."""
    x0 = torch.as_tensor(x0)
    return torch.where(torch.as_tensor(flip).bool(), 1 - x0, x0)


def bayes_step_prob(probs, a0, a1):
    """p_sample's Bayesian posterior for i > 0 (:540-545): p1 / (p0 + p1)."""
    p0 = probs * (1 - a0) + (1 - probs) * a1
    p1 = probs * a0 + (1 - probs) * (1 - a1)
    return p1 / (p0 + p1)


def p_sample(w, x0, gamma_cum, eps_cum, flip_mask, step_draws, n_layers, steps=5):
    """FlipInterestDiffusion.p_sample(steps = T, bayesian) — models/genrecv1.py:528-548, with the
    q_sample flip mask and the T Bernoulli outcomes given.  The prev-step coefficients are the
    q_sample(t = T-1) tensors re-indexed by row (:541-542 index self.alpha_bar0_t, a B x I tensor,
    by t-1), i.e. gamma_cum[T-1] / eps_cum[T-1] for every step.  Returns (x, probs, [logits])."""
    B = x0.shape[0]
    x = flip_apply(x0, flip_mask)
    a0, a1 = gamma_cum[steps - 1], eps_cum[steps - 1]
    lgs = []
    probs = None
    for j, i in enumerate(reversed(range(steps))):
        lg = denoiser(w, x, np.full(B, i), n_layers)
        lgs.append(lg)
        probs = torch.sigmoid(lg)
        x = torch.as_tensor(step_draws[j], dtype=torch.float32)
    return x, probs, lgs


def training_losses(w, x0, t, flip1, item_embeds, feats, ps_flip, ps_draws, gamma_cum, eps_cum, n_layers,
                    steps=5, sparse_temp=0.5):
    """FlipInterestDiffusion.training_losses (audio off) — models/genrecv1.py:550-606:
    bce(pos_weight) + curriculum KL (detached) + 0.01 InfoNCE(x0 E, p_sample(x0) E) (no grad path).
    The focal loss (:557-571) and the text InfoNCE (:584-587) are computed by the reference but
    unused in the returned loss.  Returns (total, bce, kl, cl, logits)."""
    x0 = torch.as_tensor(x0, dtype=torch.float32)
    pw = torch.sum(1 - x0) / (torch.sum(x0) + 1e-8)
    xt = flip_apply(x0, flip1)
    logits = denoiser(w, xt, t, n_layers)
    probs = torch.sigmoid(logits)
    bce = F.binary_cross_entropy_with_logits(logits, x0, pos_weight=pw)
    gen, _, _ = p_sample(w, x0, gamma_cum, eps_cum, ps_flip, ps_draws, n_layers, steps)
    fe = item_embeds * feats
    cl = info_nce(x0 @ fe, gen @ fe, sparse_temp)
    # KL against the true posterior; alpha tables as left by p_sample's q_sample (t = T-1)
    eps = 1e-8
    a0, a1 = gamma_cum[steps - 1], eps_cum[steps - 1]
    num = (x0 == 0).float() * (1 - a0) + (x0 == 1).float() * a1
    den = (x0 == 0).float() * (1 - a0 + a1) + (x0 == 1).float() * (a0 + 1 - a1)
    post = torch.clamp((num / (den + eps)).detach(), eps, 1 - eps)
    pr = torch.clamp(probs.detach(), eps, 1 - eps)
    kl = post * (torch.log(post + 1e-10) - torch.log(pr + 1e-10))
    kl = kl + (1 - post) * (torch.log(1 - post + 1e-10) - torch.log(1 - pr + 1e-10))
    cw = torch.clamp(torch.as_tensor(t).float() / steps, 0, 0.5)
    klm = (cw * kl.mean(1)).mean()
    return bce + klm + 0.01 * cl, bce, klm, cl, logits


# ----------------------------------------------------------------------------- rebuild
def interest_debias(x0, gen, labels, dislike_pick, like_pick):
    """InterestDebiase.interest_query_debiase — common/interest_cluster.py:248-332 with the
    random.sample picks given as (row, item) pairs.  Image labels serve every modality (:258-267,
    :343), so a 0->1 pick keeps 1 iff the item's cluster is in the row's history clusters, and a
    1->0 pick becomes 0 iff the row's count of that cluster <= min count + 1 (else 1)."""
    x0 = np.asarray(x0)
    out = np.array(gen, dtype=np.float32, copy=True)
    labels = np.asarray(labels)
    for u, i in np.asarray(dislike_pick).reshape(-1, 2):
        hist = labels[np.where(x0[u] > 0)[0]]
        out[u, i] = 1.0 if labels[i] in set(hist.tolist()) else 0.0
    for u, i in np.asarray(like_pick).reshape(-1, 2):
        hist = labels[np.where(x0[u] > 0)[0]]
        uniq, cnt = np.unique(hist, return_counts=True)
        cc = dict(zip(uniq.tolist(), cnt.tolist()))
        cur = cc.get(int(labels[i]), 0)
        mn = min(cc.values()) if cc else 0
        out[u, i] = 0.0 if cur <= mn + 1 else 1.0
    return out


def rebuild_rows(x0, ps_out, ps_probs, labels, dislike_pick, like_pick, gen_topk=5, rebuild_k=10):
    """GenRecV1Trainer rebuild of one batch — common/trainer.py:741-783: gen_topk mask on the
    p_sample probabilities, debias, then top-rebuild_k of denoised * probs (ties -> lowest index
    here; torch's CPU top-k breaks the zero-valued ties in an unspecified order)."""
    probs = torch.as_tensor(ps_probs)
    _, ind = torch.topk(probs, k=gen_topk, dim=1)
    mask = torch.zeros_like(probs, dtype=torch.bool).scatter_(1, ind, True)
    den = torch.where(mask, torch.as_tensor(ps_out), torch.as_tensor(x0, dtype=torch.float32))
    deb = torch.as_tensor(interest_debias(x0, den.numpy(), labels, dislike_pick, like_pick))
    score = (deb * probs).numpy()
    order = np.argsort(-score, axis=1, kind="stable")[:, :rebuild_k]
    return mask.numpy(), den.numpy(), deb.numpy(), order
