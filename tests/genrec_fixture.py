"""Shared loaders that turn tests/golden/genrecv1_tiny.npz into oracle / HIP-path inputs."""
import numpy as np
import torch

from oracle import genrec_ref, graph_ref, model_ref

BN_NAMES = ["image_residual_project_1", "image_modal_project_1", "text_residual_project_1",
            "text_modal_project_1", "caculate_common_1", "gate_image_modal_1", "gate_text_modal_1",
            "gate_audio_modal_1"]


def sub(g, prefix):
    n = len(prefix)
    return {k[n:]: v for k, v in g.items() if k.startswith(prefix)}


def model_params(m, requires_grad=False):
    return {k[2:]: torch.tensor(v, requires_grad=requires_grad) for k, v in m.items() if k.startswith("p_")}


def fresh_bn_state(d=64):
    return {n: (torch.zeros(d), torch.ones(d)) for n in BN_NAMES}


def model_graphs(m):
    """Oracle CSR builds of every graph of the fixture (checked against the reference COO)."""
    U, I = int(m["U"]), int(m["I"])
    N = U + I
    out = {"norm_adj": graph_ref.norm_adj_csr(U, I, m["train_rows"], m["train_cols"]),
           "R": genrec_ref.user_item_csr(U, I, m["train_rows"], m["train_cols"])}
    for key, f in (("ii_img", m["v_feat"]), ("ii_txt", m["t_feat"])):
        out[key] = genrec_ref.knn_graph_csr(f, 10)[0]
    ui = graph_ref.ui_adj_csr(U, I, np.repeat(np.arange(U), 10), m["ui_k10_items"].reshape(-1))
    out["ui_full"] = ui
    out["ui_img"] = genrec_ref.drop_edges_csr(*ui, m["ui_keep_sorted"])
    dims = {"norm_adj": (N, N), "R": (U, I), "ii_img": (I, I), "ii_txt": (I, I), "ui_full": (N, N), "ui_img": (N, N)}
    return out, dims


def sparse_graphs(csrs, dims):
    return {k: model_ref.sparse_from_csr(*v, dims[k][0], dims[k][1]) for k, v in csrs.items()}


def masks_of(m, prefix):
    names = [str(s) for s in m["fwd_mask_names"]]
    return {n.replace(".", "_"): m[f"{prefix}_mask{j}"] for j, n in enumerate(names)}


def den_params(d):
    return {k[4:]: torch.tensor(v) for k, v in d.items() if k.startswith("den_") and k != "den_names"}
