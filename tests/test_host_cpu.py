"""Host-side logic (no GPU): C-ABI exports, config layering, dataset split / eval loaders vs the
reference's golden outputs, host evaluator, synthetic data recipe."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "gmr.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gmr_\w+)\s*\(", txt)))


def test_header_and_binding_agree():
    from gmr import _lib
    assert _header_symbols() == sorted(_lib.SIGNATURES)


def test_binding_arity_matches_header():
    """Every ctypes argtypes list matches the header declaration parameter by parameter (a missing,
    extra or mistyped argument would shift or truncate every later one silently)."""
    from gmr import _lib
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "gmr.h")).read(), flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    decls = dict(re.findall(r"\b(gmr_\w+)\s*\(([^)]*)\)\s*;", txt))
    assert set(decls) == set(_lib.SIGNATURES)
    ctype = {"int64_t": _lib.I64, "int32_t": _lib.I32, "uint64_t": _lib.U64, "float": _lib.F32,
             "double": _lib.F64}
    bad = {}
    for name, params in decls.items():
        params = [p.strip() for p in params.split(",") if p.strip() not in ("", "void")]
        want = [(_lib.P, _lib.CP) if "*" in p else (ctype[re.sub(r"^const\s+|\s+\w+$", "", p)],)
                for p in params]
        got = _lib.SIGNATURES[name][1]
        if len(want) != len(got) or any(g not in w for g, w in zip(got, want)):
            bad[name] = (params, got)
    assert not bad, bad


def test_library_exports_every_symbol():
    import ctypes

    import torch  # noqa: F401  (the .so binds to torch's HIP runtime)

    from gmr import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libgmr_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in _header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.gmr_version() == 2
    # pure host helpers are callable without a GPU
    f = lib.gmr_spmm_plan_words
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32]
    assert f(10, 100, 64) > 0


def test_no_cpu_fallback_without_library(monkeypatch):
    from gmr import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libgmr_hip.so")
    with pytest.raises(_lib.HipLibraryMissing):
        _lib.load()


def test_config_layering():
    from gmr.configurator import Config
    c = Config("DiffMM", "baby", {"learning_rate": 0.01})
    assert c["learning_rate"] == 0.01                       # config_dict wins
    assert c["ssl_reg"] == 1e-2 and c["dims"] == [1000]     # model yaml (active Sports block)
    assert c["USER_ID_FIELD"] == "userID"                   # dataset yaml over overall
    assert c["inter_file_name"] == "baby.inter"
    assert c["nonexistent_key"] is None
    assert c["valid_metric_bigger"] is True
    assert "seed" in c["hyper_parameters"]
    c2 = Config("DiffRec", "baby", {})
    assert c2["steps"] == 100 and c2["learning_rate"] == 1e-4


def _cfg(tmp_path):
    from gmr.configurator import Config
    return Config("DiffMM", "tinyds", {"data_path": str(tmp_path) + "/", "inter_file_name": "tinyds.inter",
                                       "USER_ID_FIELD": "userID", "ITEM_ID_FIELD": "itemID", "RATING_FIELD": "rating",
                                       "use_gpu": False})


def test_dataset_and_eval_loader_match_reference(tmp_path, golden):
    from gmr.dataloader import EvalDataLoader, TrainDataLoader
    from gmr.dataset import RecDataset
    g = golden("dataset_tiny")
    d = tmp_path / "tinyds"
    d.mkdir()
    with open(d / "tinyds.inter", "w") as f:
        f.write("userID\titemID\tx_label\trating\n")
        for u, i, lb in g["inter"]:
            f.write(f"{u}\t{i}\t{lb}\t5\n")
    cfg = _cfg(tmp_path)
    ds = RecDataset(cfg)
    assert ds.get_user_num() == int(g["user_num"]) and ds.get_item_num() == int(g["item_num"])
    tr, va, te = ds.split()
    assert len(tr) == int(g["train_len"])
    for name, part in (("valid", va), ("test", te)):
        el = EvalDataLoader(cfg, part, additional_dataset=tr, batch_size=16)
        assert np.array_equal(el.eval_u_np, g[name + "_eval_u"])
        assert np.array_equal(np.stack([el.mask_rows_np, el.mask_cols_np]), g[name + "_mask"])
        assert np.array_equal(el.get_eval_len_list(), g[name + "_eval_len"])
        assert np.array_equal(np.concatenate(el.get_eval_items()), g[name + "_eval_items"])
        assert len(el) == int(g[name + "_nbatches"])
        b0 = g[name + "_batch0_mask"]
        n0 = int(np.searchsorted(el.mask_rows_np, 16))
        assert np.array_equal(np.stack([el.mask_rows_np[:n0], el.mask_cols_np[:n0]]), b0)
    tl = TrainDataLoader(cfg, tr, batch_size=16)
    m = tl.inter_matrix()
    assert np.array_equal(m.row, g["train_coo_rows"]) and np.array_equal(m.col, g["train_coo_cols"])


def test_host_evaluator_matches_reference(golden, golden_meta):
    from gmr.topk_evaluator import TopKEvaluator
    g = golden("diffmm_tiny")
    pos = np.split(g["eval_pos_flat"], np.cumsum(g["eval_pos_len"])[:-1])

    class ED:
        def get_eval_items(self):
            return pos

        def get_eval_len_list(self):
            return g["eval_pos_len"]

    import torch
    ev = TopKEvaluator({"metrics": ["Recall", "NDCG", "Precision", "MAP"], "topk": [5, 10, 20, 50],
                        "save_recommended_topk": False})
    got = ev.evaluate([torch.as_tensor(g["eval_topk"])], ED(), is_test=False)
    assert got == golden_meta["diffmm_metrics"]["rounded"]


def test_synthetic_recipe():
    from gmr.synthetic import make_features, make_interactions
    u, i, lb = make_interactions(300, 200, 3000, seed=0)
    assert np.bincount(u).min() >= 5
    for uu in range(300):
        it = i[u == uu]
        assert len(np.unique(it)) == len(it)
        lab = lb[u == uu]
        n = len(it)
        if n < 10:
            assert (lab == 0).sum() == n - 2 and (lab == 1).sum() == 1 and (lab == 2).sum() == 1
    v, t = make_features(200, 32, 16)
    assert (v >= 0).all() and np.allclose(np.linalg.norm(t, axis=1), 1, atol=1e-5)


def test_every_abi_call_site_matches_its_signature():
    """Static check of every _lib.call("gmr_...", ...) in the package: the argument count equals the
    ctypes signature (a surplus argument would silently shift the stream pointer)."""
    import ast
    import glob

    from gmr import _lib
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "generative-multimodal-recommendation_amd", "gmr")
    bad = []
    for f in glob.glob(os.path.join(pkg, "*.py")):
        for node in ast.walk(ast.parse(open(f).read())):
            if (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute) and node.func.attr == "call"
                    and node.args and isinstance(node.args[0], ast.Constant) and str(node.args[0].value).startswith("gmr_")):
                name = node.args[0].value
                if any(isinstance(a, ast.Starred) for a in node.args):
                    continue
                want = len(_lib.SIGNATURES[name][1])
                if len(node.args) - 1 != want:
                    bad.append(f"{os.path.basename(f)}:{node.lineno} {name}: {len(node.args) - 1} args, signature {want}")
    assert not bad, bad
