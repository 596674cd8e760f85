"""test-time evaluator extras and the top-K CSV, against the reference's own
evaluate(is_test=True) output on a small fixed top-K matrix (tests/golden/diffmm_phases_tiny.npz,
made by make_golden.py --phases with utils/topk_evaluator.py:77-270 and save_recommended_topk on).

  * host path (TopKEvaluator.evaluate, CPU): every metric and extra equal to the reference's dict
    (to the last of its 4 rounded decimals), and the CSV text identical (the file name differs
    only in its timestamp);
  * device path (evaluate_device, -m gpu): the same dict from gmr_eval_metrics(_sel) and
    gmr_topk_item_counts, and the same CSV.
The baby-shape test split (tests/test_baby_gpu.py::test_test_split_extras) checks the device
extras at the north-star shape.
"""
import json
import os
import re

import numpy as np
import pytest
import torch


class _DS:
    def __init__(self, n_items):
        self.item_num = n_items


class _Eval:
    """The EvalDataLoader surface the evaluator uses (utils/dataloader.py:330-416)."""

    def __init__(self, users, pos, n_items, device=None):
        self.eval_u_np = np.asarray(users, np.int64)
        self.pos = [np.asarray(p, np.int64) for p in pos]
        self.dataset = _DS(n_items)
        self.device = device
        self._dev = None

    def get_eval_items(self):
        return self.pos

    def get_eval_len_list(self):
        return np.asarray([len(p) for p in self.pos])

    def get_eval_users(self):
        return torch.as_tensor(self.eval_u_np)

    def to_device(self):
        if self._dev is None:
            ptr = np.concatenate([[0], np.cumsum(self.get_eval_len_list())]).astype(np.int64)
            items = np.concatenate([np.sort(p) for p in self.pos]).astype(np.int32)
            self._dev = {"pos_ptr": torch.as_tensor(ptr).to(self.device),
                         "pos_items": torch.as_tensor(items).to(self.device)}
        return self._dev


def _fixture(golden):
    ph = golden("diffmm_phases_tiny")
    lens = ph["csv_pos_len"]
    pos = np.split(ph["csv_pos_flat"], np.cumsum(lens)[:-1])
    return ph, pos


def _config(out_dir):
    from gmr.configurator import Config
    c = Config("DiffMM", "baby", {"save_recommended_topk": True, "recommend_topk": str(out_dir), "dataset": "tiny"})
    c["pop_items"] = set(range(0, 80, 3))
    c["warm_users"] = {5, 7, 30, 4}
    c["dataset"] = "tiny"
    return c


def _check(res, ph, out_dir):
    want = json.loads(str(ph["csv_extras_json"]))
    assert set(want) <= set(res), sorted(set(want) - set(res))
    # values are rounded to 4 decimals (topk_evaluator.py:120): equal, or one unit apart where the
    # unrounded value sits on a rounding boundary and the summation order decides (Warm_MAP@10 here)
    bad = {k: (res[k], v) for k, v in want.items() if abs(float(res[k]) - float(v)) > 1.01e-4}
    assert sum(abs(float(res[k]) - float(v)) > 1e-12 for k, v in want.items()) <= 2
    assert not bad, bad
    files = [f for f in os.listdir(out_dir) if f.endswith(".csv")]
    assert len(files) == 1
    stamp = re.compile(r"-[A-Z][a-z]{2}-\d{2}-\d{4}-\d{2}-\d{2}-\d{2}\.csv$")
    assert stamp.sub("", files[0]) == stamp.sub("", str(ph["csv_name"]))
    with open(os.path.join(out_dir, files[0])) as f:
        assert f.read() == str(ph["csv_text"])


def test_extras_and_csv_host(golden, tmp_path):
    from gmr.topk_evaluator import TopKEvaluator
    ph, pos = _fixture(golden)
    ev = TopKEvaluator(_config(tmp_path))
    res = ev.evaluate([torch.as_tensor(ph["csv_topk"])], _Eval(ph["csv_users"], pos, 80), is_test=True)
    _check(res, ph, tmp_path)


@pytest.mark.gpu
def test_extras_and_csv_device(golden, tmp_path):
    from gmr.topk_evaluator import TopKEvaluator
    ph, pos = _fixture(golden)
    ev = TopKEvaluator(_config(tmp_path))
    topk = torch.as_tensor(ph["csv_topk"].astype(np.int32)).to("cuda")
    res = ev.evaluate_device(topk, _Eval(ph["csv_users"], pos, 80, device="cuda"), is_test=True)
    _check(res, ph, tmp_path)
