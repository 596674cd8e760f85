"""The drop-in entry surface: utils/quick_start.py:26-182 and src/main.py:17-27 of the
reference, driven the way a user of the reference drives them.

  * quick_start(model, dataset, config_dict) in-process for the four hot-path models on the tiny
    synthetic shape: one grid point, one epoch; the returned (params, best_valid, best_test) carry the
    metric keys Trainer.fit reports (lower-case 'recall@20', ... as trainer.py:238-343), the log file
    holds the reference's log lines, and save_model writes the reference's checkpoint keys;
  * `python main.py --model X --dataset baby --synthetic tiny --epochs 1` as a fresh child process
    (its own HIP context): exit status 0 and the same metric keys in its log.
"""
import glob
import os
import re
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "generative-multimodal-recommendation_amd")


def _fit_keys(cfg):
    """The metric keys Trainer.fit returns (trainer.py:74-77 zero dict = evaluate's keys)."""
    return {f"{m.lower()}@{k}" for m in cfg["metrics"] for k in cfg["topk"]}


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model", ["DiffMM", "VBPR", "DiffRec", "GenRecV1"])
def test_quick_start_in_process(model, tmp_path, monkeypatch):
    from gmr.configurator import Config
    from gmr.quick_start import quick_start
    monkeypatch.chdir(tmp_path)
    saved = tmp_path / "saved"
    cfg_dict = {"synthetic": "tiny", "epochs": 1, "checkpoint_dir": str(saved), "save_recommended_topk": False}
    results = quick_start(model, "baby", cfg_dict, save_model=True)
    assert len(results) == 1
    params, best_valid, best_test = results[0]
    want = _fit_keys(Config(model, "baby", dict(cfg_dict)))
    assert set(best_valid) == want, sorted(set(best_valid) ^ want)
    assert want <= set(best_test)  # the test pass adds the is_test extras
    assert all(0.0 <= best_valid[k] <= 1.0 for k in want)
    logs = glob.glob(str(tmp_path / "log" / f"{model}-baby-*.log"))
    assert len(logs) == 1
    text = open(logs[0]).read()
    assert "epoch 0 training [time:" in text and "best valid result:" in text and "recall@20: " in text
    ck = torch.load(str(saved / f"{model}-baby.pth"), map_location="cpu", weights_only=True)
    assert {"config", "epoch", "state_dict", "optimizer", "best_valid_score"} <= set(ck)


@pytest.mark.timeout(420)
@pytest.mark.parametrize("model", ["DiffMM", "VBPR"])
def test_main_py_child_process(model, tmp_path):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([PKG, ROOT, env.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, os.path.join(PKG, "main.py"), "--model", model, "--dataset", "baby",
                        "--synthetic", "tiny", "--epochs", "1"], cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    logs = glob.glob(str(tmp_path / "log" / f"{model}-baby-*.log"))
    assert len(logs) == 1
    text = open(logs[0]).read()
    line = [ln for ln in text.splitlines() if "best valid result:" in ln][-1]
    got = set(re.findall(r"([a-z]+@\d+): ", line))
    from gmr.configurator import Config
    assert got == _fit_keys(Config(model, "baby", {"synthetic": "tiny"})), got
    assert os.path.exists(tmp_path / "saved" / f"{model}-baby.pth")
