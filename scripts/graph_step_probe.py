"""Per-step cost of the DiffMM BPR step: eager issue vs hipGraphLaunch vs the native executor (K.GraphExec).

python scripts/graph_step_probe.py [--steps 50]

After one warm epoch (UI graphs built, every kernel loaded) the same list of full-size batches is run
four ways (the executor on the model's side streams and on two of its own), each timed with HIP events on
the current stream over --steps steps (inputs copied into the static buffers for the graphed forms, as the
Trainer does), and the capture itself (wall time, incl.
executor creation / instantiate) is reported separately.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from gmr import kernels as K  # noqa: E402
from gmr.trainer import capture_graph  # noqa: E402


def timed(fn, batches):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for b in batches:
        fn(b)
    e1.record()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / len(batches), 1e3 * th / len(batches)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    args = argparse.Namespace(model="diffmm", shape="baby", scoring_dtype=None)
    cfg, ds, tr, tl, vl, model, trainer = bench.setup(args)
    trainer._train_epoch(tl, 0)
    torch.cuda.synchronize()
    d = tl.epoch()
    full = [b[2:] for b in tl.batches(d) if b[2].numel() == tl.batch_size][:a.steps]
    print(f"{len(full)} full-size batches", flush=True)

    def eager(b):
        model.rec_step(*b)

    static = [t.clone() for t in full[0]]
    model.rec_step(*static)
    torch.cuda.synchronize()
    t = time.perf_counter()
    g = capture_graph(lambda: model.rec_step(*static), keep_graph=True)
    t_cap = time.perf_counter() - t
    t = time.perf_counter()
    ex = K.GraphExec(g, side=model._streams)
    ex_own = K.GraphExec(g, n_side=2)
    t_ex = time.perf_counter() - t
    t = time.perf_counter()
    g.instantiate()
    torch.cuda.synchronize()
    t_inst = time.perf_counter() - t
    print(f"capture {1e3 * t_cap:.2f} ms, executor create {1e3 * t_ex:.2f} ms, instantiate {1e3 * t_inst:.2f} ms, "
          f"executor {ex.info()}", flush=True)

    def load(b):
        for dst, src in zip(static, b):
            dst.copy_(src)

    def replay(b):
        load(b)
        g.replay()

    def execute(b):
        load(b)
        ex.launch()

    def execute_own(b):
        load(b)
        ex_own.launch()

    hi = torch.cuda.Stream(priority=-1)

    def eager_main_high(b):
        hi.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(hi):
            model.rec_step(*b)
        torch.cuda.current_stream().wait_stream(hi)

    ex_serial = K.GraphExec(g, n_side=0)

    def execute_serial(b):
        load(b)
        ex_serial.launch()

    def copies_only(b):
        load(b)

    for rep in range(3):
        for name, fn in (("eager", eager), ("eager-hi", eager_main_high), ("graph", replay), ("executor", execute),
                         ("exec-own", execute_own), ("exec-1str", execute_serial), ("copies", copies_only)):
            gpu, host = timed(fn, full)
            print(f"rep {rep} {name:9s} GPU {gpu:.3f} ms/step, host issue {host:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
