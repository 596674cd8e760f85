"""Benchmark: DiffMM on Amazon-baby-shaped synthetic data, train users/s (+ full-rank eval users/s).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model diffmm|diffrec|genrecv1] [--no-legs]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N --steps K --warmup W

One "step" = one full training epoch of the model's reference trainer.  For DiffMM (the headline,
BASELINE.json) that is DiffMMTrainer._train_epoch (common/trainer.py:487-585): diffusion training
of both denoisers over all users, the graph rebuild (p_sample + top-1 + normalised UI graphs) and
the BPR/contrastive phase over all train interactions.  value = users/s = U * steps / wall (max
over ranks); after the timed epochs full-rank evaluation passes over the valid split are timed
as eval users/s.
Multi-GPU (N > 1): data parallelism over the ranks (gmr/dist.py) with the reference's global
batch: each train_batch_size batch is split over the ranks, RCCL all-reduces the gradients, the
rebuilt top-k edges are all-gathered; total work per epoch is fixed ("scaling": "strong").

Roofline: after the timed region one more epoch runs with the side streams off (GMR_SERIAL
semantics, gmr/kernels.py Streams.SERIAL) and every GEMM / SpMM / InfoNCE launch timed by HIP
events on its stream; per kernel class achieved = algorithmic work (SURVEY.md 8d formulas) /
summed duration.  `rocprofv3 --kernel-trace --stats` of `GMR_SERIAL=1 python bench.py` gives the
same per-kernel durations (profiles/).  Memory-side traffic and MFMA busy cycles come from
rocprofv3 --pmc passes (scripts/pmc_collect.sh) recorded with the SHA-256 of the library they
measured; a summary of another build is never used (traffic null then).

With no --model the default run adds two legs measured in the same process: DiffRec on the
baby shape (config 2: train epoch + 100-step p_sample eval) and GenRecV1 on the TikTok shape
with the fp16 MFMA scoring GEMM (config 5).
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "generative-multimodal-recommendation_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "train users/sec + full-rank eval users/sec, DiffMM Amazon-baby, 1/2/4/8 MI355X"
MODELS = {"diffmm": "DiffMM", "genrecv1": "GenRecV1", "diffrec": "DiffRec"}
DEFAULT_SHAPE = {"diffmm": "baby", "genrecv1": "tiktok", "diffrec": "baby"}
STEP_DESC = {"diffmm": "one DiffMMTrainer epoch (diffusion train + graph rebuild + BPR/contrastive)",
             "genrecv1": "one GenRecV1Trainer epoch (flip-diffusion train of the transformer denoiser + "
                         "graph rebuild with interest debiasing + BPR/contrastive)",
             "diffrec": "one Trainer epoch of DiffRec (training_losses + backward per interaction batch, "
                        "importance-sampled t)"}
HBM_PEAK_GBS = 8000.0
FP32_MFMA_PEAK_TFS = 157.3
# split-bf16 GEMM (gemm_x6_kernel): six v_mfma_f32_32x32x16_bf16 products per fp32 product, so its
# instruction roofline in fp32-equivalent flop/s is the dense bf16 MFMA peak (256 CUs x 4 SIMDs x
# 1,024 flop/clk x 2.4 GHz = 2,516.6 TF/s, MI355X_MICROARCH.md) / 6
X6_PEAK_TFS = round(2516.6 / 6, 1)
KERNEL_NAMES = {"gemm": "gemm_glds_kernel (fp32 MFMA v_mfma_f32_32x32x2_f32, global_load_lds staging, XCD-aware tiles)",
                "gemm_x6": "gemm_x6_kernel (fp32 operands split exactly into three bf16 terms on the "
                           "way into LDS, six "
                           "v_mfma_f32_32x32x16_bf16 products accumulated in fp32, hi*hi and the five small "
                           "products in separate accumulators: fp32-accurate, unbiased NT products)",
                "infonce": "cl6p_kernel rows + table passes (fused InfoNCE on the split-bf16 pipe: fp32 operands split "
                           "exactly into three bf16 terms; logits on six v_mfma_f32_32x32x16_bf16 products, the "
                           "gradient-only E T products on three; fp32 accumulation)",
                "infonce_f32": "cl_rows_kernel + cl_table_kernel (fused InfoNCE, fp32 MFMA)",
                "spmm": "spmm_side_kernel (bipartite side x 32-column slice per XCD, lane-group entry-stream tasks, "
                        "wave hub blocks combined in-launch) + spmm_lane_kernel for the non-bipartite graphs"}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def lib_sha256():
    from gmr import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def setup(args):
    from gmr.configurator import Config
    from gmr.dataloader import EvalDataLoader, TrainDataLoader
    from gmr.quick_start import popularity_groups
    from gmr.synthetic import make_dataset
    from gmr.utils import get_model, get_trainer, init_seed

    name = MODELS[args.model]
    over = {"synthetic": args.shape, "save_recommended_topk": False, "epochs": 1}
    if getattr(args, "scoring_dtype", None):
        if args.model != "genrecv1":
            raise SystemExit("--scoring-dtype applies to GenRecV1 (config 5)")
        over["scoring_dtype"] = args.scoring_dtype
    cfg = Config(name, "tiktok" if args.shape == "tiktok" else "baby", over)
    init_seed(999)
    t0 = time.time()
    ds = make_dataset(cfg, args.shape, seed=0)
    tr, va, te = ds.split()
    pop, warm, _, _ = popularity_groups(cfg, tr)
    cfg["pop_items"], cfg["warm_users"] = pop, warm
    tl = TrainDataLoader(cfg, tr, batch_size=cfg["train_batch_size"], shuffle=True)
    vl = EvalDataLoader(cfg, va, additional_dataset=tr, batch_size=cfg["eval_batch_size"])
    model = get_model(name)(cfg, tl)
    trainer = get_trainer(name)(cfg, model)
    torch.cuda.synchronize()
    log(f"setup {time.time() - t0:.1f}s: {name} U={ds.user_num} I={ds.item_num} train={len(tr)} "
        f"valid users={vl.pr_end}")
    return cfg, ds, tr, tl, vl, model, trainer


def pmc_summary(model="diffmm", shape=None):
    """Per-kernel-class memory-side bytes and MFMA busy cycles of this workload from the last (by name)
    profiles/*_pmc_<tag>.json made by scripts/pmc_collect.sh that was measured on the library now loaded
    (same SHA-256); none when no summary matches."""
    import glob
    tag = model if shape in (None, DEFAULT_SHAPE.get(model)) else f"{model}_{shape}"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{tag}.json")))
    if not files:
        return {}, None, "no PMC summary of this workload in profiles/"
    sha = lib_sha256()
    for fn in reversed(files):  # a summary measured on the loaded library, whatever its tag sorts as
        with open(fn) as f:
            d = json.load(f)
        if d.get("lib_sha256") == sha:
            return d, os.path.relpath(fn, ROOT), None
    src = os.path.relpath(files[-1], ROOT)
    return {}, src, f"no profiles/*_pmc_{tag}.json measured this build (lib_sha256 differs): not used"


def summarize_probe(p, model="diffmm", shape=None):
    """Aggregate HIP-event timings per kernel class into roofline objects."""
    out = {}
    pmc, pmc_src, pmc_why = pmc_summary(model, shape)
    for tag, recs in p.items():
        if not recs:
            continue
        ms = [s.elapsed_time(e) for s, e, _ in recs]
        tot_ms = float(np.sum(ms))
        if tag in ("gemm", "gemm_x6", "infonce"):
            if tag in ("gemm", "gemm_x6"):
                work = sum(2.0 * r[2][0] * r[2][1] * r[2][2] for r in recs)
                # operands read once + C written once (+ read for the in-place / aux epilogues)
                x_epi = (4, 5, 6, 8)  # POSTERIOR, DTANH, ROWSCALE_AUX, DRELU (include/gmr.h)
                alg_bytes = sum(4.0 * (M_ * K_ + K_ * N_ + M_ * N_ * (2 if ep in x_epi else 1))
                                for M_, N_, K_, _, _, ep in (r[2] for r in recs))
            else:  # rows pass S = P T^T and U = E T, table pass the same again: 4 B n 64 MACs
                work = sum(8.0 * r[2][0] * r[2][1] * 64 for r in recs)
            achieved = work / (tot_ms * 1e-3) / 1e12
            cl_x6 = tag == "infonce" and os.environ.get("GMR_CL_X6", "1") != "0"
            peak = X6_PEAK_TFS if tag == "gemm_x6" or cl_x6 else FP32_MFMA_PEAK_TFS
            out[tag] = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                        "frac": round(achieved / peak, 4), "traffic": None,
                        "launches": len(recs), "avg_us": round(1e3 * tot_ms / len(recs), 2),
                        "total_ms": round(tot_ms, 3), "algorithmic_per_launch": work / len(recs),
                        "algorithmic_unit": "flop",
                        "kernel": KERNEL_NAMES["infonce_f32" if tag == "infonce" and not cl_x6 else tag]}
            if tag in ("gemm", "gemm_x6"):
                out[tag]["algorithmic_bytes_per_launch"] = round(alg_bytes / len(recs))
            if tag == "gemm_x6" or cl_x6:
                out[tag]["peak_note"] = ("fp32-equivalent flop (2MNK) vs the split kernel's instruction roofline: "
                                         "dense bf16 MFMA peak 2516.6 TF/s / 6 products; "
                                         f"{achieved / FP32_MFMA_PEAK_TFS:.3f} of the fp32-input MFMA peak")
        else:
            # bytes = 8 nnz + 4 (n_rows+1) + 4 d n_cols (X once) + 4 d n_rows (Y once [+ read if beta])
            # (a multi-job launch, key ("jobs", job, ...), moves the sum of its jobs' bytes)
            byts = 0.0
            for key in (r[2] for r in recs):
                for nnz, nr, nc, nb, has_beta in (key[1:] if key[0] in ("jobs", "side_jobs") else (key,)):
                    d = 64 * nb
                    byts += 8.0 * nnz + 4.0 * (nr + 1) + 4.0 * d * nc + 4.0 * d * nr * (2 if has_beta else 1)
            achieved = byts / (tot_ms * 1e-3) / 1e9
            out[tag] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "launches": len(recs),
                        "avg_us": round(1e3 * tot_ms / len(recs), 2), "total_ms": round(tot_ms, 3),
                        "algorithmic_per_launch": byts / len(recs), "algorithmic_unit": "bytes",
                        "kernel": KERNEL_NAMES[tag]}
    for tag, o in out.items():
        c = pmc.get(tag) if pmc else None
        if c:
            o["traffic"] = round(c["traffic_per_launch"])
            o["traffic_unit"] = "bytes/launch (memory side: 2 x FETCH_SIZE + WRITE_SIZE)"
            alg_b = o.get("algorithmic_bytes_per_launch") or (o["algorithmic_per_launch"]
                                                            if o["algorithmic_unit"] == "bytes" else None)
            if alg_b:
                o["traffic_vs_algorithmic_bytes"] = round(c["traffic_per_launch"] / alg_b, 3)
            if c.get("mfma_util") is not None:
                o["mfma_util"] = round(c["mfma_util"], 4)
            o["pmc_source"] = pmc_src
        elif pmc_why:
            o["pmc_note"] = pmc_why
    return out


def report_shapes(p):
    """Per-shape breakdown of one probed epoch (GMR_PROBE_REPORT=1), to stderr."""
    for tag, recs in p.items():
        groups = {}
        for s_, e_, meta in recs:
            groups.setdefault(meta, []).append(s_.elapsed_time(e_))
        rows = sorted(groups.items(), key=lambda kv: -sum(kv[1]))
        log(f"--- {tag}: {len(recs)} launches, {sum(sum(v) for v in groups.values()):.2f} ms")
        for meta, ms in rows[:25]:
            tot = sum(ms)
            extra = ""
            if tag == "gemm":
                extra = f"{2.0 * meta[0] * meta[1] * meta[2] * len(ms) / (tot * 1e-3) / 1e12:7.1f} TF/s"
            log(f"  {str(meta):44s} n={len(ms):4d} total={tot:8.2f} ms avg={1e3 * tot / len(ms):8.1f} us {extra}")


def _median_time(fn, reps):
    fn()  # warm (allocator, MKL/oneDNN kernels)
    ts = []
    for _ in range(reps):
        t0 = time.time()
        fn()
        ts.append(time.time() - t0)
    return float(np.median(ts)), ts


def cpu_baseline(model, tl, reps=3):
    """Oracle (torch-CPU restatement) timed on the host: one BPR step, one diffusion batch and one
    p_sample batch at the baby shape, each the median of `reps` timed runs after a warm run,
    extrapolated to a full epoch (train users/s)."""
    from oracle import graph_ref, model_ref
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    U, I, B = model.n_users, model.n_items, 2048
    N = U + I
    s = model.rec_slab
    p = {"uEmbeds": s.view("E0")[:U].cpu().clone().requires_grad_(True),
         "iEmbeds": s.view("E0")[U:].cpu().clone().requires_grad_(True),
         "image_trans": s.view("image_trans").cpu().clone().requires_grad_(True),
         "text_trans": s.view("text_trans").cpu().clone().requires_grad_(True),
         "modal_weight": s.view("modal_weight").cpu().clone().requires_grad_(True)}
    feats = {"v": model.v_feat.cpu(), "t": model.t_feat.cpu()}
    rows = np.repeat(np.arange(U), np.diff(tl.uptr_np))
    adj = model_ref.sparse_from_csr(*graph_ref.norm_adj_csr(U, I, rows, tl.uitems_np), N)
    rng = np.random.default_rng(0)
    iadj = model_ref.sparse_from_csr(*graph_ref.ui_adj_csr(U, I, np.arange(U), rng.integers(0, I, U)), N)
    tadj = model_ref.sparse_from_csr(*graph_ref.ui_adj_csr(U, I, np.arange(U), rng.integers(0, I, U)), N)
    users = torch.as_tensor(rng.integers(0, U, B))
    pos = torch.as_tensor(rng.integers(0, I, B))
    neg = torch.as_tensor(rng.integers(0, I, B))

    def bpr():
        for v in p.values():
            v.grad = None
        model_ref.rec_loss(p, feats, adj, iadj, tadj, users, pos, neg).backward()
    t_bpr, s_bpr = _median_time(bpr, reps)
    den = model.denoise_model_image.slab
    w = {"emb_W": den.view("emb_W").cpu(), "emb_b": den.view("emb_b").cpu(), "W1": den.view("W1").cpu().contiguous(),
         "b1": den.view("b1").cpu(), "W2": den.view("W2").cpu().contiguous(), "b2": den.view("b2").cpu()}
    w = {k: v.clone().requires_grad_(True) for k, v in w.items()}
    tab = model_ref.diffmm_schedule()
    x0 = torch.zeros(B, I)
    for b in range(B):
        x0[b, tl.uitems_np[tl.uptr_np[b]:tl.uptr_np[b + 1]]] = 1.0
    ts = rng.integers(0, 5, B)
    noise, keep, gfe = torch.randn(B, I), (torch.rand(B, I) < 0.5).float(), torch.randn(I, 64)

    def dif():
        for v in w.values():
            v.grad = None
        diff, gc = model_ref.diffmm_training_losses(w, tab, x0, ts, noise, keep, p["iEmbeds"].detach(), gfe)
        (diff.mean() + 0.5 * gc.mean()).backward()
    t_dif1, s_dif = _median_time(dif, reps)
    t_dif = 2 * t_dif1  # image + text denoisers

    def ps():
        with torch.no_grad():
            model_ref.diffmm_p_sample({k: v.detach() for k, v in w.items()}, tab, x0)
    t_ps1, s_ps = _median_time(ps, reps)
    t_ps = 2 * t_ps1
    n_bpr = -(-tl.n_inter // B)
    n_dif = -(-U // B)
    epoch = t_bpr * n_bpr + t_dif * n_dif + t_ps * n_dif
    fmt = lambda xs: "/".join(f"{x:.2f}" for x in xs)  # noqa: E731
    # cores = the torch intra-op threads the port ran on (capped at 16: the GPU box's CPU share per job,
    # whatever os.cpu_count() reports there); host_cpus = what the host reports
    return {"value": round(U / epoch, 2), "unit": "users/s", "cores": threads, "host_cpus": os.cpu_count(),
            "kind": "port",
            "sample": f"oracle (torch-CPU fp32 restatement), median of {reps} timed runs after a warm run: "
                      f"1 BPR+contrastive step (B=2048, fwd+bwd) = {t_bpr:.2f}s ({fmt(s_bpr)}), "
                      f"1 diffusion batch x2 denoisers = {t_dif:.2f}s ({fmt(s_dif)} per denoiser), "
                      f"1 p_sample batch x2 = {t_ps:.2f}s ({fmt(s_ps)} per denoiser); extrapolated to {n_bpr} BPR + "
                      f"{n_dif} diffusion + {n_dif} p_sample batches = {epoch:.1f}s/epoch"}


def run_workload(args, dist_on, barrier, max_over_ranks, with_cpu_baseline):
    """Setup, warmup, timed epochs, eval passes and the serial roofline epoch of one model."""
    from gmr import kernels as K
    cfg, ds, tr, tl, vl, model, trainer = setup(args)
    U = model.n_users
    for i in range(args.warmup):
        t0 = time.time()
        trainer._train_epoch(tl, i)
        torch.cuda.synchronize()
        log(f"warmup epoch {i}: {time.time() - t0:.3f}s")
    barrier()
    t0 = time.time()
    for i in range(args.steps):
        trainer._train_epoch(tl, args.warmup + i)
        if getattr(trainer, "phase_ms", None):
            log("phases [ms]: diffusion %.2f, rebuild %.2f, bpr %.2f" % trainer.phase_ms)
    barrier()
    dt = max_over_ranks(time.time() - t0)
    train_ups = U * args.steps / dt

    trainer.evaluate(vl)
    barrier()
    t0 = time.time()
    for _ in range(args.eval_passes):
        res = trainer.evaluate(vl)
    barrier()
    et = max_over_ranks(time.time() - t0)
    eval_ups = vl.pr_end * args.eval_passes / et

    roof = None
    if not args.no_probe:
        # one more epoch, side streams off, every GEMM / SpMM / InfoNCE launch timed on its stream
        serial = K.Streams.SERIAL
        K.Streams.SERIAL = True
        K.probe_begin(["gemm", "gemm_x6", "spmm", "infonce"])
        t1 = time.time()
        trainer._train_epoch(tl, args.warmup + args.steps)
        torch.cuda.synchronize()
        serial_ms = 1e3 * (time.time() - t1)
        raw = K.probe_end()
        K.Streams.SERIAL = serial
        roof = summarize_probe(raw, args.model, args.shape)
        if os.environ.get("GMR_PROBE_REPORT"):
            report_shapes(raw)
        mfma_flop = sum(o["algorithmic_per_launch"] * o["launches"] for o in roof.values() if o["bound"] == "mfma")
        if os.environ.get("GMR_GEMM_X6", "1") != "0" and "gemm_x6" not in roof and args.model == "diffmm":
            log("note: no split-bf16 GEMM launch in the probed epoch")
        for o in roof.values():
            o["probe_scope"] = ("one extra epoch after the timed region with the side streams off (GMR_SERIAL): "
                                "HIP events around every launch of the class on its stream (a GEMM call: its "
                                "k-contiguous operand copies, the kernel and the split-K reduce)")
        roof["_epoch"] = {"mfma_flop_per_epoch": mfma_flop, "serial_epoch_ms": round(serial_ms, 2),
                          "epoch_mfma_frac": round(mfma_flop / (dt / args.steps) / 1e12 / FP32_MFMA_PEAK_TFS, 4),
                          "note": "algorithmic GEMM + InfoNCE flop of one epoch / timed ms_per_step / fp32 MFMA peak"}
    out = {"model": MODELS[args.model], "shape": args.shape, "U": U, "I": model.n_items, "n_inter": tl.n_inter,
           "train_users_per_s": round(train_ups, 1), "ms_per_step": round(1e3 * dt / args.steps, 2),
           "eval_users_per_s": round(eval_ups, 1), "eval_recall@20": res.get("recall@20"),
           "eval_scoring_dtype": getattr(model, "scoring_dtype", "fp32"), "roofline_by_kernel": roof,
           "global_batch": cfg["train_batch_size"], "eval_batch": cfg["eval_batch_size"]}
    if with_cpu_baseline and args.model == "diffmm":
        try:
            out["cpu_baseline"] = cpu_baseline(model, tl)
        except Exception as e:  # noqa: BLE001
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    del trainer, model
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def dominant(roof):
    if not roof:
        return None, None
    cls = {k: v for k, v in roof.items() if not k.startswith("_")}
    name = max(cls, key=lambda k: cls[k]["total_ms"])
    return name, cls[name]


def launch_ranks(n):
    """Run this script under torch.distributed.run with n ranks (one per GPU, RCCL over xGMI) as a
    child process; its stdout (rank 0's JSON line) is relayed; the exit code is the launcher's."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log("launching: " + " ".join(cmd))
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if lines:
        print(lines[-1], flush=True)
    if r.returncode != 0 or not lines:
        log(f"distributed bench failed (exit {r.returncode}); stdout tail: {r.stdout[-2000:]}")
        return r.returncode or 1
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default=None, choices=sorted(MODELS), help="default: DiffMM headline + legs")
    ap.add_argument("--shape", default=None, help="synthetic shape (default: baby; tiktok for GenRecV1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-legs", action="store_true", help="headline only (no DiffRec / GenRecV1 legs)")
    ap.add_argument("--eval-passes", type=int, default=3)
    ap.add_argument("--no-probe", action="store_true", help="no serial roofline epoch (A/B timing only)")
    ap.add_argument("--no-dp-local", action="store_true", help="N > 1: skip the GMR_DP_MODE=local measurement")
    ap.add_argument("--scoring-dtype", default=None, choices=["fp32", "fp16"],
                    help="GenRecV1 full-catalog scoring precision (config 5's fp16 MFMA scoring GEMM)")
    args = ap.parse_args()
    # the DiffRec / GenRecV1 legs at N = 1 only: under data parallelism an exception in one rank's leg would leave
    # the others waiting in a collective, and the scaling line is the DiffMM headline's
    legs = args.model is None and not args.no_legs and int(os.environ.get("WORLD_SIZE", "1")) == 1
    args.model = args.model or "diffmm"
    args.shape = args.shape or DEFAULT_SHAPE[args.model]

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without a launcher: start the N ranks as a child process group
        # (before anything here touches the GPU) and relay rank 0's JSON line
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; n_gpus reports WORLD_SIZE")
    if world > 1:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        backend = os.environ.get("GMR_DIST_BACKEND", "nccl")  # nccl == RCCL on ROCm; gloo only to rehearse
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    dist_on = world > 1

    def barrier():
        if dist_on:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if not dist_on:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return float(t.item())

    head = run_workload(args, dist_on, barrier, max_over_ranks, world == 1 and not args.no_cpu_baseline)
    # N > 1: the headline keeps the reference's global batch (each 2,048-row batch split over the
    # GPUs); the opt-in GMR_DP_MODE=local schedule (each GPU takes whole batches: world x 2,048 rows
    # per optimiser step, 1 / world of the steps) is measured beside it under its own key
    dp_local = None
    if dist_on and not args.no_dp_local and os.environ.get("GMR_DP_MODE", "global") != "local":
        os.environ["GMR_DP_MODE"] = "local"
        try:
            a3 = argparse.Namespace(**vars(args))
            a3.no_probe = True
            r = run_workload(a3, dist_on, barrier, max_over_ranks, False)
            dp_local = {"value": r["train_users_per_s"], "unit": "users/s", "ms_per_step": r["ms_per_step"],
                        "global_batch": world * r["global_batch"], "eval_users_per_s": r["eval_users_per_s"],
                        "eval_recall@20": r["eval_recall@20"],
                        "note": "GMR_DP_MODE=local: each GPU takes whole train_batch_size batches (world x "
                                "train_batch_size rows per optimiser step, 1/world of the reference's steps per "
                                "epoch); a different schedule from the reference's, not the headline value"}
        except Exception as e:  # noqa: BLE001
            dp_local = {"error": repr(e)}
        finally:
            os.environ.pop("GMR_DP_MODE", None)
    # the same headline epoch with every GEMM on the fp32-input MFMA (GMR_GEMM_X6=0, read once by the
    # library, so a child process), reported beside the value for comparison
    fp32_only = None
    if legs and world == 1 and os.environ.get("GMR_GEMM_X6", "1") != "0":
        import subprocess
        env = dict(os.environ, GMR_GEMM_X6="0")
        cmd = [sys.executable, os.path.abspath(__file__), "--model", "diffmm", "--no-legs", "--no-cpu-baseline",
               "--no-probe", "--steps", str(args.steps), "--warmup", str(args.warmup), "--eval-passes", "1"]
        try:
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            j = json.loads(r.stdout.strip().splitlines()[-1])
            fp32_only = {"value": j["value"], "unit": "users/s", "ms_per_step": j["ms_per_step"],
                         "eval_recall@20": j["eval_recall@20"], "note": "same epoch, GMR_GEMM_X6=0 (child process)"}
        except Exception as e:  # noqa: BLE001
            fp32_only = {"error": repr(e)}
    leg_out = {}
    if legs:
        for key, m, shape, sd in (("diffrec", "diffrec", "baby", None), ("genrecv1_fp16", "genrecv1", "tiktok", "fp16")):
            a2 = argparse.Namespace(**vars(args))
            a2.model, a2.shape, a2.scoring_dtype, a2.steps, a2.warmup = m, shape, sd, max(2, args.steps), 1
            try:
                r = run_workload(a2, dist_on, barrier, max_over_ranks, False)
                dn, dobj = dominant(r.get("roofline_by_kernel"))
                r["roofline"], r["dominant_kernel"] = dobj, dn
                r["step"] = STEP_DESC[m]
                leg_out[key] = r
            except Exception as e:  # noqa: BLE001  (a failing leg must not cost the headline line)
                leg_out[key] = {"error": repr(e)}

    if rank == 0:
        roof = head.pop("roofline_by_kernel")
        dn, dobj = dominant(roof)
        line = {
            "metric": METRIC if args.model == "diffmm" else
            f"train users/sec + full-rank eval users/sec, {MODELS[args.model]} {args.shape}-shaped",
            "value": head["train_users_per_s"], "unit": "users/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
            "data": f"synthetic ({args.shape} shape, SURVEY.md 8d recipe; random-init weights)",
            "config": {"workload": f"{head['model']} {args.shape}-shaped synthetic: {head['U']} users x {head['I']} "
                                   f"items, {head['n_inter']} train interactions; step = {STEP_DESC[args.model]}",
                       "global_batch": head["global_batch"], "eval_batch": head["eval_batch"],
                       "parallelism": f"dp{world}"},
            "eval_users_per_s": head["eval_users_per_s"], "eval_recall@20": head["eval_recall@20"],
            "eval_scoring_dtype": head["eval_scoring_dtype"],
            "roofline": dobj, "dominant_kernel": dn, "roofline_by_kernel": roof,
            "lib_sha256": lib_sha256(),
        }
        line["gemm_arith"] = (
            "fp32 operands and results; NT products (denoiser forward, p_sample) on the split-bf16 kernel: each fp32 "
            "operand split exactly into three bf16 terms, six bf16 MFMA products accumulated in fp32 (error vs fp64 "
            "within the fp32-input MFMA kernel's, tests/test_kernels_gpu.py::test_gemm_x6_fp32_accuracy); the other "
            "products on the fp32-input MFMA" if os.environ.get("GMR_GEMM_X6", "1") != "0" else
            "every product on the fp32-input MFMA (GMR_GEMM_X6=0)")
        if fp32_only:
            line["fp32_mfma_only"] = fp32_only
        if "cpu_baseline" in head:
            line["cpu_baseline"] = head["cpu_baseline"]
        if leg_out:
            line["legs"] = leg_out
        if dp_local:
            line["dp_local_batch"] = dp_local
        print(json.dumps(line), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
