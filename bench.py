"""Benchmark: DiffMM on Amazon-baby-shaped synthetic data, train users/s (+ full-rank eval users/s).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N --steps K --warmup W

One "step" = one full DiffMM training epoch of the reference's DiffMMTrainer._train_epoch
(common/trainer.py:487-585): diffusion training of both denoisers over all users, the graph
rebuild (p_sample + top-1 + normalised UI graphs) and the BPR/contrastive phase over all train
interactions.  value = users/s = U * steps / wall (max over ranks); after the timed epochs
full-rank evaluation passes over the valid split are timed as eval users/s.
Multi-GPU (N > 1): user/batch-sharded data parallelism (gmr/dist.py) — each epoch still covers
the whole dataset once, split over the ranks (per-GPU batch = train_batch_size), with RCCL
all-reduces of the gradients and an all-gather of the rebuilt top-k edges.
"""
import argparse
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
MODELS = {"diffmm": "DiffMM", "genrecv1": "GenRecV1"}
DEFAULT_SHAPE = {"diffmm": "baby", "genrecv1": "tiktok"}
STEP_DESC = {"diffmm": "one DiffMMTrainer epoch (diffusion train + graph rebuild + BPR/contrastive)",
             "genrecv1": "one GenRecV1Trainer epoch (flip-diffusion train of the transformer denoiser + "
                         "graph rebuild with interest debiasing + BPR/contrastive)"}
HBM_PEAK_GBS = 8000.0
FP32_MFMA_PEAK_TFS = 157.3


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def setup(args):
    from gmr.configurator import Config
    from gmr.dataloader import EvalDataLoader, TrainDataLoader
    from gmr.quick_start import popularity_groups
    from gmr.synthetic import make_dataset
    from gmr.utils import get_model, get_trainer, init_seed

    name = MODELS[args.model]
    over = {"synthetic": args.shape, "save_recommended_topk": False, "epochs": 1}
    if args.scoring_dtype:
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
    log(f"setup {time.time() - t0:.1f}s: U={ds.user_num} I={ds.item_num} train={len(tr)} valid users={vl.pr_end}")
    return cfg, ds, tr, tl, vl, model, trainer


def pmc_traffic(model="diffmm", shape=None):
    """HBM bytes per launch per kernel class from the newest committed PMC summary of this workload
    (profiles/*_pmc_traffic.json for DiffMM at its default shape, *_pmc_traffic_<model>[_<shape>].json
    otherwise; made by scripts/pmc_traffic.sh on the same command).  Another workload's counters are
    never reused: traffic stays null without a summary of this one."""
    import glob
    default = shape in (None, DEFAULT_SHAPE.get(model))
    tag = model if default else f"{model}_{shape}"
    pat = "*_pmc_traffic.json" if tag == "diffmm" else f"*_pmc_traffic_{tag}.json"
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pat)))
    if not files:
        return {}, None
    with open(files[-1]) as f:
        return json.load(f), os.path.relpath(files[-1], ROOT)


def spmm_kernel_name():
    from gmr import kernels as K
    if K.SPMM_SEG_NNZ & K.SPMM_LANE_PLAN:
        return (f"spmm_lane_kernel (CSR, XCD column slices, lane group per row, L={K.SPMM_SEG_NNZ & 0xFFFF}; "
                "norm_adj on the packed lane plan)")
    return "spmm_seg_kernel (CSR, wave/segment)"


def summarize_probe(p, model="diffmm", shape=None):
    """Aggregate HIP-event timings per kernel class into roofline objects."""
    out = {}
    pmc, pmc_src = pmc_traffic(model, shape)
    for tag, recs in p.items():
        if not recs:
            continue
        ms = [s.elapsed_time(e) for s, e, _ in recs]
        tot_ms = float(np.sum(ms))
        if tag == "gemm":
            work = sum(2.0 * r[2][0] * r[2][1] * r[2][2] for r in recs)
            achieved = work / (tot_ms * 1e-3) / 1e12
            out[tag] = {"bound": "mfma", "achieved": round(achieved, 2), "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": round(achieved / FP32_MFMA_PEAK_TFS, 4), "traffic": None,
                        "launches": len(recs), "avg_us": round(1e3 * tot_ms / len(recs), 2),
                        "total_ms": round(tot_ms, 3), "algorithmic_per_launch": work / len(recs),
                        "kernel": "gemm_kernel (fp32 MFMA 32x32x2)"}
        else:
            # bytes = 8 nnz + 4 (n_rows+1) + 4 d n_cols (X once) + 4 d n_rows (Y once [+ read if beta])
            byts = 0.0
            for nnz, nr, nc, nb, has_beta in (r[2] for r in recs):
                d = 64 * nb
                byts += 8.0 * nnz + 4.0 * (nr + 1) + 4.0 * d * nc + 4.0 * d * nr * (2 if has_beta else 1)
            achieved = byts / (tot_ms * 1e-3) / 1e9
            out[tag] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "launches": len(recs),
                        "avg_us": round(1e3 * tot_ms / len(recs), 2), "total_ms": round(tot_ms, 3),
                        "algorithmic_per_launch": byts / len(recs), "kernel": spmm_kernel_name()}
    for tag, o in out.items():
        if tag in pmc:
            o["traffic"] = round(pmc[tag]["traffic_per_launch"])
            o["traffic_unit"] = "bytes/launch (memory side: 2 x FETCH_SIZE + WRITE_SIZE)"
            o["traffic_source"] = pmc_src
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


def cpu_baseline(model, tl, budget_s=30.0):
    """Oracle (torch-CPU restatement) timed on the host: one BPR step, one diffusion batch and one
    p_sample batch at the baby shape, extrapolated to a full epoch (train users/s)."""
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
    t0 = time.time()
    loss = model_ref.rec_loss(p, feats, adj, iadj, tadj, users, pos, neg)
    loss.backward()
    t_bpr = time.time() - t0
    den = model.denoise_model_image.slab
    w = {"emb_W": den.view("emb_W").cpu(), "emb_b": den.view("emb_b").cpu(), "W1": den.view("W1").cpu().contiguous(),
         "b1": den.view("b1").cpu(), "W2": den.view("W2").cpu().contiguous(), "b2": den.view("b2").cpu()}
    w = {k: v.clone().requires_grad_(True) for k, v in w.items()}
    tab = model_ref.diffmm_schedule()
    x0 = torch.zeros(B, I)
    for b in range(B):
        x0[b, tl.uitems_np[tl.uptr_np[b]:tl.uptr_np[b + 1]]] = 1.0
    ts = rng.integers(0, 5, B)
    t0 = time.time()
    diff, gc = model_ref.diffmm_training_losses(w, tab, x0, ts, torch.randn(B, I), (torch.rand(B, I) < 0.5).float(),
                                                p["iEmbeds"].detach(), torch.randn(I, 64))
    (diff.mean() + 0.5 * gc.mean()).backward()
    t_dif = 2 * (time.time() - t0)  # image + text denoisers
    t0 = time.time()
    with torch.no_grad():
        model_ref.diffmm_p_sample({k: v.detach() for k, v in w.items()}, tab, x0)
    t_ps = 2 * (time.time() - t0)
    n_bpr = -(-tl.n_inter // B)
    n_dif = -(-U // B)
    epoch = t_bpr * n_bpr + t_dif * n_dif + t_ps * n_dif
    return {"value": round(U / epoch, 2), "unit": "users/s", "cores": threads, "kind": "port",
            "sample": f"oracle (torch-CPU fp32 restatement): 1 BPR+contrastive step (B=2048, fwd+bwd) = {t_bpr:.2f}s, "
                      f"1 diffusion batch x2 denoisers = {t_dif:.2f}s, 1 p_sample batch x2 = {t_ps:.2f}s; "
                      f"extrapolated to {n_bpr} BPR + {n_dif} diffusion + {n_dif} p_sample batches = {epoch:.1f}s/epoch"}


def cpu_baseline_genrec(model, tl, trainer):
    """Oracle (oracle/genrec_ref.py, torch-CPU fp32) timed on the host: one BPR step, one diffusion
    batch (training_losses fwd+bwd incl. its p_sample) and one rebuild p_sample batch at the shape,
    extrapolated to a GenRecV1Trainer epoch (train users/s)."""
    from oracle import genrec_ref, graph_ref, model_ref
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    U, I, B = model.n_users, model.n_items, 2048
    N = U + I
    s = model.rec_slab
    p = {n: s.view(n).cpu().clone().requires_grad_(True) for n in model._pnames}
    p["user_embedding_weight"] = s.view("E0")[:U].cpu().clone().requires_grad_(True)
    p["item_id_embedding_weight"] = s.view("E0")[U:].cpu().clone().requires_grad_(True)
    feats = {"image": model.v_feat.cpu(), "text": model.t_feat.cpu()}
    rows = np.repeat(np.arange(U), np.diff(tl.uptr_np))
    rng = np.random.default_rng(0)
    sp = lambda c, n, m: model_ref.sparse_from_csr(*c, n, m)  # noqa: E731
    graphs = {"norm_adj": sp(graph_ref.norm_adj_csr(U, I, rows, tl.uitems_np), N, N),
              "R": sp(genrec_ref.user_item_csr(U, I, rows, tl.uitems_np), U, I)}
    ui = graph_ref.ui_adj_csr(U, I, np.repeat(np.arange(U), 10), rng.integers(0, I, 10 * U))
    graphs["ui_img"] = sp(genrec_ref.drop_edges_csr(*ui, rng.random(len(ui[1])) < 0.5), N, N)
    for key, f in (("ii_img", feats["image"]), ("ii_txt", feats["text"])):
        graphs[key] = sp(genrec_ref.knn_graph_csr(f.numpy(), 10)[0], I, I)
    state = {n: (torch.zeros(64), torch.ones(64)) for n in
             ["image_residual_project_1", "image_modal_project_1", "text_residual_project_1", "text_modal_project_1",
              "caculate_common_1", "gate_image_modal_1", "gate_text_modal_1"]}
    users = torch.as_tensor(rng.integers(0, U, B))
    pos, neg = torch.as_tensor(rng.integers(0, I, B)), torch.as_tensor(rng.integers(0, I, B))
    t0 = time.time()
    genrec_ref.calculate_loss(p, feats, graphs, state, users, pos, neg).backward()
    t_bpr = time.time() - t0
    den = model.denoise_model_image
    w = {n: den.v(n).cpu().clone().requires_grad_(True) for n in den.names}
    w["input_proj_weight"] = den.v("input_proj_weight").cpu().contiguous().clone().requires_grad_(True)
    x0 = torch.zeros(B, I)
    for b in range(B):
        x0[b, tl.uitems_np[tl.uptr_np[b]:tl.uptr_np[b + 1]]] = 1.0
    g, e = genrec_ref.flip_schedule(x0)
    ts = rng.integers(0, 5, B)
    flips = [(torch.rand(B, I) < 0.4).float().numpy() for _ in range(2)]
    draws = [(torch.rand(B, I) < 0.3).float().numpy() for _ in range(5)]
    t0 = time.time()
    total = genrec_ref.training_losses(w, x0, ts, flips[0], p["item_id_embedding_weight"].detach(), torch.randn(I, 64),
                                       flips[1], draws, g, e, den.L)[0]
    total.backward()
    t_dif = time.time() - t0
    t0 = time.time()
    with torch.no_grad():
        genrec_ref.p_sample({k: v.detach() for k, v in w.items()}, x0, g, e, flips[0], draws, den.L)
    t_ps = time.time() - t0
    n_bpr = -(-tl.n_inter // B)
    n_dif = -(-U // B)
    epoch = t_bpr * n_bpr + (t_dif + t_ps) * n_dif
    return {"value": round(U / epoch, 2), "unit": "users/s", "cores": threads, "kind": "port",
            "sample": f"oracle (torch-CPU fp32 restatement of GenRecV1): 1 BPR+InfoNCE step (B=2048, fwd+bwd) = "
                      f"{t_bpr:.2f}s, 1 diffusion batch (training_losses incl. its p_sample, fwd+bwd) = {t_dif:.2f}s, "
                      f"1 rebuild p_sample batch = {t_ps:.2f}s; extrapolated to {n_bpr} BPR + {n_dif} diffusion + "
                      f"{n_dif} rebuild batches = {epoch:.1f}s/epoch"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="diffmm", choices=sorted(MODELS))
    ap.add_argument("--shape", default=None, help="synthetic shape (default: baby for DiffMM, tiktok for GenRecV1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eval-passes", type=int, default=3)
    ap.add_argument("--no-probe", action="store_true", help="no HIP-event probes (A/B timing only)")
    ap.add_argument("--scoring-dtype", default=None, choices=["fp32", "fp16"],
                    help="GenRecV1 full-catalog scoring precision (config 5's fp16 MFMA scoring GEMM)")
    args = ap.parse_args()
    args.shape = args.shape or DEFAULT_SHAPE[args.model]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        backend = os.environ.get("GMR_DIST_BACKEND", "nccl")  # nccl == RCCL on ROCm; gloo only to rehearse
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    dist = world > 1

    def barrier():
        if dist:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if not dist:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return float(t.item())

    from gmr import kernels as K

    cfg, ds, tr, tl, vl, model, trainer = setup(args)
    U = model.n_users

    # warmup (the first warmup epoch is also probed to rank the kernel classes)
    probe_all = None
    graphs = getattr(trainer, "_use_graphs", False)
    for i in range(args.warmup):
        probed = i == args.warmup - 1 and not args.no_probe
        if probed:  # eager epoch: every launch individually timed
            trainer._use_graphs = False
            K.probe_begin(["gemm", "spmm"])
        t0 = time.time()
        trainer._train_epoch(tl, i)
        torch.cuda.synchronize()
        trainer._use_graphs = graphs
        if probed:
            raw = K.probe_end()
            probe_all = summarize_probe(raw, args.model, args.shape)
            if os.environ.get("GMR_PROBE_REPORT"):
                report_shapes(raw)
        log(f"warmup epoch {i}: {time.time() - t0:.3f}s")
    dominant = max(probe_all, key=lambda k: probe_all[k]["total_ms"]) if probe_all else "gemm"

    # timed epochs (live events around the dominant kernel class's launches; launches replayed
    # inside the BPR-step HIP graphs are not individually timed)
    if not args.no_probe:
        K.probe_begin([dominant], every=4)  # 1-in-4 sample: keeps the events' own cost out of the epoch time
    barrier()
    t0 = time.time()
    for i in range(args.steps):
        trainer._train_epoch(tl, args.warmup + i)
    barrier()
    dt = max_over_ranks(time.time() - t0)
    live = summarize_probe(K.probe_end(), args.model, args.shape) if not args.no_probe else {}
    train_ups = U * args.steps / dt

    # full-rank evaluation passes (valid split)
    trainer.evaluate(vl)
    barrier()
    t0 = time.time()
    for _ in range(args.eval_passes):
        res = trainer.evaluate(vl)
    barrier()
    et = max_over_ranks(time.time() - t0)
    eval_ups = vl.pr_end * args.eval_passes / et

    if rank == 0:
        roof = live.get(dominant) or (probe_all or {}).get(dominant)
        if roof is not None:
            roof["probe_scope"] = ("timed epochs, launches outside the BPR-step HIP graphs" if graphs and dominant in live
                                   else "timed epochs" if dominant in live else "last warmup epoch (eager)")
        line = {
            "metric": METRIC if args.model == "diffmm" else
            "train users/sec + full-rank eval users/sec, GenRecV1 TikTok-shaped (config 5)", "value": round(train_ups, 1), "unit": "users/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
            "data": f"synthetic ({args.shape} shape, SURVEY.md 8d recipe; random-init weights)",
            "config": {"workload": f"{MODELS[args.model]} {args.shape}-shaped synthetic: {U} users x {model.n_items} "
                                   f"items, {tl.n_inter} train interactions; step = {STEP_DESC[args.model]}",
                       "global_batch": cfg["train_batch_size"], "eval_batch": cfg["eval_batch_size"],
                       "parallelism": f"dp{world}"},
            "eval_users_per_s": round(eval_ups, 1), "eval_recall@20": res.get("recall@20"),
            "eval_scoring_dtype": getattr(model, "scoring_dtype", "fp32"),
            "roofline": roof, "roofline_by_kernel": probe_all, "dominant_kernel": dominant,
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = (cpu_baseline(model, tl) if args.model == "diffmm"
                                        else cpu_baseline_genrec(model, tl, trainer))
            except Exception as e:  # noqa: BLE001
                line["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(line), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
