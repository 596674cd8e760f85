"""Trainers — mirror common/trainer.py of the reference (Trainer :58-408, DiffMMTrainer :410-585).

Same epoch structure, log lines, early stopping, checkpointing and return values as the
reference; the per-step work runs through the fused HIP paths of the models:
  * BPR phase: device-sampled epoch, one fused forward+backward per batch, flat-slab Adam;
    the epoch loss is accumulated on the device and read once per epoch (the reference syncs
    on loss.item() every batch; its NaN check therefore happens at epoch end here);
  * DiffMM diffusion phase + graph rebuild: fused denoiser steps and device p_sample/top-k/CSR;
  * evaluation: forward once per pass, then per eval batch score -> mask -> top-K on the device
    and Recall/NDCG/Precision/MAP sums on the device.
"""
import itertools
import os
from logging import getLogger
from time import time

import numpy as np
import torch

from . import _lib
from . import dist
from . import kernels as K
from .kernels import ptr, stream
from .slab import FlatAdam
from .tape import Tape
from .topk_evaluator import TopKEvaluator
from .utils import dict2str, early_stopping

# full-rank eval through the fused score -> mask -> top-k kernel (gmr_score_topk_f32); GMR_EVAL_FUSED=0
# keeps the score GEMM + mask + radix top-k over an E x I buffer (A/B)
FUSED_EVAL = os.environ.get("GMR_EVAL_FUSED", "1") != "0"
# DiffMM diffusion phase, one process: each denoiser's chain of steps and Adam updates runs on its own stream
# with one join after the phase (GMR_INDEP_DENOISERS=0: join after every step, Adam on the main stream).
# Diffusion phase 22.6 -> 22.0-22.8 ms, epoch 68.3 -> 67.9 ms averaged over three pairs (within the box's
# noise; profiles/r05ze_indep_denoisers_ab.txt)
INDEP_DENOISERS = os.environ.get("GMR_INDEP_DENOISERS", "1") != "0"
# one process, full-size BPR batches of models whose rec step is a fixed call sequence (DiffMM: `tape_safe`): the
# step's C-ABI calls are recorded once per epoch (per graph rebuild) and replayed without the Python layer
# (gmr/tape.py); GMR_TAPE=0 issues every step through Python
TAPE = os.environ.get("GMR_TAPE", "1") != "0"


_CAPTURE = {}


def capture_graph(body, keep_graph=False):
    """Capture body()'s launches into a torch.cuda.CUDAGraph on a side capture stream (the graph's own private
    memory pool).  torch.cuda.graph() would also empty the allocator's cache on every
    capture (each rebuilt epoch recaptures), so every later allocation of the epoch would go back to
    hipMalloc; this does only what capture needs: the capture stream waits for the current one, and the
    current one for the capture."""
    dev = torch.cuda.current_device()
    if dev not in _CAPTURE:
        _CAPTURE[dev] = torch.cuda.Stream()
    cs = _CAPTURE[dev]
    g = torch.cuda.CUDAGraph(keep_graph=keep_graph)
    cur = torch.cuda.current_stream()
    cs.wait_stream(cur)
    with torch.cuda.stream(cs):
        g.capture_begin()
        try:
            body()
        finally:
            g.capture_end()
    cur.wait_stream(cs)
    return g


def reduce_slab_grads(model, slabs):
    """SUM all-reduce of the gradient slabs after one data-parallel step.  A model may have started
    the first `early_reduce_cut(slab)` words itself inside rec_step (DiffMM: E0, overlapped with its
    last GEMMs); then only the rest is reduced here and the early one is waited for.  A rank that ran
    no rec_step (idle in a short last batch) issues the same two reduces, so collectives match."""
    if not dist.is_dist():
        return
    early = model.take_early_reduce() if hasattr(model, "take_early_reduce") else None
    for s_ in slabs:
        cut = model.early_reduce_cut(s_) if hasattr(model, "early_reduce_cut") else None
        if cut is None:
            dist.all_reduce_(s_.grad)
        else:
            if early is None:
                dist.all_reduce_(s_.grad[:cut])
            dist.all_reduce_(s_.grad[cut:])
    dist.wait(early)


class Trainer:
    def __init__(self, config, model, mg=False):
        self.config = config
        self.model = model
        self.logger = getLogger()
        self.learner = config["learner"]
        self.learning_rate = config["learning_rate"]
        self.epochs = config["epochs"]
        self.eval_step = min(config["eval_step"], self.epochs)
        self.stopping_step = config["stopping_step"]
        self.clip_grad_norm = config["clip_grad_norm"]
        if self.clip_grad_norm:
            raise NotImplementedError("clip_grad_norm is unset in the hot-path configs")
        self.valid_metric = config["valid_metric"].lower()
        self.valid_metric_bigger = config["valid_metric_bigger"]
        self.test_batch_size = config["eval_batch_size"]
        self.device = config["device"]
        wd = config["weight_decay"]
        self.weight_decay = (eval(wd) if isinstance(wd, str) else wd) if wd is not None else 0.0
        self.req_training = config["req_training"]
        self.start_epoch = 0
        self.cur_step = 0
        zero = {f"{j.lower()}@{k}": 0.0 for j, k in itertools.product(config["metrics"], config["topk"])}
        self.best_valid_score = -1
        self.best_valid_result = zero
        self.best_test_upon_valid = zero
        self.train_loss_dict = {}
        self.optimizer = self._build_optimizer()
        sched = config["learning_rate_scheduler"] or [1.0, 50]
        self.lr_factor = lambda e: sched[0] ** (e / sched[1])
        self._sched_epoch = 0
        self.evaluator = TopKEvaluator(config)
        self.mg = mg
        self._loss_acc = torch.zeros(2, dtype=torch.float32, device=self.device)
        # GMR_GRAPHS=1: full-size BPR steps of models that expose graph_key() (DiffMM) replay a HIP
        # graph of the whole rec step, side streams included (torch.cuda.CUDAGraph; captured on the
        # first step and again when the model's device graphs change, i.e. after each rebuild).
        # Off by default: measured slower in the epoch (104-106 vs 95-97 ms, profiles/r04g_graphs_ab.txt;
        # the replay appears to lose the three-stream overlap of the eager step).
        self._use_graphs = os.environ.get("GMR_GRAPHS", "0") == "1" and hasattr(model, "graph_key")
        self._graph = None
        self._use_tape = TAPE and getattr(model, "tape_safe", False)
        self._tape = None
        self.fused_eval = FUSED_EVAL  # per trainer, so a test can run both eval paths in one process

    def _build_optimizer(self):
        if (self.learner or "adam").lower() != "adam":
            raise NotImplementedError(f"learner {self.learner}: the hot-path configs use adam")
        return FlatAdam(self.model.optim_slabs(), lr=self.learning_rate, weight_decay=self.weight_decay)

    # ------------------------------------------------------------------ training
    def _train_epoch(self, train_data, epoch_idx, loss_func=None):
        if not self.req_training:
            return 0.0, []
        self.model.train()
        d = train_data.epoch()
        acc = self._loss_acc
        K.zero_(acc)
        W = dist.world()
        slabs = self.model.optim_slabs()
        if W > 1 and hasattr(self.model, "dp_early_reduce"):
            self.model.dp_early_reduce = True  # reduce_slab_grads below takes the handle every step
        hook = getattr(self.model, "dp_step_end", None)  # per-global-step model state sync (DiffRec)
        # one optimiser step per train_batch_size batch, as the reference (trainer.py:144-208);
        # under data parallelism every batch is split over the ranks
        for b, rank_rows, u, p, ng, pb, pc in train_data.batches(d):
            norm, share = dist.dp_scales(rank_rows)
            if u.numel() > 0:
                if self._use_graphs and W == 1 and u.numel() == train_data.batch_size:
                    self._graphed_step(u, p, ng, pb, pc, norm, share, acc)
                elif self._use_tape and W == 1 and u.numel() == train_data.batch_size and K._probe is None:
                    self._taped_step(u, p, ng, pb, pc, norm, share, acc)
                elif W > 1 and getattr(self.model, "rec_step_takes_batch", False):
                    # in-batch terms see the whole global step (GenRecV1's B x B InfoNCE keys)
                    loss = self.model.rec_step(u, p, ng, pb, pc, norm_rows=norm, reg_share=share,
                                               gbatch=train_data.step_rows(d, b))
                    _lib.call("gmr_sum_f32", 1, ptr(loss.view(1)), 1.0, ptr(acc), 1, stream())
                elif getattr(self.model, "rec_step_takes_acc", False):  # the step adds its loss to acc itself
                    self.model.rec_step(u, p, ng, pb, pc, norm_rows=norm, reg_share=share, acc=acc)
                else:
                    loss = self._rec_step(u, p, ng, pb, pc, norm, share, sum(rank_rows[:dist.rank()]))
                    _lib.call("gmr_sum_f32", 1, ptr(loss.view(1)), 1.0, ptr(acc), 1, stream())
            else:
                for s_ in slabs:
                    s_.zero_grad()
            if W > 1:
                reduce_slab_grads(self.model, slabs)
            if hook is not None:
                hook()
            self.optimizer.step()
        dist.all_reduce_(acc)
        total = float(acc[0].item())
        fb = train_data.fallbacks() if hasattr(train_data, "fallbacks") else 0
        if fb:
            self.logger.warning(f"epoch {epoch_idx}: {fb} BPR rows kept a negative from the user's history "
                                f"(no true negative in 4096 draws)")
        if np.isnan(total):
            self.logger.info("Loss is nan at epoch: {}. Exiting.".format(epoch_idx))
            return torch.tensor(float("nan")), []
        return total, []

    def _rec_step(self, u, p, ng, pb, pc, norm, share, row0):
        if getattr(self.model, "rec_step_takes_row0", False):
            return self.model.rec_step(u, p, ng, pb, pc, norm_rows=norm, reg_share=share, row0=row0)
        return self.model.rec_step(u, p, ng, pb, pc, norm_rows=norm, reg_share=share)

    def _taped_step(self, u, p, ng, pb, pc, norm, share, acc):
        """One full-size BPR step replayed from a host tape (gmr/tape.py): the eager step's calls, streams and
        order, without the Python layer.  Recorded on the first step after the model's device graphs, the
        batch shape, the current stream or the stream probes change (the recording step runs eagerly)."""
        m = self.model
        key = (u.numel(), norm, share, m.graph_key(), stream().value, K.Streams.SERIAL, K.Streams.PERTURB)
        inputs = (u, p, ng, pb, pc)
        if self._tape is None or self._tape[0] != key:
            self._tape = None
            t = Tape(inputs)
            with t.recording():
                if getattr(m, "rec_step_takes_acc", False):
                    m.rec_step(u, p, ng, pb, pc, norm_rows=norm, reg_share=share, acc=acc)
                else:
                    loss = m.rec_step(u, p, ng, pb, pc, norm_rows=norm, reg_share=share)
                    _lib.call("gmr_sum_f32", 1, ptr(loss.view(1)), 1.0, ptr(acc), 1, stream())
            self._tape = (key, t)
            return
        self._tape[1].replay(inputs)
        m.tape_replayed()

    def _graphed_step(self, u, p, ng, pb, pc, norm, share, acc):
        """One full-size BPR step replayed from a HIP graph (torch.cuda.CUDAGraph over the fused
        step's ~75 launches), removing the per-launch host cost.  The graph is captured on first
        use and again whenever the model's device graphs (the rebuilt UI adjacencies) or the
        data-parallel scales change; batch inputs are copied into its static buffers."""
        key = (u.numel(), norm, share, self.model.graph_key() if hasattr(self.model, "graph_key") else None)
        if self._graph is None or self._graph[0] != key:
            self._graph = None
            static = [t.clone() for t in (u, p, ng, pb, pc)]

            def body():
                loss = self.model.rec_step(*static, norm_rows=norm, reg_share=share)
                _lib.call("gmr_sum_f32", 1, ptr(loss.view(1)), 1.0, ptr(acc), 1, stream())
            g = capture_graph(body)
            self._graph = (key, g, static)
        _, g, static = self._graph
        for dst, src in zip(static, (u, p, ng, pb, pc)):
            dst.copy_(src)
        g.replay()

    def _generate_train_loss_output(self, epoch_idx, s_time, e_time, losses):
        out = "epoch %d training [time: %.2fs, " % (epoch_idx, e_time - s_time)
        if isinstance(losses, tuple):
            out = ", ".join("train_loss%d: %.4f" % (i + 1, l) for i, l in enumerate(losses))
        else:
            out += "train loss: %.4f" % losses
        return out + "]"

    def _valid_epoch(self, valid_data, is_test=False):
        res = self.evaluate(valid_data, is_test=is_test)
        score = res[self.valid_metric] if self.valid_metric else res["NDCG@20"]
        return score, res

    def fit(self, train_data, valid_data=None, test_data=None, saved=False, verbose=True):
        self._train_data = train_data
        for epoch_idx in range(self.start_epoch, self.epochs):
            t0 = time()
            self.model.pre_epoch_processing()
            train_loss, _ = self._train_epoch(train_data, epoch_idx)
            if torch.is_tensor(train_loss):
                break
            self._sched_epoch += 1
            self.optimizer.set_lr_factor(self.lr_factor(self._sched_epoch))
            self.train_loss_dict[epoch_idx] = sum(train_loss) if isinstance(train_loss, tuple) else train_loss
            t1 = time()
            msg = self._generate_train_loss_output(epoch_idx, t0, t1, train_loss)
            post = self.model.post_epoch_processing()
            if verbose:
                self.logger.info(msg)
                if post is not None:
                    self.logger.info(post)
            if (epoch_idx + 1) % self.eval_step == 0:
                v0 = time()
                valid_score, valid_result = self._valid_epoch(valid_data)
                self.best_valid_score, self.cur_step, stop_flag, update_flag = early_stopping(
                    valid_score, self.best_valid_score, self.cur_step, max_step=self.stopping_step,
                    bigger=self.valid_metric_bigger)
                v1 = time()
                _, test_result = self._valid_epoch(test_data, is_test=True)
                if verbose:
                    self.logger.info("epoch %d evaluating [time: %.2fs, valid_score: %f]" % (epoch_idx, v1 - v0,
                                                                                            valid_score))
                    self.logger.info("valid result: \n" + dict2str(valid_result))
                    self.logger.info("test result: \n" + dict2str(test_result))
                if update_flag:
                    if verbose:
                        self.logger.info("██ " + str(self.config["model"]) + "--Best validation results updated!!!")
                    self.best_valid_result = valid_result
                    self.best_test_upon_valid = test_result
                    if saved:
                        self._save_checkpoint(epoch_idx)
                if stop_flag:
                    if verbose:
                        self.logger.info("+++++Finished training, best eval result in epoch %d" %
                                         (epoch_idx - self.cur_step * self.eval_step))
                    break
        return self.best_valid_score, self.best_valid_result, self.best_test_upon_valid

    def _save_checkpoint(self, epoch):
        """trainer.py:345-366 (same keys), plus the generated UI graphs.  Data parallel: every rank
        holds the same parameters; rank 0 writes, the others wait at the barrier."""
        if dist.rank() != 0:
            dist.barrier()
            return
        d = self.config["checkpoint_dir"] or "saved"
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "{}-{}.pth".format(self.config["model"], self.config["dataset"]))
        torch.save(self.checkpoint_state(epoch), path)
        self.logger.info("Saved best model to {}".format(path))
        dist.barrier()

    def checkpoint_state(self, epoch):
        """The reference's checkpoint keys (trainer.py:345-366: config, epoch, state_dict, optimizer,
        best_valid_score) plus what a resume needs to continue the same run: the generated UI graphs
        (the reference does not save them, diffmm.py:263-274), the denoiser optimisers, and the
        positions of the device random streams (sampler epoch, diffusion permutations)."""
        def plain(v):
            if isinstance(v, (set, frozenset)):
                return sorted(plain(x) for x in v)
            if isinstance(v, (list, tuple)):
                return [plain(x) for x in v]
            if isinstance(v, dict):
                return {str(k): plain(x) for k, x in v.items()}
            return v if isinstance(v, (str, int, float, bool, type(None))) else str(v)
        state = {"config": {k: plain(v) for k, v in self.config.final_config_dict.items() if k != "device"},
                 "epoch": epoch, "state_dict": {k: v.detach().cpu() for k, v in self.model.state_dict().items()},
                 "optimizer": self.optimizer.state_dict(), "best_valid_score": self.best_valid_score}
        extra = getattr(self.model, "extra_state", None)
        if callable(extra):
            state["generated_graphs"] = extra()
        state["denoise_optimizers"] = {n: getattr(self, n).state_dict() for n in ("denoise_opt_image", "denoise_opt_text")
                                       if hasattr(self, n)}
        td = getattr(self, "_train_data", None)
        state["trainer_state"] = {"sched_epoch": self._sched_epoch, "cur_step": self.cur_step,
                                  "epoch_ctr": getattr(self, "_epoch_ctr", 0),
                                  "sampler_epoch": getattr(td, "_epoch", None),
                                  "best_valid_result": plain(self.best_valid_result),
                                  "best_test_upon_valid": plain(self.best_test_upon_valid)}
        return state

    def resume_checkpoint(self, path, train_data=None):
        """Continue a run from a checkpoint written by _save_checkpoint: parameters, optimisers,
        generated graphs and random-stream positions are restored, so the next epoch is the one the
        uninterrupted run would have trained (tests/test_resume_gpu.py)."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        self.load_checkpoint_state(ck, train_data)

    def load_checkpoint_state(self, ck, train_data=None):
        with torch.no_grad():
            self.model.load_state_dict({k: v.to(self.device) for k, v in ck["state_dict"].items()})
        self.optimizer.load_state_dict(ck["optimizer"])
        for n, sd in (ck.get("denoise_optimizers") or {}).items():
            getattr(self, n).load_state_dict(sd)
        load_extra = getattr(self.model, "load_extra_state", None)
        if callable(load_extra) and ck.get("generated_graphs"):
            load_extra(ck["generated_graphs"])
        ts = ck.get("trainer_state") or {}
        self.start_epoch = int(ck["epoch"]) + 1
        self.best_valid_score = ck["best_valid_score"]
        self._sched_epoch = int(ts.get("sched_epoch", self.start_epoch))
        self.optimizer.set_lr_factor(self.lr_factor(self._sched_epoch))
        self.cur_step = int(ts.get("cur_step", 0))
        if hasattr(self, "_epoch_ctr"):
            self._epoch_ctr = int(ts.get("epoch_ctr", self._epoch_ctr))
        if train_data is not None and ts.get("sampler_epoch") is not None:
            train_data._epoch = int(ts["sampler_epoch"])
        if ts.get("best_valid_result"):
            self.best_valid_result = ts["best_valid_result"]
            self.best_test_upon_valid = ts.get("best_test_upon_valid", self.best_test_upon_valid)
        self.logger.info("Resumed from epoch {} (next epoch {})".format(ck["epoch"], self.start_epoch))

    # ------------------------------------------------------------------ evaluation
    @torch.no_grad()
    def evaluate(self, eval_data, is_test=False, idx=0):
        self.model.eval()
        kmax = max(self.config["topk"])
        topk = self.topk_all(eval_data, kmax)
        return self.evaluator.evaluate_device(topk, eval_data, is_test=is_test, idx=idx)

    @torch.no_grad()
    def topk_all(self, eval_data, kmax, out_val=None):
        """Top-k indices of every eval user (n_eval x k int32, device); reference trainer.py:369-388.
        Data parallel: each rank scores a contiguous shard of the eval users; rows are all-gathered.
        out_val (n_eval x k fp32, single process only): the scores of the picked items, as the eval
        kernel computed them (the parity tests' near-tie rule reads them)."""
        d = eval_data.to_device()
        n = eval_data.pr_end
        E = eval_data.step
        lo_r, hi_r, size = dist.padded_shard(n)
        W = dist.world()
        out = getattr(self, "_topk_buf", None)
        if out is None or out.shape != (W * size, kmax):
            out = torch.zeros((W * size, kmax), dtype=torch.int32, device=self.device)
            self._topk_buf = out
        if out_val is not None and (W > 1 or out_val.shape != (n, kmax)):
            raise ValueError("topk_all: out_val is (n_eval, k) and single-process only")
        m = self.model
        fused = False
        if hasattr(m, "forward_embeddings"):
            usr, itm = m.forward_embeddings()  # identical for every batch of the pass (no_grad)
            fused = self.fused_eval and getattr(m, "fused_eval", True) and usr.shape[1] in (64, 128) and hi_r > lo_r
            if not fused:
                sb = getattr(self, "_score_buf", None)
                if sb is None or sb.shape[0] < min(E, n):
                    sb = torch.empty((min(E, n), (m.n_items + 3) // 4 * 4), dtype=torch.float32, device=self.device)
                    self._score_buf = sb
        mptr = d["mask_ptr"]
        off = dist.rank() * size - lo_r  # row of user lo_r inside the padded gather buffer
        if fused:  # scores -> mask -> top-k in one launch over the whole shard: no E x I buffer
            K.score_topk(usr, itm, d["eval_u32"][lo_r:hi_r], d["mask_ptr_dev"][lo_r:], d["mask_cols_sorted"], kmax,
                         out[off + lo_r:off + hi_r], out_val)
        for lo in range(lo_r, hi_r, E) if not fused else ():
            hi = min(hi_r, lo + E)
            users = d["eval_u32"][lo:hi]
            m0, m1 = int(mptr[lo]), int(mptr[hi])
            rows = d["mask_rows"][m0:m1] - lo
            cols = d["mask_cols"][m0:m1]
            dst = out[off + lo:off + hi]
            val = out_val[lo:hi] if out_val is not None else None
            if hasattr(m, "forward_embeddings"):
                m.topk_from_embeddings(usr, itm, users, rows, cols, kmax, dst, sb, out_val=val)
            else:
                scores = m.full_sort_predict([users.long()])
                K.mask_scores(scores, rows, cols)
                K.topk_rows(scores, kmax, dst, val)
        dist.all_gather_rows_(out, size)
        if W == 1:
            return out
        parts = [out[r * size:r * size + (dist.padded_shard(n, W, r)[1] - dist.padded_shard(n, W, r)[0])]
                 for r in range(W)]
        return torch.cat(parts)


class DiffMMTrainer(Trainer):
    def __init__(self, config, model, mg=False):
        super().__init__(config, model, mg)
        lr = config["learning_rate"]
        self.denoise_opt_image = FlatAdam([model.denoise_model_image.slab], lr=lr, weight_decay=0.0)
        self.denoise_opt_text = FlatAdam([model.denoise_model_text.slab], lr=lr, weight_decay=0.0)
        self.item_num, self.user_num = model.n_items, model.n_users
        self._perm = torch.empty(self.user_num, dtype=torch.int32, device=self.device)
        self._dloss = torch.zeros(2, dtype=torch.float64, device=self.device)
        self._epoch_ctr = 0

    def diffusion_phase(self, epoch_idx):
        """trainer.py:487-527 — train both denoisers over all users in shuffled batches of
        train_batch_size users, two Adam steps per batch.  Data parallel: each batch is split over
        the ranks (contiguous slices); t / noise / dropout draws are keyed by the row's index in the
        batch, so the gradient sum equals the single-process one up to fp32 reassociation."""
        m = self.model
        m.train()
        B = self.config["train_batch_size"]
        U = self.user_num
        W, r = dist.world(), dist.rank()
        w = m._work(1)
        m._project(w)                                         # image/text feats, detached (:501-502)
        feats_i, feats_t = w["F"][:, :64], w["F"][:, 64:]
        iE = m.rec_slab.view("E0")[U:]                        # getItemEmbeds().detach() (:496)
        _lib.call("gmr_permutation", U, m.seed, 1000 + self._epoch_ctr, ptr(self._perm), stream())
        K.zero_(self._dloss)
        dens = ((m.denoise_model_image, feats_i), (m.denoise_model_text, feats_t))
        opts = (self.denoise_opt_image, self.denoise_opt_text)
        st = m._streams
        steps = 0
        for g, lo, hi, _, _, rank_rows, row0 in dist.step_slices(U, B, W, r):
            users = self._perm[lo:hi]
            nb = users.numel()
            norm = sum(rank_rows)
            base = (self._epoch_ctr * 100000 + g) * 2
            # the two denoisers are independent until their Adam steps: the text one runs on a side
            # stream (own work buffers, slot 1) beside the image one; under DP the image gradient
            # exchange starts as soon as its step is issued (one bucket per slab)
            # data parallel: each denoiser's [W2 | b2] gradient tail starts its all-reduce inside the
            # backward as soon as it is final (beside the dpre / dW1 products), the head after it
            def one(j):
                den, feats = dens[j]
                if nb > 0:
                    diff, gc = m.diffusion_step(den, users, feats, iE, base + j, norm_rows=norm, slot=j, row0=row0,
                                                early_reduce=W > 1)
                    _lib.call("gmr_sum_f64", nb, ptr(diff), 1.0 / norm, ptr(self._dloss[j:j + 1]), 1, stream())
                    _lib.call("gmr_sum_f64", nb, ptr(gc), m.e_loss / norm, ptr(self._dloss[j:j + 1]), 1, stream())
                else:  # an idle rank issues the same two reduces
                    den.slab.zero_grad()
                    if W > 1:
                        den.early_handle = dist.all_reduce_start(den.slab.grad[den.slab_head_words():])
                return (den.early_handle if W > 1 else None,
                        dist.all_reduce_start(den.slab.grad[:den.slab_head_words()]) if W > 1 else None)

            if W == 1 and INDEP_DENOISERS:
                # one process: the two denoisers' chains (step + Adam) run independently, text on side stream 1
                # and image on the main stream, joined once after the phase (no per-step join)
                with st.on(1):
                    one(1)
                    opts[1].step()
                one(0)
                opts[0].step()
                steps += 1
                continue
            with st.on(1):
                pend_t = one(1)
            pend_i = one(0)
            st.join(1)
            for hs, opt in zip((pend_i, pend_t), opts):
                for h in hs:
                    dist.wait(h)
                opt.step()
            steps += 1
        if W == 1 and INDEP_DENOISERS:
            st.join(1)
        dist.all_reduce_(self._dloss)
        self._epoch_ctr += 1
        return steps

    def _train_epoch(self, train_data, epoch_idx, loss_func=None):
        timed = os.environ.get("GMR_PHASE_TIMES") == "1"  # phase wall times (adds 3 device syncs)
        t0 = time()
        steps = self.diffusion_phase(epoch_idx)
        if timed:
            torch.cuda.synchronize()
            t1 = time()
        self.model.rebuild_ui_graphs()                      # trainer.py:529-576
        if timed:
            torch.cuda.synchronize()
            t2 = time()
        rec_loss, batches = super()._train_epoch(train_data, epoch_idx)
        if timed:
            t3 = time()
            self.phase_ms = (1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2))
            self.logger.info("phases [ms]: diffusion %.2f, rebuild %.2f, bpr %.2f" % self.phase_ms)
        dl = self._dloss.cpu().numpy() / max(steps, 1)
        self.logger.info(f"Diffusion Loss: Image={dl[0]:.4f}, Text={dl[1]:.4f}")
        return rec_loss, batches


class GenRecV1Trainer(Trainer):
    """common/trainer.py:588-820 — per epoch: diffusion training of the image denoiser (FlipInterest
    diffusion over all users), the image UI-graph rebuild (p_sample, gen_topk mask, InterestDebiase,
    rebuild_k top-k, SpAdjDropEdge), then the BPR/contrastive epoch.  The kNN item-item graphs and the
    K-means interest clusters are built once at construction, on the device."""

    # optimal cluster counts by dataset (trainer.py:632-648); other datasets use the TikTok values
    OPTIMAL_K = {"tiktok": (18, 59), "baby": (6, 11), "sports": (9, 12)}

    def __init__(self, config, model, mg=False):
        super().__init__(config, model, mg)
        lr = config["learning_rate"]
        self.denoise_opt_image = FlatAdam([model.denoise_model_image.slab], lr=lr, weight_decay=0.0)
        self.item_num, self.user_num = model.n_items, model.n_users
        model.build_item_item_graphs(int(config["knn_k"] or 10))
        self.multimodal_interest_space = None
        self.debias = bool(config["OpenInterestDebiase"]) if "OpenInterestDebiase" in config else False
        self.sample_ratio = float(config["sample_ratio"] if config["sample_ratio"] is not None else 0.1)
        if self.debias:
            self._init_interest_clustering()
        self._perm = torch.empty(self.user_num, dtype=torch.int32, device=self.device)
        self._users = torch.arange(self.user_num, dtype=torch.int32, device=self.device)
        self._dloss = torch.zeros(4, dtype=torch.float32, device=self.device)
        self._one = torch.ones(1, dtype=torch.float32, device=self.device)
        self._epoch_ctr = 0

    def _init_interest_clustering(self):
        """MultimodalCluster.multimodal_specific_cluster for image and text (trainer.py:611-671): labels by
        device K-means; InterestDebiase consumes the image labels (interest_cluster.py:258-267)."""
        from .kmeans import kmeans_labels
        ik, tk = self.OPTIMAL_K.get(str(self.config["dataset"]), (18, 59))
        m = self.model
        self.logger.info("Performing Multimodal Clustering...")
        img = kmeans_labels(m.v_feat, ik, seed=m.seed)
        txt = kmeans_labels(m.t_feat, min(tk, 64), seed=m.seed + 1)
        self.multimodal_interest_space = {"image_modal": img, "text_modal": txt}
        self.logger.info("Multimodal Clustering Done.")

    def diffusion_phase(self, epoch_idx):
        """trainer.py:689-728: train the image denoiser over all users in shuffled batches of
        train_batch_size users.  Data parallel: each batch is split over the ranks (contiguous
        slices); the schedule / pos_weight use the whole batch, as the reference's batch does."""
        m = self.model
        m.train()
        B = self.config["train_batch_size"]
        U = self.user_num
        W, r = dist.world(), dist.rank()
        iE = m.rec_slab.view("E0")[m.n_users:]                # getItemEmbeds().detach() (:698)
        feats_i = m.getImageFeats()                           # train mode: BN statistics + dropout (:699)
        m.getTextFeats()                                      # :700 (its BN statistics update)
        den = m.denoise_model_image
        diff = m.diffusion_model
        _lib.call("gmr_permutation", U, m.seed, 2000 + self._epoch_ctr, ptr(self._perm), stream())
        K.zero_(self._dloss)
        steps = 0
        for g, lo, hi, blo, bhi, rank_rows, row0 in dist.step_slices(U, B, W, r):
            users = self._perm[lo:hi]
            # draws keyed by (global step, global row): any rank count draws the single process's noise
            step = (self._epoch_ctr * 100000 + g) * 4
            if users.numel() > 0:
                lv = diff.training_step(den, users, iE, feats_i, m.seed, step, norm_rows=sum(rank_rows),
                                        sched_users=self._perm[blo:bhi], row0=row0,
                                        rank_rows=rank_rows if W > 1 else None)
                _lib.call("gmr_axpy_dev_f32", 4, ptr(self._one), ptr(lv), ptr(self._dloss), stream())
            else:
                den.slab.zero_grad()
                if W > 1:
                    diff.idle_step(rank_rows)
            if W > 1:
                dist.all_reduce_(den.slab.grad)
            self.denoise_opt_image.step()
            steps += 1
        dist.all_reduce_(self._dloss)  # [bce, kl, cl, total] of the whole step (each rank holds its share)
        self._epoch_ctr += 1
        return steps

    @torch.no_grad()
    def rebuild(self, chunk=None):
        """trainer.py:730-789 on the device, in chunks of train_batch_size users (the schedule, the
        debias sample and the draws of a chunk depend on the chunk, as the reference's batches do).
        Data parallel: whole chunks are dealt round-robin over the ranks, so each chunk computes what
        it computes in one process; the top-k rows are summed over the ranks (each row is written by
        exactly one rank, the others hold zeros)."""
        m = self.model
        U, I = self.user_num, self.item_num
        kg, kr = m.gen_topk, m.rebuild_k
        B = chunk or self.config["train_batch_size"]
        dev = self.device
        W, r = dist.world(), dist.rank()
        topk = torch.zeros((U, kr), dtype=torch.int32, device=dev)
        den, diff = m.denoise_model_image, m.diffusion_model
        labels = self.multimodal_interest_space["image_modal"] if self.debias else None
        base = self._epoch_ctr * 100000 * 1000
        from .genrecv1 import OVERLAP_PSAMPLE, REBUILD_STREAMS
        nst = max(1, REBUILD_STREAMS) if OVERLAP_PSAMPLE else 1
        st = diff.side() if nst > 1 else None
        for q, (j, lo) in enumerate((j, lo) for j, lo in enumerate(range(0, U, B)) if j % W == r):
            hi = min(U, lo + B)
            k = q % nst
            if k:  # chunk q on side stream k - 1 through twin context k
                d2, den2 = diff.twin(den, k)
                with st.on(k - 1):
                    d2.rebuild_rows(den2, self._users[lo:hi], topk[lo:hi], labels, self.sample_ratio, m.seed,
                                    base + 4 * j)
            else:
                diff.rebuild_rows(den, self._users[lo:hi], topk[lo:hi], labels, self.sample_ratio, m.seed,
                                  base + 4 * j)
        if st is not None:
            st.join(*range(nst - 1))
        dist.all_reduce_(topk)
        uptr = torch.empty(U + 1, dtype=torch.int32, device=dev)
        uitems = torch.empty(U * kr, dtype=torch.int32, device=dev)
        K.topk_to_user_csr(topk, uptr, uitems)
        g = K.bipartite_symnorm(U, I, uptr, uitems, self_loops=True, deg_eps=0.0)
        st = 5000 + self._epoch_ctr                                                      # edgeDropper (:789)
        gd = K.csr_drop_edges(g, m.keep_rate, seed=m.seed, step=st)
        gt = K.csr_drop_edges(g, m.keep_rate, seed=m.seed, step=st, transposed=True)    # same draws, transposed
        m.set_image_ui_matrix(gd, gt)

    def _train_epoch(self, train_data, epoch_idx, loss_func=None):
        steps = self.diffusion_phase(epoch_idx)
        self.rebuild()
        rec_loss, batches = super()._train_epoch(train_data, epoch_idx)
        dl = self._dloss.cpu().numpy() / max(steps, 1)
        self.logger.info(f"Diffusion Loss: {dl[3]:.4f}")
        return rec_loss, batches
