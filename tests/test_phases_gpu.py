"""Phase-level parity of the DiffMM trainer loops through their optimiser steps (SURVEY.md 8a D16,
D18), against the reference's own loops run on the tiny DiffMM of diffmm_tiny.npz
(tests/golden/make_golden.py --phases -> diffmm_phases_tiny.npz):

  D16  DiffMMTrainer diffusion phase (common/trainer.py:491-527): all users in shuffled batches of
       40 (the permutation and every batch's t / noise / dropout draws recorded from the
       reference's seeded RNG and injected), both denoisers' training_losses, backward and their
       two Adam steps per batch: per-batch losses and both denoisers' parameters afterwards;
  D18  Trainer._train_epoch (common/trainer.py:144-208): three recorded BPR batches through
       calculate_loss, backward and Adam over the rec parameters: losses and parameters.

Tolerances: losses 1e-5 relative (fp32 reassociation); parameters after the Adam steps
rtol 1e-3 / atol 2e-6 (Adam divides each gradient by its own running magnitude, so the fp32
gradient differences of the golden tests pass through at their relative size; each step moves a
parameter by at most lr = 1e-3).
"""
import numpy as np
import pytest
import torch

from test_diffmm_gpu import build_model

pytestmark = pytest.mark.gpu

DEV = "cuda"
DEN = {"emb_W": "emb_layer_weight", "emb_b": "emb_layer_bias", "W1": "in_layers_0_weight",
       "b1": "in_layers_0_bias", "W2": "out_layers_0_weight", "b2": "out_layers_0_bias"}


def test_diffusion_phase_vs_reference(golden):
    from gmr.slab import FlatAdam
    g, ph = golden("diffmm_tiny"), golden("diffmm_phases_tiny")
    m = build_model(g)
    U = int(g["U"])
    for ours, ref in DEN.items():
        np.testing.assert_array_equal(m.denoise_model_image.slab.view(ours).cpu().numpy(), ph["init_image_" + ref])
        m.denoise_model_text.slab.load(ours, torch.as_tensor(ph["init_text_" + ref]))
    w = m._work(1)
    m._project(w)
    feats = (w["F"][:, :64], w["F"][:, 64:])
    iE = m.rec_slab.view("E0")[U:]
    dens = (m.denoise_model_image, m.denoise_model_text)
    opts = [FlatAdam([d.slab], lr=1e-3, weight_decay=0.0) for d in dens]
    perm = torch.as_tensor(ph["dif_perm"].astype(np.int32)).to(DEV)
    B = 40
    for b in range(int(ph["dif_batches"])):
        users = perm[b * B:(b + 1) * B]
        nb = users.numel()
        for j, mod in enumerate(("image", "text")):
            inj = {k: torch.as_tensor(ph[f"dif{b}_{mod}_{k}"]).to(DEV) for k in ("noise", "keep")}
            t = torch.as_tensor(ph[f"dif{b}_{mod}_t"].astype(np.int32)).to(DEV)
            diff, gc = m.diffusion_step(dens[j], users, feats[j], iE, 0, noise=inj["noise"], keep=inj["keep"], t=t,
                                        norm_rows=nb, slot=j)
            loss = float(diff.sum().item()) / nb + 0.5 * float(gc.sum().item()) / nb
            np.testing.assert_allclose(loss, ph["dif_losses"][b, j], rtol=1e-5, err_msg=f"batch {b} {mod}")
        for o in opts:
            o.step()
    for j, mod in enumerate(("image", "text")):
        for ours, ref in DEN.items():
            np.testing.assert_allclose(dens[j].slab.view(ours).cpu().numpy(), ph[f"final_{mod}_{ref}"], rtol=1e-3,
                                       atol=2e-6, err_msg=f"{mod} {ours}")


def test_bpr_phase_vs_reference(golden):
    from gmr.slab import FlatAdam
    g, ph = golden("diffmm_tiny"), golden("diffmm_phases_tiny")
    m = build_model(g)
    U = int(g["U"])
    names = ("uEmbeds", "iEmbeds", "image_trans", "text_trans", "modal_weight")
    s = m.rec_slab

    def params():
        e0 = s.view("E0").cpu().numpy()
        return {"uEmbeds": e0[:U], "iEmbeds": e0[U:], "image_trans": s.view("image_trans").cpu().numpy(),
                "text_trans": s.view("text_trans").cpu().numpy(), "modal_weight": s.view("modal_weight").cpu().numpy()}
    p0 = params()
    for n in names:
        np.testing.assert_array_equal(p0[n], ph["bpr_init_" + n])
    opt = FlatAdam(m.optim_slabs(), lr=1e-3, weight_decay=0.0)
    for st in range(3):
        inter = ph[f"bpr{st}_inter"].astype(np.int32)
        u, p, n = (torch.as_tensor(inter[i]).to(DEV) for i in range(3))
        loss = m.rec_step(u, p, n)
        np.testing.assert_allclose(loss.item(), ph["bpr_losses"][st], rtol=1e-5, err_msg=f"step {st}")
        opt.step()
    p1 = params()
    for n in names:
        np.testing.assert_allclose(p1[n], ph["bpr_final_" + n], rtol=1e-3, atol=2e-6, err_msg=n)
