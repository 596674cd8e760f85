"""ctypes binding of libgmr_hip.so (the C-ABI declared in include/gmr.h).

The HIP library is the ONLY compute path of this package: when it is missing or cannot be
loaded, every op raises immediately — there is no CPU or eager-PyTorch fallback.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GMR_HIP_LIB", os.path.join(_HERE, "libgmr_hip.so"))

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
F32 = ctypes.c_float
F64 = ctypes.c_double
CP = ctypes.c_char_p



class SpmmJob(ctypes.Structure):
    """gmr_spmm_job (include/gmr.h)."""
    _fields_ = [("col", P), ("val", P), ("plan", P), ("partial", P), ("n_rows", I64), ("nnz", I64),
                ("seg_nnz", I32), ("n_blocks", I32), ("flags", I32), ("reserved", I32),
                ("x_lo", P * 4), ("ld_lo", I64 * 4), ("x_hi", P * 4), ("ld_hi", I64 * 4), ("split", I64),
                ("alpha", F32), ("beta", F32), ("y", P * 4), ("ld_y", I64 * 4)]


# name: (restype, argtypes) — must match include/gmr.h
SIGNATURES = {
    "gmr_last_error_string": (CP, []),
    "gmr_version": (I32, []),
    "gmr_device_name": (I32, [P, I32]),
    "gmr_zero": (I32, [P, I64, P]),
    "gmr_spmm_plan_words": (I64, [I64, I64, I32]),
    "gmr_sqnorm_nparts": (I64, [I64]),
    "gmr_spmm_partial_rows": (I64, [I64, I64, I32]),
    "gmr_spmm_plan_build": (I32, [P, I64, I64, I32, P, P]),
    "gmr_spmm_plan_build_split": (I32, [P, I64, I64, I32, I64, P, P]),
    "gmr_spmm_plan_pack": (I32, [P, P, P, I64, I64, I32, P, P]),
    "gmr_spmm_plan_info": (I32, [P, P, P]),
    "gmr_event_create": (I32, [P]),
    "gmr_event_destroy": (I32, [P]),
    "gmr_stream_fork": (I32, [P, P, P]),
    "gmr_delay": (I32, [I32, P]),
    "gmr_score_f16": (I32, [I64, I64, I64, P, I64, P, I64, P, I64, P]),
    "gmr_spmm_multi_f32": (I32, [P, P, I64, I64, P, I32, I32, P, P, P, P, I64, F32, F32, P, P, P, I32, P]),
    "gmr_spmm_jobs_f32": (I32, [I32, P, P]),
    "gmr_spmm_panel_f32": (I32, [P, P, I64, I64, P, I32, I32, P, I64, F32, F32, P, I64, P, I32, P]),
    "gmr_spmm_csr_f32": (I32, [P, P, P, I64, I64, P, I32, P, I32, P, P, P, P, I64, F32, F32, P, I64, I32, P]),
    "gmr_spmm_side_plan_words": (I64, [P, I64, I64, I32]),
    "gmr_spmm_side_plan_build": (I32, [P, I64, I64, I32, P, I64]),
    "gmr_spmm_side_scratch_floats": (I64, [P]),
    "gmr_spmm_side_pack": (I32, [P, P, P, I64, I64, I64, P, P]),
    "gmr_spmm_side_pack_classes": (I32, [P, P, P, P, P, P]),
    "gmr_spmm_side_tune": (I32, [I32, I32]),
    "gmr_spmm_side_f32": (I32, [P, I32, P, P, P, P, I64, F32, F32, P, P, P, I32, P]),
    "gmr_spmm_side2_f32": (I32, [P, I32, P, P, P, P, I64, F32, F32, P, P, P, P, I32, P, I32, P]),
    "gmr_spmm_side_jobs_f32": (I32, [I32, P, P, I32, P, P, P, P, P, F32, F32, P, P, I32, P]),
    "gmr_bipartite_nnz": (I64, [I64, I64, I64, I32]),
    "gmr_bipartite_workspace_ints": (I64, [I64, I64]),
    "gmr_bipartite_symnorm_build": (I32, [I64, I64, P, P, I64, I32, F64, P, P, P, P, P]),
    "gmr_topk_to_user_csr": (I32, [I64, I32, P, I64, P, P, P]),
    "gmr_gemm_workspace_floats": (I64, [I32, I32, I64, I64, I64, I32, I32]),
    "gmr_gemm_kernel_kind": (I32, [I32, I32, I64, I64, I64, I32, I32, I32]),
    "gmr_gemm_f32": (I32, [I32, I32, I64, I64, I64, F32, P, I64, P, I64, F32, P, I64, I32, P, P, I64, P, I64, P, P,
                           F32, I32, I32, P, I64, P]),
    "gmr_split3_planes": (I32, [I64, I64, P, I64, P, I64, I64, P]),
    "gmr_dmm_combine_fwd": (I32, [I64, P, P, P, P, P, F32, P, P]),
    "gmr_dmm_final_fwd": (I32, [I64, P, P, F32, P, P, P]),
    "gmr_dmm_cl_fwd": (I32, [I64, P, P, P, P, P, P]),
    "gmr_dmm_final_bwd": (I32, [I64, P, P, P, P, F32, P, P, P, P, P]),
    "gmr_dmm_final_bwd_partials": (I64, [I64]),
    "gmr_dmm_mw_grad": (I32, [I64, P, P, P, I32, P]),
    "gmr_dmm_dg": (I32, [I64, I64, P, P, P, P]),
    "gmr_dmm_cl_bwd": (I32, [I64, P, P, P, F32, P, P, P]),
    "gmr_dmm_assemble": (I32, [I64, I64, P, P, P, P, P, F32, P, P, P]),
    "gmr_dmm_final_bwd2": (I32, [I64, P, P, P, P, F32, P, P, P, P, I32, F32, P, P, P]),
    "gmr_dmm_cl_bwd2": (I32, [I64, P, P, P, F32, P, P, I32, I32, P]),
    "gmr_dmm_assemble2": (I32, [I64, I64, P, P, P, P, P, F32, P, P, P, P, F32, P, I32, P]),
    "gmr_dmm_bpr_sqnorm": (I32, [I32, I64, P, P, P, P, P, P, F32, I64, P, P, P]),
    "gmr_dmm_loss_mw": (I32, [I64, P, F32, P, I64, F32, P, P, F32, P, P, I64, P, P, P, P]),
    "gmr_scatter_sorted_nbwd_f32": (I32, [I32, P, P, I64, P, P, I64, P, P]),
    "gmr_contrast_fused_nbwd_f32": (I32, [I32, I64, P, I64, P, I64, P, P, I64, F32, F32, P, P, I64, P, I64, P, I64, P, P,
                                          I64, P]),
    "gmr_normalize_rows_f32": (I32, [I64, I32, P, I64, P, I64, P, P]),
    "gmr_normalize_rows_bwd_f32": (I32, [I64, I32, P, I64, P, P, I64, P, I64, F32, I32, P]),
    "gmr_bpr_fwd_bwd": (I32, [I32, I64, P, P, P, P, P, P, F32, P]),
    "gmr_row_softmax_f32": (I32, [I64, I64, P, I64, F32, P, P]),
    "gmr_contrast_rows": (I32, [I32, P, P, I64, P, F32, F32, P, P, I64, P]),
    "gmr_contrast_workspace_floats": (I64, [I32, I64]),
    "gmr_contrast_fused_f32": (I32, [I32, I64, P, I64, P, I64, P, P, I64, F32, F32, P, P, I64, P, I64, P, I64, P]),
    "gmr_gather_rows_f32": (I32, [I32, I32, P, I64, P, I64, P, I64, P]),
    "gmr_scatter_sorted_f32": (I32, [I32, I32, P, P, I64, P, I64, P]),
    "gmr_sort_batch_keys": (I32, [I64, P, P, P, I32, I64, P, I64, I32, P]),
    "gmr_sum_f32": (I32, [I64, P, F32, P, I32, P]),
    "gmr_sqnorm_f32": (I32, [I64, P, F32, P, I32, P, P]),
    "gmr_sqnorm_part_f32": (I32, [I64, P, P, P]),
    "gmr_dmm_loss_total": (I32, [I64, P, F32, P, I64, F32, P, P, F32, P, P]),
    "gmr_sum_f64": (I32, [I64, P, F64, P, I32, P]),
    "gmr_colsum_f32": (I32, [I64, I64, P, I64, P, I32, P, I32, P]),
    "gmr_sample_epoch": (I32, [I64, P, P, P, P, P, I64, U64, U64, P, P, P, P, P]),
    "gmr_permutation": (I32, [I64, U64, U64, P, P]),
    "gmr_diff_sample_t": (I32, [I32, I32, U64, U64, I64, P, P]),
    "gmr_diff_qsample": (I32, [I32, I32, P, P, P, P, P, P, P, I64, P, I64, F32, I32, U64, U64, I64, P, I64, P]),
    "gmr_diff_densify": (I32, [I32, I32, P, P, P, P, I64, P]),
    "gmr_diff_time_bias": (I32, [I32, I32, P, P, P, I64, I64, P, I32, P, P, P, P]),
    "gmr_diff_loss_rows": (I32, [I32, I32, P, P, P, P, P, P, P, I64, F32, P, P, P, I32, P]),
    "gmr_vbpr_loss_fwd_bwd": (I32, [I32, I32, P, I64, P, P, P, I64, F32, P, P, P, P, P, I64, P]),
    "gmr_fill2d_f32": (I32, [I64, I64, P, I64, F32, P]),
    "gmr_transpose_f32": (I32, [I64, I64, P, I64, P, I64, P]),
    "gmr_diff_sparse_hidden": (I32, [I32, I32, P, P, P, P, I64, P, P, I64, P]),
    "gmr_diff_sparse_pre": (I32, [I32, I32, P, P, P, P, I64, P, P, I64, P, I64, P]),
    "gmr_tanh_bias_f32": (I32, [I64, I32, P, I64, P, P, I64, P]),
    "gmr_diff_sample_t_importance": (I32, [I32, I32, I32, P, P, F64, U64, U64, I64, P, P, P]),
    "gmr_diff_history_update": (I32, [I32, I32, I32, P, P, P, P, P]),
    "gmr_diff_gc_rows": (I32, [I32, P, P, P, P, I64, P, I64, F32, P, I64, P, P]),
    "gmr_diff_time_bwd": (I32, [I32, I32, I32, P, P, P, P, I64, I64, P, P, P, P, I32, P]),
    "gmr_mask_scores_f32": (I32, [I64, P, P, P, I64, F32, P]),
    "gmr_topk_rows_f32": (I32, [I64, I64, P, I64, I32, P, I64, P, P]),
    "gmr_score_topk_f32": (I32, [I64, P, P, I64, I64, P, I64, I64, P, P, F32, I32, P, I64, P, P]),
    "gmr_score_topk_x6": (I32, [I64, P, P, I64, I64, P, I64, I64, I64, P, P, F32, I32, P, I64, P, P]),
    "gmr_eval_metrics_partials": (I64, [I64]),
    "gmr_eval_metrics": (I32, [I64, P, I64, I32, P, P, I32, P, P, P, P]),
    "gmr_eval_metrics_sel": (I32, [I64, P, P, I64, I32, P, P, I32, P, P, P, P]),
    "gmr_topk_item_counts": (I32, [I64, P, I64, I32, P, I64, P, P]),
    "gmr_adam_f32": (I32, [I64, P, P, P, P, F32, F32, F32, F32, F32, F32, P]),
    "gmr_colsum_split_floats": (I64, [I64]),
    "gmr_colsum_split_f32": (I32, [I64, I64, P, I64, P, I32, P, I64, P]),
    # GenRecV1
    "gmr_bn_parts_doubles": (I64, [I64]),
    "gmr_bn_fwd_f32": (I32, [I64, P, I64, I32, F32, F32, P, P, P, P, P, P, P, I32, F32, P, I64, F32, P, I64, I32, P, I64, P, P, I64, P, P]),
    "gmr_bn_bwd_f32": (I32, [I64, P, I64, P, P, P, P, I32, F32, P, I64, F32, P, I64, P, I64, P, P, P, P, P, P, P, I32, P, I64, I32, P]),
    "gmr_gr_parts": (I64, [I64]),
    "gmr_gr_content_fwd": (I32, [I64, P, P, P, P, P, P, P]),
    "gmr_gr_content_bwd": (I32, [I64, P, P, P, P, P, P, P, P, F32, P, P, P, P, P]),
    "gmr_gr_fusion_fwd": (I32, [I64, P, P, P, P, P, P, P, P, P]),
    "gmr_gr_fusion_bwd": (I32, [I64, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "gmr_mul64_f32": (I32, [I64, P, I64, P, I64, P, I64, F32, I32, P]),
    "gmr_dot64_f32": (I32, [I64, P, I64, P, I64, P, F32, P, I32, P]),
    "gmr_nce_rows_f32": (I32, [I64, P, I64, F32, P, P]),
    "gmr_nce_rows_off_f32": (I32, [I64, I64, P, I64, I64, F32, P, P]),
    "gmr_bpr_logsigmoid_f32": (I32, [I32, I64, P, P, P, P, P, P, F32, P]),
    "gmr_axpy_dev_f32": (I32, [I64, P, P, P, P]),
    "gmr_mul_f32": (I32, [I64, P, P, P, P]),
    "gmr_keep_mask_u8": (I32, [I64, F32, U64, U64, U64, P, P]),
    "gmr_csr_transpose": (I32, [I64, I64, I64, P, P, P, P, P, P, P, P, P, P]),
    "gmr_csr_drop_count": (I32, [I64, P, P, I32, P, F32, U64, U64, P, P, P]),
    "gmr_csr_drop_write": (I32, [I64, P, P, P, I32, P, F32, U64, U64, P, P, P, P]),
    "gmr_knn_symnorm_csr": (I32, [I64, I32, P, I64, P, I64, P, P, P, P, P]),
    "gmr_gen_mask": (I32, [I32, I32, I32, P, I64, P, P, I64, P, P]),
    "gmr_debias_select": (I32, [I32, I32, P, I64, P, P, I64, F32, U64, U64, P, P, I32, P, P]),
    "gmr_debias_apply": (I32, [I32, P, P, I32, P, I64, I32, P, P, I64, P]),
    "gmr_kmeans_standardize": (I32, [I64, I32, P, I64, P, P, P, I64, P, P]),
    "gmr_kmeans_pp_pick": (I32, [I64, P, U64, U64, P, P]),
    "gmr_kmeans_take_center": (I32, [I32, P, I64, P, P, I64, I32, P, P, P]),
    "gmr_kmeans_min_dist": (I32, [I64, P, P, I64, P, I32, P, I32, P]),
    "gmr_kmeans_pp_greedy": (I32, [I64, I32, P, P, I64, P, P, P, I64, I32, P, I64, I32, P, P]),
    "gmr_kmeans_parts": (I64, [I64]),
    "gmr_kmeans_assign": (I32, [I64, I32, P, I64, P, P, P, P, I64, P, P, P]),
    "gmr_kmeans_centroids": (I32, [I32, I32, P, I64, P, I64, I64, P, I64, P, P]),
    "gmr_flip_schedule": (I32, [I32, P, P, I32, I32, P, P]),
    "gmr_flip_qsample": (I32, [I32, I32, P, I64, P, I32, P, I32, F32, P, I64, U64, U64, I64, P, I64, P]),
    "gmr_flip_step": (I32, [I32, I32, P, I64, P, I32, I32, I32, P, I64, U64, U64, I64, P, I64, P, I64, P]),
    "gmr_flip_loss_rows": (I32, [I32, I32, P, I64, P, I64, P, P, I32, F32, P, I64, P, P, P]),
    "gmr_flip_total": (I32, [P, P, F32, P, P]),
    "gmr_layernorm_fwd": (I32, [I64, I32, P, I64, P, I64, P, I64, F32, P, P, F32, I32, P, I64, P, I64, P, P, P]),
    "gmr_layernorm_drop_fwd": (I32, [I64, I32, P, I64, P, I64, F32, U64, U64, U64, P, I64, F32, P, P, F32, I32, P, I64,
                                     P, I64, P, P, P]),
    "gmr_layernorm_parts_floats": (I64, [I64, I32]),
    "gmr_layernorm_bwd": (I32, [I64, I32, P, I64, P, P, P, P, I32, P, I64, P, I64, I32, P, P, P, I32, P]),
    "gmr_adaln_fwd": (I32, [I64, I32, P, I64, P, I32, P, I64, P, I64, P]),
    "gmr_adaln_bwd": (I32, [I64, I32, P, I64, P, I64, P, P, I64, P, I64, P, I64, P]),
    "gmr_dropout_f32": (I32, [I64, I32, I32, P, I64, F32, P, P, I64, U64, U64, I64, P, I64, P]),
    "gmr_time_embedding": (I32, [I32, I32, P, P]),
    "gmr_silu_f32": (I32, [I64, P, P, P, P]),
    "gmr_xattn_table_f32": (I32, [I32, I32, I32, P, P, I64, F32, P, P]),
    "gmr_decoder_layers_fwd_f32": (I32, [I64, I64, I32, I32, I32, P, P, I64, I32, F32, U64, U64, I64, I32, P, P, I32, P,
                                         I64, P]),
    "gmr_xattn_fwd_f32": (I32, [I64, I32, I32, P, P, F32, P, P, I64, U64, U64, I64, P, I64, P]),
    "gmr_xattn_bwd_workspace_floats": (I64, [I64, I32, I32]),
    "gmr_xattn_bwd_f32": (I32, [I64, I32, I32, P, I64, P, I64, P, P, F32, P, P, P, I64, P]),
    "gmr_nce_pairs_f32": (I32, [I32, I64, I64, I64, P, P, P, I64, P, I64, P]),
    "gmr_nce_combine_f32": (I32, [I32, I64, I64, I64, P, P, P, I64, P, I64, P, I64, P]),
}

_lib = None


class HipLibraryMissing(RuntimeError):
    pass


def load():
    """Load libgmr_hip.so (after torch, so the process shares torch's HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (loads torch's libamdhip64 first; our .so binds to it by SONAME)

    if not os.path.exists(LIB_PATH):
        raise HipLibraryMissing(
            f"libgmr_hip.so not found at {LIB_PATH}; build it with `make -C generative-multimodal-recommendation_amd`"
            " or __graft_entry__.build(). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, name="gmr"):
    if rc != 0:
        msg = load().gmr_last_error_string()
        raise RuntimeError(f"{name} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


_fns = {}
# a gmr.tape.Tape while one records a step (every call below is also noted on it), else None
recorder = None


def call(name, *args):
    """Call an int-returning entry point and raise on a non-zero status (argument count checked:
    ctypes would silently pass surplus arguments to a C function)."""
    ent = _fns.get(name)
    if ent is None:
        fn = getattr(load(), name)
        ent = _fns[name] = (fn, len(fn.argtypes))
    fn, n = ent
    if len(args) != n:
        raise TypeError(f"{name} takes {n} arguments, got {len(args)}")
    rc = fn(*args)
    if rc != 0:
        return check(rc, name)
    if recorder is not None:
        recorder.note(name, fn, args)
    return rc
