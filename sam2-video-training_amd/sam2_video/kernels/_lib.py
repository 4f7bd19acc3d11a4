"""ctypes binding of libsam2hip.so (the C ABI declared in include/sam2hip.h).

The library is the product: there is no CPU or PyTorch fallback.  Loading fails
loudly when the shared object is missing, and every launch checks the HIP
status it returns.  `torch` is imported first so the HIP runtime torch ships
(same SONAME libamdhip64.so.7) is the one the library binds to: a single
runtime, shared streams and device pointers.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_int64, c_uint64, c_void_p

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# S2H_LIB_PATH: measurement override (A/B of two builds of the same library)
LIB_PATH = os.environ.get("S2H_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "_lib", "libsam2hip.so")

P = c_void_p
I = c_int
L = c_int64
F = c_float

# name -> argtypes (restype is int: a hipError_t value, 0 == success)
SIGNATURES = {
    "s2h_version": [],
    "s2h_rng_bind": [P],
    "s2h_gemm": [I, I, I, I, I, I, P, L, L, L, P, L, L, L, P, L, L, P, I, P, L, L, P, L, L, I, P, F, c_uint64, c_uint64,
                 F, F, I, P],
    "s2h_linear_wgrad": [I, L, I, I, P, L, P, L, P, L, P, I, P],
    "s2h_linear_rope": [I, I, I, P, L, P, L, P, P, L, P, P, I, I, I, I, I, P],
    "s2h_linear_add_ln": [I, I, I, P, L, P, L, P, P, L, F, c_uint64, c_uint64, P, L, P, P, F, P, L, P, P, P],
    "s2h_linear_dgrad_ln_bwd_ws_bytes": [I, I],
    "s2h_linear_dgrad_ln_bwd": [I, I, I, P, L, P, L, F, P, L, P, P, P, P, L, P, L, P, P, P, P],
    "s2h_ffn_bwd_dgrad": [I, I, P, L, P, P, P, L, F, P, L, P, L, P],
    "s2h_dec_sched": [I],
    "s2h_dec_self": [I, I, I, F, P, P, P, P, P, P, P, P, P, P, P, P, F, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "s2h_dec_post_a": [I, I, P, P, P, P, P, P, F, P, P, P, P, P],
    "s2h_dec_post_b": [I, I, I, P, P, P, P, F, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "s2h_dec_final": [I, I, P, P, P, P, P, P, F, P, P, P, P, P],
    "s2h_ffn_fwd": [I, I, P, L, P, P, P, P, F, c_uint64, c_uint64, c_uint64, c_uint64, P, L, P, L, P],
    "s2h_ln_wgrad_finalize": [I, I, P, P, P, P],
    "s2h_mlp_heads": [I, I, P, P, P, P, P, P, P, P, P, P, P, P],
    "s2h_attn_fwd_ws_bytes": [I, I, I, I, I, I],
    "s2h_attn_config": [I],
    "s2h_flash_variant2": [I],
    "s2h_gemm_f32_small": [I],
    "s2h_gemm_config": [I],
    "s2h_gemm_split_target": [I],
    "s2h_gemm_tiny_config": [I],
    "s2h_gemm_w41": [I],
    "s2h_gemm_class_config": [I, I],
    "s2h_gemm_tiny_splitk": [I],
    "s2h_gemm_areg": [I],
    "s2h_wgrad_workspace": [P, L, I],
    "s2h_grad_defer": [P, L, P, L],
    "s2h_grad_defer_flush": [P],
    "s2h_grad_defer_reset": [],
    "s2h_grad_defer_pending": [],
    "s2h_wgrad_force": [I, I],
    "s2h_flash_fwd_sets": [I],
    "s2h_attn_win": [I],
    "s2h_mx8_quant": [I, I, I, P, L, L, P, L, P, L, P],
    "s2h_gemm_mx8": [I, I, I, P, L, P, L, P, L, P, L, P, I, L, P, P, L, P, L, I, F, c_uint64, c_uint64, F, F, I, P],
    "s2h_mx8_config": [I],
    "s2h_attn_bwd_ws_bytes": [I, I, I, I, I, I],
    "s2h_attn_fwd": [I, I, I, I, I, I, P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L, P, F, F, c_uint64, c_uint64, P, P, L,
                     P],
    "s2h_attn_keep_words": [I, I, I, I],
    "s2h_attn_bwd": [I, I, I, I, I, I,
                     P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L,
                     P, L, L, L, P, L, L, L, P, L, L, L,
                     P, P, F, F, c_uint64, c_uint64, P, P, L, P],
    "s2h_flash_bwd_ok": [I, I, I],
    "s2h_flash_bwd_frames": [I, I, I, I, I, P, P, P, P, L, L, L, P, L, L, P, L, L, P, L, L, L, P, L, L, L, P, L, L, L,
                             P, L, L, P, L, L, P, P, F, F, c_uint64, P, P, P],
    "s2h_flash_bwd_frames_rope": [I, I, I, I, I, P, P, P, P, L, L, L, P, L, L, P, L, L, P, L, L, L, P, L, L, L, P, L,
                                  L, L, P, L, L, P, L, L, P, P, F, F, c_uint64, P, P, P, P, I, P, P],
    "s2h_attn_fwd_vfold_ws_bytes": [I, I, I],
    "s2h_attn_fwd_vfold": [I, I, I, P, L, L, P, L, L, P, L, L, P, L, L, P, F, F, c_uint64, c_uint64, P, P, L, P],
    "s2h_flash_bwd_frames_vfold": [I, I, I, P, P, P, P, L, L, P, L, P, L, P, L, L, P, L, L, P, L, L, P, L, P, P, F, F,
                                   c_uint64, P, P, P],
    "s2h_flash_bwd_frames_vfold_rope": [I, I, I, P, P, P, P, L, L, P, L, P, L, P, L, L, P, L, L, P, L, L, P, L, P, P, F, F,
                                   c_uint64, P, P, P, P, I, P, P],
    "s2h_flash_bwd_frames_vfold_rope_qk": [I, I, I, P, P, P, P, L, L, P, L, P, L, P, L, L, P, L, L, P, L, L, P, L, P,
                                           P, F, F, c_uint64, P, P, P, P, I, P, P, P],
    "s2h_vfold_weight": [I, I, I, P, P, P, P],
    "s2h_vfold_grad": [I, I, I, P, P, P, P],
    "s2h_layernorm_fwd": [I, I, I, P, L, P, L, I, P, P, P, F, P, L, P, P, P],
    "s2h_layernorm_fwd_pe": [I, I, I, P, P, P, F, P, P, P, P, I, P, P],
    "s2h_layernorm_bwd_ws_bytes": [I, I, I],
    "s2h_layernorm_bwd": [I, I, I, P, L, P, L, P, P, P, P, L, I, P, L, P, P, P, P],
    "s2h_add": [I, L, P, P, F, F, P, P],
    "s2h_add_bcast": [I, L, L, P, F, P, L, F, P, P],
    "s2h_act_fwd": [I, L, P, I, F, F, P, P],
    "s2h_act_bwd": [I, L, P, P, I, P, I, P],
    "s2h_cast": [I, I, L, P, P, P],
    "s2h_dropout": [I, L, P, P, F, c_uint64, c_uint64, P, P],
    "s2h_act_dropout_bwd": [I, L, P, P, I, F, c_uint64, c_uint64, P, P],
    "s2h_relu_mask_bwd": [I, L, P, P, F, P, P],
    "s2h_rope": [I, L, I, I, P, L, L, P, L, L, P, P, I, I, P],
    "s2h_maxpool2_fwd": [I, I, I, I, I, P, L, P, P],
    "s2h_maxpool2_bwd": [I, I, I, I, I, P, L, P, P, L, P],
    "s2h_window": [I, I, I, I, I, I, P, P, I, I, P],
    "s2h_window_pad": [I, I, I, I, I, I, P, P, P, P],
    "s2h_window_pad_colsum": [I, I, I, I, I, I, P, P, P],
    "s2h_copy2d_batch": [I, P, P, P, P, P, P, P],
    "s2h_up2_add": [I, I, I, I, I, P, P, P, P],
    "s2h_pool2_sum": [I, I, I, I, I, P, P, I, P],
    "s2h_bilinear_fwd": [I, I, I, I, I, P, P, P],
    "s2h_bilinear_bwd": [I, I, I, I, I, P, P, P],
    "s2h_colsum": [I, L, I, P, L, P, I, P],
    "s2h_colsum_seg": [I, I, L, I, P, L, P, P, P, P],
    "s2h_memory_pos": [I, I, I, I, P, P, P, P, P],
    "s2h_sum_outer": [I, I, L, P, P, I, P],
    "s2h_sum_outer_batched": [I, I, I, L, P, P, I, P],
    "s2h_im2col": [I, I, I, I, I, I, I, I, I, I, I, L, P, P, P],
    "s2h_mask_down_stage": [I, I, I, I, I, I, P, I, F, F, P, P, P, P, F, P, P],
    "s2h_dwconv": [I, I, I, I, I, I, I, P, P, P, P, P],
    "s2h_convt2": [I, I, I, I, I, P, P, P, P, I, P],
    "s2h_convt2_store": [I, I, I, I, I, P, P, P, I, P, P],
    "s2h_convt2_tail": [I, I, I, I, I, P, P, P, I, P, P, P, P, P],
    "s2h_convt2_ln_gelu": [I, I, I, I, I, P, P, P, I, P, P, F, P, P, P, P, P, P],
    "s2h_row_gate": [I, L, L, P, P, F, P, I, P],
    "s2h_row_gate_cast": [I, I, L, L, P, P, F, P, I, P, P],
    "s2h_gate_mix": [I, L, L, P, P, P, I, I, P, P],
    "s2h_mask_stats": [I, L, P, L, P, L, F, P, P],
    "s2h_mask_loss_finalize": [I, L, P, P, P, F, F, F, F, P, P, P],
    "s2h_mask_loss_bwd": [I, L, P, L, P, L, F, P, P, L, P, P, P],
    "s2h_bce_stats": [I, L, P, L, P, L, F, P, P, P],
    "s2h_bce_finalize": [I, L, P, I, F, P, P, P],
    "s2h_bce_bwd": [I, L, P, L, P, L, F, P, P, P, P, L, P],
    "s2h_mask_eval_counts": [I, L, P, L, P, L, P, P],
    "s2h_group_max_fwd": [I, L, P, P, P, L, P, L, P, P],
    "s2h_group_max_bwd": [I, L, P, P, P, L, P, L, P],
    "s2h_group_wavg_fwd": [I, I, P, P, P, P, P, P],
    "s2h_group_wavg_bwd": [I, I, P, P, P, P, P, P, P, P, P],
    "s2h_sigmoid_grad_axpy": [I, L, P, L, P, P, L, P],
    "s2h_grad_norm": [L, P, P, F, F, P, P],
    "s2h_adamw": [L, P, P, P, P, P, F, F, F, F, F, I, P, P],
    "s2h_pos_embed": [I, I, I, I, I, P, P, P, P],
    "s2h_pos_embed_bwd": [I, I, I, I, I, P, P, P, P],
    "s2h_point_embed": [I, I, I, P, P, P, P, P, P],
    "s2h_point_embed_bwd": [I, I, I, P, P, P, P],
    "s2h_point_embed_bwd_rows": [I, I, I, P, P, P, P],
    "s2h_prof_enable": [I],
    "s2h_prof_select": [I],
    "s2h_prof_reset": [],
    "s2h_prof_count": [],
    "s2h_prof_read": [I, P, P],
    "s2h_prof_read_tags": [I, P],
    "s2h_trace_marker": [I, P],
    "s2h_prompt_objects": [I, I, I, P, I, P, P, P, P, I],
    "s2h_prompt_object_masks": [I, I, I, P, I, P, I],
    "s2h_mask_moments": [I, I, I, P, P, I],
}

_LIB = None


# entry points that do not return a hipError_t
RESTYPES = {"s2h_attn_fwd_ws_bytes": c_int64, "s2h_attn_bwd_ws_bytes": c_int64, "s2h_attn_keep_words": c_int64,
            "s2h_attn_fwd_vfold_ws_bytes": c_int64,
            "s2h_layernorm_bwd_ws_bytes": c_int64, "s2h_linear_dgrad_ln_bwd_ws_bytes": c_int64,
            "s2h_grad_defer_pending": c_int}


class HipKernelError(RuntimeError):
    pass


def lib():
    """The loaded library (raises if it is missing: no fallback path exists)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libsam2hip.so not found at {LIB_PATH}; build it with `python __graft_entry__.py` "
                "or `make -C sam2-video-training_amd/csrc` (there is no CPU fallback)")
        h = ctypes.CDLL(LIB_PATH)
        missing = []
        for name, argtypes in SIGNATURES.items():
            fn = getattr(h, name, None)
            if fn is None:
                missing.append(name)
                continue
            fn.argtypes = argtypes
            fn.restype = RESTYPES.get(name, c_int)
        # an older build selected by S2H_LIB_PATH (A/B runs) may lack newer entry points (calling one
        # raises); the shipped library must have them all
        if missing and not os.environ.get("S2H_LIB_PATH"):
            raise RuntimeError(f"{LIB_PATH} lacks entry points {missing} (a stale build): rebuild it with "
                               "`make -C sam2-video-training_amd/csrc`")
        if os.environ.get("S2H_GEMM_CFG"):  # measurement override of the GEMM tiling choice
            h.s2h_gemm_config(int(os.environ["S2H_GEMM_CFG"]))
        if os.environ.get("S2H_GEMM_SPLIT_TARGET"):  # workgroups a split-K launch aims at (A/B)
            h.s2h_gemm_split_target(int(os.environ["S2H_GEMM_SPLIT_TARGET"]))
        if os.environ.get("S2H_GEMM_TINY_CFG"):  # ... of the tiny-M (<= 128 rows) GEMMs only
            h.s2h_gemm_tiny_config(int(os.environ["S2H_GEMM_TINY_CFG"]))
        if os.environ.get("S2H_ATTN_CFG"):  # flash switch | forward key-split target << 8 (A/B)
            h.s2h_attn_config(int(os.environ["S2H_ATTN_CFG"]))
        if os.environ.get("S2H_GEMM_F32_SMALL"):  # small fp32 GEMMs on 32 x 32 tiles (1) / 64 x 64 (0)
            h.s2h_gemm_f32_small(int(os.environ["S2H_GEMM_F32_SMALL"]))
        if os.environ.get("S2H_FLASH_V2"):  # round-6 flash kernel variants (A/B bits, s2h_flash_variant2)
            h.s2h_flash_variant2(int(os.environ["S2H_FLASH_V2"]))
        if os.environ.get("S2H_DEC_SCHED"):  # token self-attention block weights a phase ahead (A/B)
            h.s2h_dec_sched(int(os.environ["S2H_DEC_SCHED"]))
        if os.environ.get("S2H_ATTN_WIN"):  # small-window attention kernels on / off (A/B)
            h.s2h_attn_win(int(os.environ["S2H_ATTN_WIN"]))
        if os.environ.get("S2H_GEMM_AREG"):  # ... short-K GEMMs with A in registers (A/B)
            h.s2h_gemm_areg(int(os.environ["S2H_GEMM_AREG"]))
        if os.environ.get("S2H_FLASH_QS"):  # ... forward 16-query sets per wave, V-fold | plain << 4 (A/B)
            h.s2h_flash_fwd_sets(int(os.environ["S2H_FLASH_QS"]))
        if os.environ.get("S2H_GEMM_CLASS"):  # tiling per GEMM class "c0,..,c4" (0 = rules; A/B)
            for i, c in enumerate(os.environ["S2H_GEMM_CLASS"].split(",")[:6]):
                h.s2h_gemm_class_config(i, int(c or 0))
        if os.environ.get("S2H_GEMM_TINY_SPLITK"):  # split-K + reduce-epilogue for tiny-M long-K GEMMs (A/B)
            h.s2h_gemm_tiny_splitk(int(os.environ["S2H_GEMM_TINY_SPLITK"]))
        if os.environ.get("S2H_GEMM_W41"):  # ... bf16-output GEMMs on 4 x 1 wave grids (A/B)
            h.s2h_gemm_w41(int(os.environ["S2H_GEMM_W41"]))
        _LIB = h
    return _LIB


_HOST_LIB = None
# the prompt stage's host-only entry points (csrc/prompts_host.cpp), resolvable from a separate
# host build: tools/sanitize_host.sh points S2H_HOST_LIB_PATH at an ASan + UBSan build of them
HOST_FUNCS = ("s2h_prompt_objects", "s2h_prompt_object_masks", "s2h_mask_moments")


def host_lib():
    """library holding the host-only prompt-stage entry points: libsam2hip.so, or the build named by
    S2H_HOST_LIB_PATH (sanitizer runs)"""
    global _HOST_LIB
    path = os.environ.get("S2H_HOST_LIB_PATH")
    if not path:
        return lib()
    if _HOST_LIB is None:
        h = ctypes.CDLL(path)
        for name in HOST_FUNCS:
            fn = getattr(h, name)
            fn.argtypes = SIGNATURES[name]
            fn.restype = c_int
        _HOST_LIB = h
    return _HOST_LIB


def host_call(name, *args):
    rc = getattr(host_lib(), name)(*args)
    if rc != 0:
        raise HipKernelError(f"{name} failed with error {rc}")
    return rc


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise HipKernelError(f"{name} failed with hipError {rc}")
    return rc
