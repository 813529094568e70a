"""ctypes binding of libvclip.so (include/vclip.h).

The product path has no fallback: if the library is missing or a call fails, an
exception is raised.  torch is imported before the library is opened so that the
process holds one HIP runtime (the one torch loaded; see build.py).
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  (must precede dlopen of libvclip.so: one HIP runtime per process)

from .build import LIB_PATH, INCLUDE

_lib = None

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_f = ctypes.c_float
c_p = ctypes.c_void_p

# name -> argtypes (restype int unless noted); mirrors include/vclip.h
SIGNATURES = {
    "vc_version": ([], ctypes.c_char_p),
    "vc_last_error": ([], ctypes.c_char_p),
    "vc_frame_gather": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_int, c_f, c_f, c_p, c_p], c_int),
    "vc_tubelet_im2col": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_p, c_i64, c_p], c_int),
    "vc_patch_im2col": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_int, c_int, c_p, c_i64, c_p],
                        c_int),
    "vc_layernorm_f32": ([c_p, c_i64, c_i64, c_i64, c_p, c_p, c_f, c_p, c_i64, c_p], c_int),
    "vc_gemm_bf16": ([c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_int, c_p, c_i64, c_p, c_i64,
                      c_i64, c_i64, c_i64, c_p], c_int),
    "vc_gemm_bf16_cfg": ([c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_int, c_p, c_i64, c_p, c_i64,
                          c_i64, c_i64, c_i64, c_int, c_p], c_int),
    "vc_layernorm_f32_bf16": ([c_p, c_i64, c_i64, c_i64, c_p, c_p, c_f, c_p, c_i64, c_p], c_int),
    "vc_attention_fwd": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_int, c_p, c_i64, c_p], c_int),
    "vc_attention_fwd_rebase_always": ([c_p, c_i64, c_i64, c_i64, c_i64, c_f, c_p, c_i64, c_p], c_int),
    "vc_patch_im2col_h16": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_int, c_int, c_int, c_p,
                             c_i64, c_p], c_int),
    "vc_gemm_pick": ([c_i64, c_i64, c_i64, c_int, c_i64, c_i64, c_p], c_int),
    "vc_gemm_h16_wrap": ([c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_int, c_p, c_i64, c_p, c_i64,
                          c_i64, c_i64, c_i64, c_int, c_p], c_int),
    "vc_patch_im2col_split_h16": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_int, c_int, c_int,
                                   c_p, c_i64, c_p], c_int),
    "vc_gemm_h16": ([c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_int, c_p, c_i64, c_p, c_i64,
                     c_i64, c_i64, c_i64, c_int, c_int, c_p], c_int),
    "vc_layernorm_f32_h16": ([c_p, c_i64, c_i64, c_i64, c_p, c_p, c_f, c_int, c_p, c_i64, c_p], c_int),
    "vc_attention_fwd_h16": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_int, c_int, c_p, c_i64, c_p], c_int),
    "vc_spin": ([c_i64, c_i64, c_p], c_int),
    "vc_cls_init": ([c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p], c_int),
    "vc_cls_head": ([c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_f, c_p, c_p, c_i64, c_p, c_p], c_int),
    "vc_temporal_attention": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_int, c_p, c_i64, c_p], c_int),
    "vc_window_attention3d": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_int, c_int,
                               c_int, c_p, c_i64, c_p, c_i64, c_p], c_int),
    "vc_window_attention3d_mb": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_int, c_int,
                               c_int, c_p, c_i64, c_p, c_i64, c_p], c_int),
    "vc_window_attention3d_lse": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int, c_int,
                                   c_int, c_int, c_p, c_i64, c_p, c_i64, c_p, c_p], c_int),
    "vc_window_attention3d_bwd": ([c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                   c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_i64,
                                   c_p, c_p], c_int),
    "vc_patch_merge_layernorm": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_f, c_p, c_i64, c_p], c_int),
    "vc_pool_head": ([c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_f, c_p, c_p, c_i64, c_p, c_p, c_p], c_int),
    "vc_pool_head_pooled": ([c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_f, c_p, c_p, c_i64, c_p, c_p, c_p, c_p],
                            c_int),
    "vc_pool_head_bwd": ([c_p, c_p, c_p, c_i64, c_i64, c_i64, c_f, c_p, c_p, c_p, c_p], c_int),
    "vc_conv3d_im2col": ([c_p, c_i64, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p], c_int),
    "vc_conv3d_gemm_bf16": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64,
                             c_p, c_int, c_p, c_i64, c_p, c_i64, c_p], c_int),
    "vc_conv3d_gemm_bf16_ring": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64,
                                  c_p, c_int, c_p, c_i64, c_p, c_i64, c_int, c_p], c_int),
    "vc_conv3d_gemm_bf16_cfg": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64,
                                 c_p, c_int, c_p, c_i64, c_p, c_i64, c_int, c_int, c_p], c_int),
    "vc_conv3d_stem_pack": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p], c_int),
    "vc_conv3d_stem_gemm_bf16": ([c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_p, c_int,
                                  c_p, c_i64, c_p], c_int),
    "vc_maxpool3d": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p], c_int),
    "vc_avgpool_head": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_i64, c_p, c_p, c_p], c_int),
    "vc_col2im_cl": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p], c_int),
    "vc_maxpool3d_bwd": ([c_p, c_i64, c_p, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64,
                          c_p], c_int),
    "vc_batchnorm_train_fwd": ([c_p, c_i64, c_i64, c_i64, c_p, c_p, c_f, c_f, c_p, c_p, c_p, c_int, c_i64, c_int, c_p,
                                c_i64, c_p, c_p, c_i64, c_p], c_int),
    "vc_batchnorm_train_bwd": ([c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_i64, c_p, c_i64, c_int, c_p, c_i64, c_p,
                                c_i64, c_p, c_p, c_p, c_i64, c_p], c_int),
    "vc_resnet_head_train": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_p, c_p, c_p, c_i64, c_p, c_p, c_p],
                             c_int),
    "vc_resnet_head_train_bwd": ([c_p, c_i64, c_i64, c_i64, c_i64, c_int, c_p, c_p, c_i64, c_p], c_int),
    "vc_resample_u8": ([c_p, c_i64, c_i64, c_i64, c_i64, c_int, c_i64, c_p, c_p, c_i64, c_p, c_p], c_int),
    "vc_resize_linear_u8": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_int, c_p, c_p], c_int),
    "vc_video_transform": ([c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p,
                            c_p, c_int, c_int, c_p, c_p], c_int),
    "vc_video_transform_clips": ([c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_p, c_p, c_int,
                                  c_int, c_p, c_p], c_int),
    "vc_divided_add_layernorm": ([c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_f, c_int, c_p,
                                  c_i64, c_p], c_int),
    # train step
    "vc_attention_fwd_lse": ([c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_int, c_p, c_i64, c_p, c_p], c_int),
    "vc_attention_bwd": ([c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p],
                         c_int),
    "vc_attention_bwd_2s": ([c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p,
                             c_p], c_int),
    "vc_layernorm_bwd": ([c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_f, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p,
                          c_p, c_i64, c_p], c_int),
    "vc_colsum": ([c_p, c_int, c_i64, c_i64, c_i64, c_i64, c_f, c_p, c_p, c_i64, c_p], c_int),
    "vc_wgrad_bf16": ([c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_f, c_p, c_i64, c_p, c_i64, c_p], c_int),
    "vc_wgrad_pick": ([c_i64, c_i64, c_i64, c_i64], c_int),
    "vc_cls_head_bwd": ([c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_f, c_p, c_i64, c_p, c_p, c_i64, c_p, c_i64, c_p,
                         c_p, c_p, c_p, c_p], c_int),
    "vc_embed_bwd": ([c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_i64, c_p], c_int),
    "vc_adamw_multi": ([c_p, c_i64, c_i64, c_f, c_f, c_f, c_f, c_f, c_i64, c_f, c_p], c_int),
    "vc_adamw": ([c_p, c_p, c_p, c_p, c_i64, c_f, c_f, c_f, c_f, c_f, c_i64, c_f, c_p], c_int),
    "vc_adamw_step_table": ([c_f, c_f, c_f, c_i64, c_p], c_int),
    "vc_adamw_tab": ([c_p, c_p, c_p, c_p, c_i64, c_f, c_f, c_f, c_f, c_f, c_p, c_p, c_i64, c_f, c_p], c_int),
    "vc_adamw_step_tick": ([c_p, c_p], c_int),
    "vc_pack_weight": ([c_p, c_i64, c_i64, c_i64, c_f, c_p, c_p, c_p], c_int),
    # TimeSformer train step
    "vc_temporal_attention_bwd": ([c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p], c_int),
    "vc_gelu_erf": ([c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_p], c_int),
    "vc_gelu_erf_bwd": ([c_p, c_int, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_p], c_int),
}


def header_functions() -> list:
    """Function names declared in include/vclip.h."""
    with open(os.path.join(INCLUDE, "vclip.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(vc_[a-z0-9_]+)\s*\(", txt)))


class VclipError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Open libvclip.so and bind every entry point.  Raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise VclipError(f"libvclip.so not built at {path}: run __graft_entry__.build() "
                         "(the HIP extension is required; there is no CPU fallback)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (argtypes, restype) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = lib
    return lib


def call(name: str, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.vc_last_error().decode(errors="replace")
        raise VclipError(f"{name} failed ({rc}): {msg}")
    return rc
