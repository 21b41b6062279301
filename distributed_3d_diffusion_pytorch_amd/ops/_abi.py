"""ctypes signatures of the C ABI exported by ``libd3d_hip.so``
(sources in ``ops/csrc/*.hip``).  Pointers are passed as integers
(``tensor.data_ptr()``), streams as the raw ``hipStream_t`` handle."""
from __future__ import annotations

import ctypes as C

P = C.c_void_p
I = C.c_int
L = C.c_long
F = C.c_float
U64 = C.c_ulonglong
IP = C.POINTER(C.c_int)

SIGNATURES = {
    # norm.hip
    "d3d_gn_plan": [I, I, I, IP, IP],
    "d3d_gn_cfg": [I, I, I],
    "d3d_gn_cfg_small": [I, I],
    "d3d_gn_stats": [P, I, I, I, I, F, P, P, P, I, P],
    "d3d_gn_apply": [P, P, P, P, P, I, I, I, I, I, P],
    "d3d_gn_film": [P, P, P, P, P, P, I, I, I, I, F, U64, I, P, P],
    "d3d_gn_bwd": [I, P, P, P, P, P, P, I, I, I, I, F, U64, P, P, P, P, P, P, P, P],
    "d3d_ray_dir": [P, P, P, P, I, I, I, I, P],
    "d3d_border_fix": [P, P, I, I, I, I, I, I, I, P, P],
    "d3d_border_sums": [P, P, I, I, I, I, P],
    "d3d_gn_apply2": [I, P, P, P, P, P, P, P, I, I, I, I, F, F, U64, I, P, P, I, I, P, P],
    "d3d_set_words64": [P, I, C.c_longlong, C.c_longlong, C.c_longlong, P],
    "d3d_sgemm_jobs": [P, I, I, P],
    "d3d_gn_ab": [P, P, P, P, P, I, I, I, I, F, I, P],
    "d3d_gn_ab_silu": [P, P, P, I, I, I, P],
    "d3d_gn_img_cfg": [I],
    "d3d_gn_img_ok": [I, I, I],
    "d3d_gn_img_ok_n": [I, I, I, I],
    "d3d_gn_img_wide_cfg": [I, I],
    "d3d_gn_img_fwd": [I, P, P, P, P, P, P, I, I, I, I, F, F, U64, I, P, P, I, P, P],
    "d3d_gn_img_bwd": [I, P, P, P, P, P, P, I, I, I, I, F, U64, P, P, P, I, P, P, P, I, P, F, P, F, P],
    "d3d_gn_bwd2": [I, P, P, P, P, P, P, I, I, I, I, F, U64, P, P, P, P, P, P, P, I, I, P, P, P, I, P, F, P, F, P],
    "d3d_conv_s64_cfg": [I],
    "d3d_conv_hsm_cfg": [I],
    "d3d_gemm_small_k": [I],
    "d3d_gemm_mf": [I],
    "d3d_gemm_w8_waves": [I],
    "d3d_attn_bwd_cfg": [I],
    "d3d_attn_fwd_cfg": [I],
    "d3d_colsum_jobs": [P, I, P],
    "d3d_conv_halo_cfg": [I],
    "d3d_conv_res_cfg": [I],
    # elementwise.hip
    "d3d_period_sum": [P, P, I, L, P],
    "d3d_silu": [P, P, L, P],
    "d3d_dsilu": [P, P, P, L, P],
    "d3d_avgpool2": [P, P, I, I, I, I, I, P],
    "d3d_upsample2": [P, P, I, I, I, I, I, P],
    "d3d_add_scale": [P, P, P, F, L, P],
    "d3d_set_words": [P, I, F, F, F, F, F, F, F, F, P],
    "d3d_add_scale_gn": [P, P, P, F, L, I, I, I, P, P],
    "d3d_sampler_step": [P, P, P, P, P, I, I, F, F, F, F, F, I, U64, P],
    "d3d_sampler_inputs": [P, P, I, I, P, P, U64, L, P, P, P],
    "d3d_sampler_step2": [P, P, P, I, I, P, P, U64, L, P],
    "d3d_randn_hash": [P, L, U64, L, P],
    "d3d_diffusion_fwd2": [P, I, I, U64, P, L, F, F, F, P, P, P, P, P],
    "d3d_diff_loss": [P, P, I, I, I, I, P, P, P],
    "d3d_diff_loss_bwd": [P, P, P, I, I, I, I, P, P],
    # adam.hip
    "d3d_adam": [P, P, P, P, P, L, F, F, F, F, F, F, F, F, P],
    "d3d_adam_dev": [P, P, P, P, P, L, P, P],
    # conv.hip
    "d3d_conv3x3": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, P],
    "d3d_conv_wgrad_plan": [I, I, I, I, I, IP, IP],
    "d3d_conv3x3_wgrad": [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, P],
    "d3d_chansum": [P, P, P, P, I, I, I, I, P],
    "d3d_colsum": [P, L, I, P, P, P, I, P],
    "d3d_pack_conv_weight": [P, P, I, I, I, I, I, P],
    "d3d_conv": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, I, P, I, P],
    "d3d_conv2": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, I, P, I, P, I, IP, P],
    "d3d_conv3_gn_ok": [I, I, I, I, I],
    "d3d_conv3_gn": [P, P, P, P, I, I, I, I, I, I, P, I, IP, P, P],
    "d3d_conv3": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, F, I, I, P, I, P, I, IP, P, IP, P],
    "d3d_conv_plan": [I, I, I, I, I, I],
    "d3d_set_conv_korder": [I],
    "d3d_set_wgrad_impl": [I],
    "d3d_conv_wgrad_plan2": [I, I, I, I, I, I, IP, IP],
    "d3d_conv_wgrad_plan3": [I, I, I, I, I, I, I, I, I, IP, IP],
    "d3d_conv_wgrad": [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P],
    "d3d_pack_weight": [P, P, I, I, I, I, I, I, P],
    "d3d_set_conv_impl": [I, P],
    "d3d_pack_all": [P, P, I, P],
    "d3d_conv_wgrad_cat": [P, P, P, I, P, P, P, I, I, I, I, I, I, P],
    "d3d_conv_wgrad_seg": [P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, P],
    "d3d_wgrad_scatter": [P, I, I, I, I, P, I, I, P, P, P, P],
    "d3d_conv_wgrad2": [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P],
    "d3d_conv_wgrad3": [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, F, P],
    # rays.hip
    "d3d_ray_posenc": [P, P, P, P, P, P, P, P, I, I, I, P],
    "d3d_cond_prep": [P, P, P, I, C.c_double, C.c_double, P, P, P, P],
    # attention.hip
    "d3d_attn_fwd": [P, P, P, I, I, I, I, I, F, P],
    "d3d_adam_fused": [P, P, P, P, P, P, P, P, I, P, P, I, I, P],
    # mlp.hip
    "d3d_mlp_ws": [I, I, I],
    "d3d_mlp_pe": [P, I, I, F, P, P],
    "d3d_mlp_mm": [P, P, I, I, I, I, I, I, P, P, P, P, P],
    "d3d_mlp_wgrad": [P, P, I, I, I, I, P, P, I, P],
    "d3d_gemm": [P, P, P, P, I, P, I, I, I, I, I, I, I, F, F, P, I, I, I, P],
    "d3d_gemm_cat": [P, P, P, I, P, P, I, I, I, I, I, F, F, P],
    # small_gemm.hip
    "d3d_sgemm_strided": [P, P, P, I, I, I, I, L, L, L, L, L, L, L, L, L, F, F, P],
    # wgrad_gemm.hip
    "d3d_wgrad_tn_plan": [I, I, L, I, I],
    "d3d_wgrad_tn": [P, P, P, P, I, I, L, I, I, I, P],
    "d3d_wgrad_tn_tune": [I],
    "d3d_gemm_nt_ok": [I, I, I, I, I],
    "d3d_gemm_tune": [I, I, I],
    "d3d_gemm_nt": [P, P, P, P, P, I, I, I, I, I, I, I, F, F, P],
    "d3d_gemm_nt_gn": [P, P, P, P, P, I, I, I, I, I, I, I, F, F, P, I, I, P],
    "d3d_attn_bwd": [P, P, P, P, P, P, I, I, I, I, I, F, P],
    "d3d_attn_bwd_slabs": [I, I, I, I],
    # wgrad_group.hip (job tables: arrays of hip_impl._WgJob)
    "d3d_wgrad_group_cfg": [I, I, I],
    "d3d_wgrad_group_ok": [P],
    "d3d_wgrad_group_stages": [I],
    "d3d_wgrad_group_halo": [I, I, I],
    "d3d_wgrad_group_halo_big": [I, I],
    "d3d_wgrad_group_halo_pk": [I],
    "d3d_wgrad_group_engine": [P],
    "d3d_wgrad_group": [P, I, P, L, P],
    "d3d_wgrad_group_plan": [P, I, IP, IP, C.POINTER(C.c_long)],
}


def declare(lib: C.CDLL) -> None:
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:          # an older build (A/B runs via D3D_LIB_PATH): calls fail when made
            continue
        fn.argtypes = args
        fn.restype = C.c_long if name in RET_LONG else C.c_int


RET_LONG = {"d3d_mlp_ws", "d3d_wgrad_group"}
