"""ctypes binding of libencdiff_hip.so (include/encdiff_hip.h).

The library is loaded after torch so that it binds to the HIP runtime torch has
already mapped (same SONAME libamdhip64.so.7).  There is no fallback: if the
library is missing or a symbol is absent, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (load torch's HIP runtime first)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ENCDIFF_LIB", os.path.join(HERE, "libencdiff_hip.so"))

# enums (mirror include/encdiff_hip.h)
OPA_ROWK, OPA_IM2COL, OPA_ROWM = 0, 1, 2
OPB_ROWK, OPB_ROWN, OPB_CONV_DGRAD, OPB_IM2COL = 0, 1, 2, 3
DT_BF16, DT_F32 = 0, 1  # EncdiffGemmArgs / GroupNorm / LayerNorm / Attn / Ew .dtype
OUT_BF16, OUT_F32, OUT_F32_ATOMIC, OUT_F32_ATOMIC_CONVW, OUT_F32_ACCUM, OUT_BF16_GEGLU, OUT_BF16_GEGLU_BWD = \
    0, 1, 2, 3, 4, 5, 6
RESAMPLE_NONE, RESAMPLE_DOWN2, RESAMPLE_UP2, RESAMPLE_STRIDE2, RESAMPLE_K4S2, RESAMPLE_K4S2_T, RESAMPLE_K4S2_TP = \
    0, 1, 2, 3, 4, 5, 6
(EW_COPY, EW_SILU, EW_SILU_BWD, EW_GEGLU, EW_GEGLU_BWD, EW_ADD, EW_RESAMPLE, EW_RESAMPLE_BWD,
 EW_F32_TO_BF16, EW_BF16_TO_F32) = range(10)

vp = C.c_void_p


class ConvGeom(C.Structure):
    _fields_ = [("batch", C.c_int), ("h", C.c_int), ("w", C.c_int), ("cin", C.c_int),
                ("resample", C.c_int), ("pad_", C.c_int), ("ld_src", C.c_long)]


class GemmArgs(C.Structure):
    _fields_ = [("M", C.c_int), ("N", C.c_int), ("K", C.c_int),
                ("a_mode", C.c_int), ("b_mode", C.c_int), ("c_mode", C.c_int),
                ("a", vp), ("lda", C.c_long), ("b", vp), ("ldb", C.c_long), ("c", vp), ("ldc", C.c_long),
                ("conv", ConvGeom), ("conv_cout", C.c_int), ("convw_cin", C.c_int),
                ("alpha", C.c_float), ("split_k", C.c_int),
                ("bias", vp), ("resid", vp), ("ld_resid", C.c_long), ("bias_grad", vp),
                ("tile", C.c_int), ("dtype", C.c_int), ("workspace", vp),
                ("aux", vp), ("ld_aux", C.c_long), ("gn_stats", vp), ("ld_gn_stats", C.c_long),
                ("ln_gamma", vp), ("ln_beta", vp), ("ln_y", vp), ("ld_ln_y", C.c_long), ("ln_stats", vp),
                ("ln_eps", C.c_float), ("pad3_", C.c_int), ("split_counters", vp),
                ("agn_gamma", vp), ("agn_beta", vp), ("agn_film", vp), ("ld_agn_film", C.c_long),
                ("agn_eps", C.c_float), ("agn_silu", C.c_int),
                ("lna_gamma", vp), ("lna_beta", vp), ("lna_eps", C.c_float)]


class GroupNormArgs(C.Structure):
    _fields_ = [("batch", C.c_int), ("hw", C.c_int), ("c", C.c_int), ("groups", C.c_int),
                ("eps", C.c_float), ("silu", C.c_int),
                ("x", vp), ("ldx", C.c_long), ("gamma", vp), ("beta", vp),
                ("film", vp), ("ld_film", C.c_long), ("y", vp), ("ldy", C.c_long), ("stats", vp),
                ("dy", vp), ("lddy", C.c_long), ("dx", vp), ("lddx", C.c_long),
                ("accumulate_dx", C.c_int), ("dtype", C.c_int),
                ("dgamma_part", vp), ("dbeta_part", vp), ("ld_part", C.c_long), ("dfilm", vp),
                ("ld_dfilm", C.c_long), ("resid", vp), ("ld_resid", C.c_long), ("in_stats", vp),
                ("ld_in_stats", C.c_long), ("x_from", vp), ("dy_resample", C.c_int), ("resid_resample", C.c_int),
                ("w", C.c_int), ("pad_rs_", C.c_int), ("dsilu", vp), ("ld_dsilu", C.c_long),
                ("fold_plan", vp), ("fold_blocks", C.c_int), ("pad_fold_", C.c_int)]


class LayerNormArgs(C.Structure):
    _fields_ = [("rows", C.c_int), ("c", C.c_int), ("eps", C.c_float),
                ("x", vp), ("ldx", C.c_long), ("gamma", vp), ("beta", vp), ("y", vp), ("ldy", C.c_long),
                ("stats", vp), ("dy", vp), ("lddy", C.c_long), ("dx", vp), ("lddx", C.c_long),
                ("accumulate_dx", C.c_int), ("dgamma_part", vp), ("dbeta_part", vp), ("ld_part", C.c_long),
                ("parts", C.c_int), ("dtype", C.c_int), ("resid", vp), ("ld_resid", C.c_long),
                ("dy_from", vp)]


class AttnArgs(C.Structure):
    _fields_ = [("batch", C.c_int), ("heads", C.c_int), ("sq", C.c_int), ("sk", C.c_int), ("dh", C.c_int),
                ("scale", C.c_float),
                ("q", vp), ("ldq", C.c_long), ("k", vp), ("ldk", C.c_long), ("v", vp), ("ldv", C.c_long),
                ("o", vp), ("ldo", C.c_long), ("lse", vp),
                ("d_o", vp), ("lddo", C.c_long), ("dq", vp), ("lddq", C.c_long),
                ("dk", vp), ("lddk", C.c_long), ("dv", vp), ("lddv", C.c_long), ("fp8_qk", C.c_int),
                ("dtype", C.c_int)]


class EwArgs(C.Structure):
    _fields_ = [("op", C.c_int), ("rows", C.c_int), ("cols", C.c_int),
                ("x", vp), ("ldx", C.c_long), ("x2", vp), ("ldx2", C.c_long), ("y", vp), ("ldy", C.c_long),
                ("accumulate", C.c_int), ("resample", C.c_int), ("batch", C.c_int), ("h", C.c_int),
                ("w", C.c_int), ("dtype", C.c_int)]


class SmallConvArgs(C.Structure):
    _fields_ = [("batch", C.c_int), ("h", C.c_int), ("w", C.c_int), ("cin", C.c_int), ("cout", C.c_int),
                ("x", vp), ("ldx", C.c_long), ("x_f32", C.c_int), ("weight", vp), ("bias", vp),
                ("y", vp), ("ldy", C.c_long), ("y_f32", C.c_int), ("pad_", C.c_int),
                ("dy", vp), ("lddy", C.c_long), ("dy_f32", C.c_int), ("pad2_", C.c_int),
                ("dx", vp), ("lddx", C.c_long), ("dweight", vp), ("dbias", vp)]


class BatchNormArgs(C.Structure):
    _fields_ = [("rows", C.c_int), ("c", C.c_int), ("eps", C.c_float), ("momentum", C.c_float),
                ("relu", C.c_int), ("x_f32", C.c_int), ("x", vp), ("ldx", C.c_long), ("gamma", vp), ("beta", vp),
                ("y", vp), ("ldy", C.c_long), ("mean", vp), ("rstd", vp), ("running_mean", vp), ("running_var", vp),
                ("partials", vp), ("counter", vp), ("dy", vp), ("lddy", C.c_long), ("dx", vp), ("lddx", C.c_long),
                ("dgamma", vp), ("dbeta", vp), ("y_split", C.c_int), ("pad2_", C.c_int)]


class StTailArgs(C.Structure):
    _fields_ = [("rows", C.c_int), ("c", C.c_int), ("tokens", C.c_int), ("heads", C.c_int), ("n_ctx", C.c_int),
                ("ln_eps", C.c_float), ("scale", C.c_float), ("pad_", C.c_int),
                ("o1", vp), ("ld_o1", C.c_long), ("t0", vp), ("ld_t0", C.c_long), ("x", vp), ("ld_x", C.c_long),
                ("k2", vp), ("v2", vp), ("ld_kv", C.c_long),
                ("w_out1", vp), ("ld_out1", C.c_long), ("b_out1", vp), ("g2", vp), ("be2", vp),
                ("w_q2", vp), ("ld_q2", C.c_long), ("w_out2", vp), ("ld_out2", C.c_long), ("b_out2", vp),
                ("g3", vp), ("be3", vp), ("w_ff1", vp), ("ld_ff1", C.c_long), ("b_ff1", vp),
                ("w_ff2", vp), ("ld_ff2", C.c_long), ("b_ff2", vp), ("w_po", vp), ("ld_po", C.c_long), ("b_po", vp),
                ("out", vp), ("ld_out", C.c_long),
                ("save_t1", vp), ("save_n2", vp), ("save_q2", vp), ("save_o2", vp), ("save_t2", vp),
                ("save_n3", vp), ("save_f", vp), ("save_a", vp), ("save_t3", vp), ("ld_save", C.c_long),
                ("save_s2", vp), ("save_s3", vp), ("save_lse2", vp), ("gn_stats", vp), ("ld_gn_stats", C.c_long),
                ("gn_stats_add", C.c_int), ("pad2_", C.c_int), ("head_t2", vp), ("head_n3", vp),
                ("ld_head", C.c_long)]


class StHeadArgs(C.Structure):
    _fields_ = [("rows", C.c_int), ("c", C.c_int), ("tokens", C.c_int), ("pad_", C.c_int),
                ("gn_eps", C.c_float), ("ln_eps", C.c_float), ("x", vp), ("ld_x", C.c_long),
                ("gn_in_stats", vp), ("ld_gn_in_stats", C.c_long), ("gn_gamma", vp), ("gn_beta", vp),
                ("gn", vp), ("ld_gn", C.c_long), ("gn_stats", vp), ("w_in", vp), ("ld_in", C.c_long), ("b_in", vp),
                ("g1", vp), ("be1", vp), ("w_qkv", vp), ("ld_w_qkv", C.c_long), ("t0", vp), ("ld_t0", C.c_long),
                ("n1", vp), ("ld_n1", C.c_long), ("s1", vp), ("qkv", vp), ("ld_qkv", C.c_long)]


class StTailBwdArgs(C.Structure):
    _fields_ = [("rows", C.c_int), ("c", C.c_int), ("tokens", C.c_int), ("heads", C.c_int), ("n_ctx", C.c_int),
                ("scale", C.c_float), ("part_rows", C.c_int), ("pad_", C.c_int),
                ("dy", vp), ("ld_dy", C.c_long), ("f", vp), ("ld_f", C.c_long),
                ("t2", vp), ("t1", vp), ("q2", vp), ("o2", vp), ("ld_save", C.c_long),
                ("s3", vp), ("s2", vp), ("lse2", vp), ("k2", vp), ("v2", vp), ("ld_kv", C.c_long),
                ("w_po_t", vp), ("w_ff2_t", vp), ("w_ff1_t", vp), ("w_out2_t", vp), ("w_q2_t", vp), ("w_out1_t", vp),
                ("g3", vp), ("g2", vp),
                ("d_t3", vp), ("d_t2", vp), ("d_q2", vp), ("d_t1", vp), ("d_o1", vp), ("ld_d", C.c_long),
                ("d_f", vp), ("ld_df", C.c_long),
                ("ln3_dg", vp), ("ln3_db", vp), ("ln2_dg", vp), ("ln2_db", vp), ("ld_part", C.c_long),
                ("dk2", vp), ("dv2", vp), ("ld_dkv", C.c_long), ("kv_part", vp)]


class StHeadBwdArgs(C.Structure):
    _fields_ = [("rows", C.c_int), ("c", C.c_int), ("part_rows", C.c_int), ("pad_", C.c_int),
                ("d_qkv", vp), ("ld_dqkv", C.c_long), ("d_t1", vp), ("ld_dt1", C.c_long),
                ("t0", vp), ("ld_t0", C.c_long), ("s1", vp), ("g1", vp), ("w_qkv_t", vp), ("w_in_t", vp),
                ("d_t0", vp), ("ld_dt0", C.c_long), ("d_gn", vp), ("ld_dgn", C.c_long),
                ("ln1_dg", vp), ("ln1_db", vp), ("ld_part", C.c_long),
                ("kv_part", vp), ("kv_tiles", C.c_int), ("n_ctx", C.c_int), ("batch", C.c_int), ("pad2_", C.c_int),
                ("dk2", vp), ("dv2", vp), ("ld_dkv", C.c_long)]


class WgradProb(C.Structure):
    _fields_ = [("dy", vp), ("ld_dy", C.c_long), ("x", vp), ("ld_x", C.c_long), ("dw", vp), ("ld_dw", C.c_long),
                ("db", vp), ("M", C.c_int), ("N", C.c_int), ("K", C.c_int), ("pad_", C.c_int)]


class ResConvArgs(C.Structure):
    _fields_ = [("batch", C.c_int), ("h", C.c_int), ("cin", C.c_int), ("cout", C.c_int), ("resample", C.c_int),
                ("groups", C.c_int), ("silu", C.c_int), ("eps", C.c_float), ("x", vp), ("ld_x", C.c_long),
                ("gamma", vp), ("beta", vp), ("film", vp), ("ld_film", C.c_long), ("w", vp), ("ld_w", C.c_long),
                ("bias", vp), ("resid", vp), ("ld_resid", C.c_long), ("resid_resample", C.c_int), ("cskip", C.c_int),
                ("xskip", vp), ("ld_xskip", C.c_long), ("wskip", vp), ("ld_wskip", C.c_long), ("bskip", vp),
                ("y", vp), ("ld_y", C.c_long), ("tile_m", C.c_int), ("tile_n", C.c_int),
                ("skip_stages", C.c_int), ("pad_", C.c_int)]


class ZeroJob(C.Structure):
    _fields_ = [("ptr", vp), ("rows", C.c_longlong), ("row_bytes", C.c_longlong), ("ld_bytes", C.c_longlong)]


class StepPrologueArgs(C.Structure):
    _fields_ = [("jobs", vp), ("njobs", C.c_int), ("batch", C.c_int), ("timesteps", C.c_int), ("pad_", C.c_int),
                ("seed", C.c_ulonglong), ("rng_counter", vp), ("data_step", vp), ("t", vp), ("noise", vp),
                ("n_noise", C.c_longlong), ("done", vp), ("pad2_", C.c_int)]


class PackJob(C.Structure):
    _fields_ = [("src_off", C.c_longlong), ("dst_off", C.c_longlong), ("rows", C.c_int), ("cols", C.c_int),
                ("kind", C.c_int), ("cin", C.c_int)]


_PROTOS = {
    "encdiff_gemm": [C.POINTER(GemmArgs), vp],
    "encdiff_gemm_pair": [C.POINTER(GemmArgs), C.POINTER(GemmArgs), vp],
    "encdiff_gemm_pair_ex": [C.POINTER(GemmArgs), C.POINTER(GemmArgs), C.POINTER(GemmArgs), C.c_int, vp],
    "encdiff_gemm_finalize": [C.POINTER(GemmArgs), vp],
    "encdiff_wgrad_group_plan": [C.POINTER(GemmArgs), C.c_int, vp, C.c_long, vp, C.c_int, vp, C.c_long,
                                 C.POINTER(C.c_long)],
    "encdiff_wgrad_group_launch": [vp, vp, vp],
    "encdiff_gemm_ex": [C.POINTER(GemmArgs), C.c_int, C.POINTER(C.c_int), vp],
    "encdiff_gemm_pair_dx": [C.POINTER(GemmArgs), C.POINTER(GemmArgs), C.POINTER(GemmArgs), C.c_int, C.c_int,
                             C.POINTER(C.c_int), vp],
    "encdiff_groupnorm_fwd": [C.POINTER(GroupNormArgs), vp],
    "encdiff_groupnorm_bwd": [C.POINTER(GroupNormArgs), vp],
    "encdiff_layernorm_fwd": [C.POINTER(LayerNormArgs), vp],
    "encdiff_layernorm_bwd": [C.POINTER(LayerNormArgs), vp],
    "encdiff_attention_fwd": [C.POINTER(AttnArgs), vp],
    "encdiff_attention_bwd": [C.POINTER(AttnArgs), vp],
    "encdiff_elementwise": [C.POINTER(EwArgs), vp],
    "encdiff_small_conv_fwd": [C.POINTER(SmallConvArgs), vp],
    "encdiff_small_conv_bwd": [C.POINTER(SmallConvArgs), vp],
    "encdiff_timestep_embedding": [vp, C.c_int, C.c_int, C.c_float, vp, vp],
    "encdiff_timestep_embedding_f32": [vp, C.c_int, C.c_int, C.c_float, vp, vp],
    "encdiff_nchw_rows_f32": [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_long, C.c_int, vp],
    "encdiff_q_sample": [vp, vp, vp, vp, vp, C.c_int, C.c_int, vp, vp],
    "encdiff_q_sample_scaled": [vp, vp, vp, vp, vp, vp, C.c_int, C.c_int, vp, vp],
    "encdiff_l1_loss": [vp, vp, vp, vp, C.c_int, C.c_int, C.c_float, vp, vp, vp, vp, vp],
    "encdiff_ddim_step": [vp, vp, vp, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, vp, vp, vp],
    "encdiff_ddim_step_indexed": [vp, vp, vp, C.c_int, vp, vp, C.c_int, vp, vp, vp],
    "encdiff_adamw_ema": [vp, vp, vp, vp, vp, C.c_longlong, vp, C.c_longlong, vp],
    "encdiff_adamw_ema_mirror": [vp, vp, vp, vp, vp, C.c_longlong, vp, C.c_longlong, vp, vp],
    "encdiff_pack_weights": [vp, vp, vp, C.c_int, vp],
    "encdiff_reduce_partials": [vp, C.c_long, C.c_int, C.c_int, vp, vp, vp],
    "encdiff_grad_fold": [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp],
    "encdiff_encoder_warp_fwd": [vp, C.c_long, C.c_int, C.c_int, vp, C.c_long, C.c_int, vp, C.c_long, vp],
    "encdiff_encoder_warp_bwd": [vp, C.c_long, C.c_int, C.c_int, vp, C.c_long, C.c_int, vp, C.c_long, vp, C.c_long,
                                 vp, vp, vp],
    "encdiff_encoder_warp_partials_floats": [C.c_int, C.c_int, C.c_long],
    "encdiff_encoder_head_fwd": [vp, C.c_long, C.c_int, C.c_int, vp, vp, C.c_int, vp, C.c_long, vp],
    "encdiff_encoder_head_bwd": [vp, C.c_long, C.c_int, C.c_int, vp, C.c_int, vp, C.c_long, vp, C.c_long, vp, vp,
                                 vp],
    "encdiff_gather_images_u8": [vp, C.c_longlong, C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, C.c_int, C.c_int,
                                 vp, vp],
    "encdiff_batchnorm_partials_floats": [C.c_int, C.c_int],
    "encdiff_batchnorm_fwd": [C.POINTER(BatchNormArgs), vp],
    "encdiff_batchnorm_bwd": [C.POINTER(BatchNormArgs), vp],
    "encdiff_batchnorm_apply": [C.POINTER(BatchNormArgs), vp],
    "encdiff_nchw_to_rows": [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_long, vp],
    "encdiff_nchw_to_rows_split3": [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_long, vp],
    "encdiff_st_tail_fwd": [C.POINTER(StTailArgs), vp],
    "encdiff_st_head_fwd": [C.POINTER(StHeadArgs), vp],
    "encdiff_st_tail_bwd": [C.POINTER(StTailBwdArgs), vp],
    "encdiff_st_head_bwd": [C.POINTER(StHeadBwdArgs), vp],
    "encdiff_st_tail_bwd_tile": [C.c_int, C.c_int, C.c_int],
    "encdiff_st_wgrad_plan": [vp, C.c_int, vp, C.c_long, vp, C.c_long, vp],
    "encdiff_st_wgrad_launch": [vp, vp, vp],
    "encdiff_st_wgrad_launch_nofold": [vp, vp, vp, C.POINTER(vp), C.POINTER(C.c_int)],
    "encdiff_resconv_fwd": [C.POINTER(ResConvArgs), vp],
    "encdiff_resconv_query": [C.POINTER(ResConvArgs), C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "encdiff_step_prologue": [C.POINTER(StepPrologueArgs), vp],
    "encdiff_version": [],
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libencdiff_hip.so not built ({LIB_PATH}); run encdiff_amd.build.build() / "
                          f"__graft_entry__.build()")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, args in _PROTOS.items():
        fn = getattr(lib, name)  # AttributeError == missing export: fail loudly
        fn.argtypes = args
        fn.restype = C.c_int
    return lib


lib = _load()
EXPORTS = tuple(_PROTOS)


class HipError(RuntimeError):
    pass


_ERRS = {-1: "ENCDIFF_ERR_ARG", -2: "ENCDIFF_ERR_SHAPE", -3: "ENCDIFF_ERR_UNSUPPORTED"}


def check(rc: int, what: str):
    if rc != 0:
        if rc <= -1000:
            raise HipError(f"{what}: HIP launch failure (hipError_t {-1000 - rc})")
        raise HipError(f"{what}: {_ERRS.get(rc, rc)}")
