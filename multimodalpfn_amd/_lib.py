"""ctypes binding of the C-ABI in ``include/mmpfn_hip.h`` (``libmmpfn_hip.so``).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C
multimodalpfn_amd/csrc``).  There is no fallback: if the shared library is missing
or cannot be loaded, every engine entry point raises ``RuntimeError``.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "libmmpfn_hip.so"

MMPFN_OK = 0
MMPFN_MAX_LANES = 8
MMPFN_ERR_INVALID = -1
MMPFN_ERR_HIP = -2
MMPFN_ERR_NAN = -3
MMPFN_ERR_STATE = -4
MMPFN_ERR_WEIGHT = -5

PREC_F32 = 0       # parity mode: split-bf16 three-product MFMAs (fp32 operands to 2^-16), fp32 softmax / LN
PREC_BF16 = 1      # 16-bit mode with bf16 operands on an fp32 state (MMPFN_AUTOCAST=bf16)
PREC_F32_MFMA = 2  # parity mode on fp32-input MFMA (exact fp32 fma chains, 1/16 of the bf16 rate)
PREC_BF16_F8 = 3   # bf16 mode with the sample-axis attention's P.V on fp8 MFMA (P e4m3): config E's fp8 path
PREC_BF16_F8E5 = 4  # the same with P in e5m2
PREC_F16 = 5       # the reference's fp16 autocast: fp16 state between kernels, fp16 MFMA operands, fp32 statistics
PREC_F16_F8 = 6    # PREC_F16 with the fp8 P.V (P e4m3)
PREC_F16_F8E5 = 7  # PREC_F16 with the fp8 P.V (P e5m2)
ATTN_QK_BF16 = 0x100  # mmpfn_item_attention_layer_ex: code 5-7 | this = the fp16 forward's form (bf16 q / k, fp16 out)


def f32_precision() -> int:
    """Engine code of an fp32 forward: PREC_F32, or PREC_F32_MFMA under ``MMPFN_F32_MODE=mfma``."""
    return PREC_F32_MFMA if os.environ.get("MMPFN_F32_MODE", "").lower() == "mfma" else PREC_F32


def precision_of_dtype(dtype) -> int:
    """Engine code of a forced ``inference_precision`` dtype (the reference's ``force_inference_dtype``):
    fp32 / fp64 -> the parity mode; ``torch.float8_e4m3fn`` / ``torch.float8_e5m2`` -> the 16-bit mode with
    the attention's P.V on fp8 MFMA (P in that format); any other dtype -> the 16-bit performance mode."""
    import torch

    if dtype in (torch.float32, torch.float64):
        return f32_precision()
    if dtype == torch.float16:
        return PREC_F16
    if dtype == torch.bfloat16:
        return PREC_BF16
    base = autocast_precision()
    if dtype == torch.float8_e4m3fn:
        return PREC_F16_F8 if base == PREC_F16 else PREC_BF16_F8
    if dtype == torch.float8_e5m2:
        return PREC_F16_F8E5 if base == PREC_F16 else PREC_BF16_F8E5
    return base


def autocast_precision() -> int:
    """Engine code of the reference's GPU default (``inference_precision="auto"``: fp16 autocast,
    utils.py:150-190): PREC_F16 -- fp16 state and operands, 3-8x closer to the fp32 reference than bf16 operands
    and faster -- unless ``MMPFN_AUTOCAST=bf16`` selects PREC_BF16."""
    return PREC_BF16 if os.environ.get("MMPFN_AUTOCAST", "f16").lower() == "bf16" else PREC_F16

MIXER_NONE, MIXER_MGM, MIXER_MGM_CAP, MIXER_MOE = 0, 1, 2, 3
MIXER_CODES = {"MGM": MIXER_MGM, "MGM+CAP": MIXER_MGM_CAP, "MoE": MIXER_MOE, None: MIXER_NONE}


class ModelDesc(ctypes.Structure):
    _fields_ = [
        ("emsize", ctypes.c_int),
        ("nhead", ctypes.c_int),
        ("nlayers", ctypes.c_int),
        ("nhid", ctypes.c_int),
        ("features_per_group", ctypes.c_int),
        ("encoder_features", ctypes.c_int),
        ("n_out", ctypes.c_int),
        ("mixer_type", ctypes.c_int),
        ("mgm_heads", ctypes.c_int),
        ("cap_heads", ctypes.c_int),
        ("two_sets_of_queries", ctypes.c_int),
        ("remove_duplicate_features", ctypes.c_int),
        ("ln_eps", ctypes.c_float),
        ("outlier_sigma", ctypes.c_float),
    ]


# (name, restype, argtypes) of every symbol the header declares
_vp, _i, _i64, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
SIGNATURES = [
    ("mmpfn_create", _vp, [_i, _vp]),
    ("mmpfn_destroy", None, [_vp]),
    ("mmpfn_last_error", ctypes.c_char_p, [_vp]),
    ("mmpfn_set_stream", _i, [_vp, _vp]),
    ("mmpfn_version", ctypes.c_char_p, []),
    ("mmpfn_set_model", _i, [_vp, ctypes.POINTER(ModelDesc)]),
    ("mmpfn_load_weight", _i, [_vp, ctypes.c_char_p, _vp, _i64]),
    ("mmpfn_finalize_weights", _i, [_vp]),
    ("mmpfn_mixer_tokens", _i, [_vp, _i]),
    ("mmpfn_mixer_forward", _i, [_vp, _vp, _i, _i, _vp, _i]),
    ("mmpfn_forward", _i, [_vp, _vp, _i, _i, _vp, _i, _vp, _i, _vp, _i, _vp, _vp, _i]),
    ("mmpfn_embed", _i, [_vp, _vp, _i, _i, _vp, _i, _vp, _i, _vp, _i, _vp, _i]),
    ("mmpfn_run_layers", _i, [_vp, _i, _i]),
    ("mmpfn_decode", _i, [_vp, _vp]),
    ("mmpfn_copy_state", _i, [_vp, _vp, _i64]),
    ("mmpfn_state_tokens", _i, [_vp]),
    ("mmpfn_status", _i, [_vp]),
    ("mmpfn_aggregate", _i, [_vp, _vp, _i, _i, _i, _vp, _i, _f, _i, _vp, _vp]),
    ("mmpfn_item_attention", _i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i]),
    ("mmpfn_item_attention_layer", _i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i]),
    ("mmpfn_item_attention_cached", _i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i]),
    ("mmpfn_item_attention_layer_ex", _i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i]),
    ("mmpfn_select_lane", _i, [_vp, _i]),
    ("mmpfn_forward_batch", _i, [_vp, _i, _vp, _i, _i, _vp, _i, _vp, _i, _vp, _vp, _vp, _vp, _i]),
    ("mmpfn_cache_build", _i, [_vp, _vp, _i, _i, _vp, _i, _vp, _vp, _i, _vp, _i, ctypes.POINTER(_vp)]),
    ("mmpfn_cache_predict", _i, [_vp, _vp, _vp, _i, _i, _vp, _i, _vp]),
    ("mmpfn_cache_bytes", _i64, [_vp]),
    ("mmpfn_cache_free", None, [_vp, _vp]),
    ("mmpfn_kernel_timing", _i, [_vp, _i]),
    ("mmpfn_feature_attention", _i, [_vp, _i, _vp, _i, _i, _i]),
    ("mmpfn_item_attention_block", _i, [_vp, _i, _vp, _i, _i, _i, _i]),
    ("mmpfn_mlp_ln", _i, [_vp, _i, _vp, _i64, _i]),
    ("mmpfn_mgm", _i, [_vp, _vp, _i, _i, _vp, _i]),
    ("mmpfn_cap", _i, [_vp, _vp, _i, _i, _vp, _i]),
    ("mmpfn_kernel_timing_read", _i, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64),
                                      ctypes.POINTER(ctypes.c_double)]),
    ("mmpfn_siphash24_rows", _i, [_vp, _i64, _i64, _vp]),
    ("mmpfn_set_parity_attention_min_keys", _i, [_i, _i]),
]

# include/mmpfn_modality.h (modality encoders: DINOv2 ViT, ELECTRA text tower)
MMPFN_ENC_VIT = 1
MMPFN_ENC_TEXT = 2


class EncDesc(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int),
        ("dim", ctypes.c_int),
        ("depth", ctypes.c_int),
        ("heads", ctypes.c_int),
        ("mlp_hidden", ctypes.c_int),
        ("ln_eps", ctypes.c_float),
        ("patch", ctypes.c_int),
        ("in_chans", ctypes.c_int),
        ("pos_grid", ctypes.c_int),
        ("interp_offset", ctypes.c_double),
        ("layerscale", ctypes.c_int),
        ("vocab", ctypes.c_int),
        ("max_pos", ctypes.c_int),
        ("type_vocab", ctypes.c_int),
        ("embedding_size", ctypes.c_int),
    ]


MODALITY_SIGNATURES = [
    ("mmpfn_enc_create", _vp, [_i, _vp]),
    ("mmpfn_enc_destroy", None, [_vp]),
    ("mmpfn_enc_last_error", ctypes.c_char_p, [_vp]),
    ("mmpfn_enc_set_stream", _i, [_vp, _vp]),
    ("mmpfn_enc_set_model", _i, [_vp, ctypes.POINTER(EncDesc)]),
    ("mmpfn_enc_load_weight", _i, [_vp, ctypes.c_char_p, _vp, _i64]),
    ("mmpfn_enc_finalize", _i, [_vp]),
    ("mmpfn_vit_forward", _i, [_vp, _vp, _i, _i, _i, _vp, _vp, _i]),
    ("mmpfn_text_forward", _i, [_vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _i]),
    ("mmpfn_enc_attention", _i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i]),
]

_LIB = None


def diagnostics_enabled() -> bool:
    """``MMPFN_DIAGNOSTICS=1``: the only way a variant library (an A/B or stamps build) may be loaded."""
    return os.environ.get("MMPFN_DIAGNOSTICS") == "1"


def load_library(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Load ``libmmpfn_hip.so`` (loud failure, no fallback).

    Variant builds (``tools/build_variant*.sh``, ``make dbg``) export ``mmpfn_variant_flags`` and
    are refused unless ``MMPFN_DIAGNOSTICS=1``; so is any library named by ``MMPFN_LIB``.  The product
    path therefore only ever runs the in-tree production build."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    env = os.environ.get("MMPFN_LIB")
    if path is None and env and not diagnostics_enabled():
        raise RuntimeError("MMPFN_LIB names a diagnostics library; set MMPFN_DIAGNOSTICS=1 to load it")
    p = Path(path) if path is not None else Path(env or str(LIB_PATH))
    if not p.exists():
        raise RuntimeError(
            f"MMPFN HIP engine library not found at {p}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (make -C multimodalpfn_amd/csrc)"
        )
    # torch must own the HIP runtime first so both resolve the same libamdhip64.so.7
    import torch  # noqa: F401

    lib = ctypes.CDLL(str(p))
    if hasattr(lib, "mmpfn_variant_flags") and not diagnostics_enabled():
        flags = ctypes.c_char_p.in_dll(lib, "mmpfn_variant_flags").value
        raise RuntimeError(f"{p} is a variant build ({flags!r}); set MMPFN_DIAGNOSTICS=1 to load it")
    for name, res, args in SIGNATURES + MODALITY_SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _LIB = lib
    return lib


class EngineError(RuntimeError):
    pass


def check(lib, ctx, rc: int, what: str) -> None:
    if rc == MMPFN_OK:
        return
    msg = lib.mmpfn_last_error(ctx)
    msg = msg.decode() if msg else ""
    if rc == MMPFN_ERR_NAN:
        raise ValueError(f"{what}: {msg}")
    raise EngineError(f"{what} failed (rc={rc}): {msg}")


def check_enc(lib, enc, rc: int, what: str) -> None:
    """Status of a modality-encoder call (include/mmpfn_modality.h)."""
    if rc == MMPFN_OK:
        return
    msg = lib.mmpfn_enc_last_error(enc)
    msg = msg.decode() if msg else ""
    if rc == MMPFN_ERR_INVALID:
        raise ValueError(f"{what}: {msg}")
    raise EngineError(f"{what} failed (rc={rc}): {msg}")
