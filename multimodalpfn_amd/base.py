"""Model initialisation, precision choice and engine construction (mirror of ``base.py``).

``initialize_mmpfn_model`` / ``determine_precision`` / ``create_inference_engine``
keep the reference signatures (``mmpfn/models/mmpfn/base.py:54-270``).
"""

from __future__ import annotations

from pathlib import Path
from typing import Any, Literal

import torch

from multimodalpfn_amd.constants import AUTOCAST_DTYPE_BYTE_SIZE, DEFAULT_DTYPE_BYTE_SIZE
from multimodalpfn_amd.inference import InferenceEngineCacheKV, InferenceEngineCachePreprocessing, InferenceEngineOnDemand
from multimodalpfn_amd.utils import infer_fp16_inference_mode, load_model_criterion_config


def initialize_mmpfn_model(
    model_path: str | Path | Literal["auto"],
    which: Literal["classifier", "regressor"],
    fit_mode: Literal["low_memory", "fit_preprocessors", "fit_with_cache"],
    static_seed: int,
    mixer_type: str,
    mgm_heads: int,
    cap_heads: int,
    features_per_group: int,
):
    """Load the checkpoint -> (model, config, None) for the classifier (``base.py:54-120``)."""
    if isinstance(model_path, str) and model_path == "auto":
        model_path = None  # type: ignore[assignment]
    model, _, config = load_model_criterion_config(
        model_path=model_path,
        check_bar_distribution_criterion=False,
        cache_trainset_representation=(fit_mode == "fit_with_cache"),
        which=which,
        version="v2",
        download=False,
        model_seed=static_seed,
        mixer_type=mixer_type,
        mgm_heads=mgm_heads,
        cap_heads=cap_heads,
        features_per_group=features_per_group,
    )
    return model, config, None


def determine_precision(inference_precision, device_: torch.device) -> tuple[bool, torch.dtype | None, int]:
    """(use_autocast, forced dtype, byte size), ``base.py:123-165``.

    On the engine, autocast selects the bf16-MFMA mode (fp32 accumulation, fp32
    residual stream / LayerNorm); a forced float32 / float64 selects the fp32 parity
    mode; a forced 16-bit dtype selects bf16.
    """
    if inference_precision in ("autocast", "auto"):
        use_autocast = infer_fp16_inference_mode(
            device=device_, enable=True if inference_precision == "autocast" else None
        )
        return use_autocast, None, AUTOCAST_DTYPE_BYTE_SIZE if use_autocast else DEFAULT_DTYPE_BYTE_SIZE
    if isinstance(inference_precision, torch.dtype):
        return False, inference_precision, inference_precision.itemsize
    raise ValueError(f"Unknown inference_precision={inference_precision}")


def create_inference_engine(
    *,
    X_train,
    y_train,
    image_train,
    model,
    ensemble_configs: Any,
    cat_ix: list[int],
    fit_mode: Literal["low_memory", "fit_preprocessors", "fit_with_cache"],
    device_: torch.device,
    rng,
    n_jobs: int,
    byte_size: int,
    forced_inference_dtype_: torch.dtype | None,
    memory_saving_mode,
    use_autocast_: bool,
):
    """Engine per ``fit_mode`` (``base.py:168-270``)."""
    common = dict(cat_ix=cat_ix, model=model, ensemble_configs=ensemble_configs, n_workers=n_jobs, rng=rng,
                  dtype_byte_size=byte_size, force_inference_dtype=forced_inference_dtype_,
                  save_peak_mem=memory_saving_mode)
    if fit_mode == "low_memory":
        return InferenceEngineOnDemand.prepare(X_train, y_train, image_train, **common)
    if fit_mode == "fit_preprocessors":
        return InferenceEngineCachePreprocessing.prepare(X_train, y_train, image_train, **common)
    if fit_mode == "fit_with_cache":
        return InferenceEngineCacheKV.prepare(X_train, y_train, image_train, device=device_,
                                              autocast=use_autocast_, **common)
    raise ValueError(f"Invalid fit_mode: {fit_mode}")
