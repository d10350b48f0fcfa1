"""Checkpoint loading: a reference ``{"state_dict", "config"}`` file -> HIP-backed model.

Mirror of ``load_model`` (``mmpfn/models/mmpfn/model/loading.py:401-542``): the
checkpoint's ``config`` supplies the trunk hyper-parameters (``InferenceConfig``,
``model/config.py:18-108``); the caller supplies the mixer (``mixer_type``,
``mgm_heads``, ``cap_heads``) and the model's ``features_per_group``, exactly as
the reference passes them.  Differences, both deliberate:

* the file is read with ``torch.load(..., weights_only=True)``: tensors and plain
  containers only, nothing executed from the file;
* ``strict=False`` (``loading.py:540``): a modality head (``mgm.*`` / ``cap.*`` /
  ``moe.*``) missing from the file -- a base TabPFN checkpoint that was never
  fine-tuned with images -- keeps its initialisation, as in the reference.  The
  reference's init draws from the unseeded global RNG; here it is drawn from
  ``torch.manual_seed(model_seed)`` with the reference modules' own init rules, so it
  is reproducible, and a warning names the missing heads.  A missing TRUNK parameter
  (encoders, layers, decoder) is still an error: no reference checkpoint lacks one.
"""

from __future__ import annotations

import warnings
from pathlib import Path
from typing import Any

import torch
from torch import nn

from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec
from multimodalpfn_amd.model.transformer import PerFeatureTransformer

# InferenceConfig fields read by the forward; the rest only matter for training
_CONFIG_FIELDS = {
    "emsize", "nhead", "nlayers", "nhid_factor", "features_per_group", "max_num_classes",
    "remove_duplicate_features", "two_sets_of_queries", "task_type", "batch_size", "seq_len",
    "num_buckets", "max_num_features", "adaptive_max_seq_len_to_max_full_table_size",
    "aggregate_k_gradients", "differentiable_hps_as_style", "dropout", "encoder_use_bias",
    "feature_positional_embedding", "multiquery_item_attention", "nan_handling_enabled",
    "nan_handling_y_encoder", "normalize_by_used_features", "normalize_on_train_only",
    "normalize_to_ranking", "normalize_x", "num_global_att_tokens", "progress_bar", "recompute_attn",
    "recompute_layer", "remove_empty_features", "remove_outliers", "semisupervised_enabled", "timing",
    "use_separate_decoder", "use_flash_attention", "multi_query_factor",
    "multiquery_item_attention_for_test_set", "attention_init_gain",
}

# architecture switches the engine implements only in their (universal) reference setting
_FIXED = {
    "feature_positional_embedding": "subspace",
    "multiquery_item_attention": False,
    "multiquery_item_attention_for_test_set": True,
    "encoder_use_bias": False,
    "nan_handling_enabled": True,
    "nan_handling_y_encoder": True,
    "normalize_by_used_features": True,
    "normalize_on_train_only": True,
    "normalize_to_ranking": False,
    "normalize_x": True,
    "remove_empty_features": True,
    "use_separate_decoder": False,
}


def model_config_from_checkpoint(config: dict, *, model_seed: int, mixer_type: str, mgm_heads: int,
                                 cap_heads: int, features_per_group: int) -> ModelConfig:
    unknown = set(config) - _CONFIG_FIELDS
    if unknown:
        warnings.warn(f"Fields in config not in Config class: {unknown}", stacklevel=3)
    for key, want in _FIXED.items():
        if key in config and config[key] is not None and config[key] != want:
            raise NotImplementedError(f"checkpoint config {key}={config[key]!r} (engine implements {want!r})")
    max_classes = int(config.get("max_num_classes", 10))
    if max_classes == 0:
        raise NotImplementedError("regression checkpoints (bar-distribution decoder) are not served")
    return ModelConfig(
        emsize=int(config.get("emsize", 192)),
        nhead=int(config.get("nhead", 6)),
        nlayers=int(config.get("nlayers", 12)),
        nhid_factor=int(config.get("nhid_factor", 4)),
        features_per_group=int(features_per_group),
        encoder_features=int(config.get("features_per_group", 2)),
        max_num_classes=max_classes,
        mixer_type=mixer_type,
        mgm_heads=int(mgm_heads),
        cap_heads=int(cap_heads),
        two_sets_of_queries=bool(config.get("two_sets_of_queries") or False),
        remove_duplicate_features=bool(config.get("remove_duplicate_features", False)),
        # load_model builds the encoder with config.remove_outliers (False in every config);
        # the classifier switches it on afterwards (update_encoder_outlier_params)
        remove_outliers_sigma=None,
        model_seed=model_seed,
    )


MIXER_PREFIXES = ("mgm.", "cap.", "moe.")


@torch.no_grad()
def init_mixer_(model: PerFeatureTransformer, seed: int) -> None:
    """Initialise the modality heads like the reference constructors (transformer.py:33-128):
    ``nn.Linear`` / ``nn.LayerNorm`` defaults, ``nn.MultiheadAttention._reset_parameters``,
    CAP queries ``randn * 1e-2`` (:64) -- from ``torch.manual_seed(seed)`` instead of the
    reference's unseeded global stream."""
    with torch.random.fork_rng(devices=[]):
        torch.manual_seed(seed)
        for name in ("mgm", "moe", "cap"):
            mod = getattr(model, name, None)
            if mod is None:
                continue
            for m in mod.modules():  # constructor order: the layers first, then the MHA's own reset
                if isinstance(m, (nn.Linear, nn.LayerNorm)):
                    m.reset_parameters()
            for m in mod.modules():
                if isinstance(m, nn.MultiheadAttention):
                    m._reset_parameters()  # in_proj xavier, in_proj / out_proj biases zero
            if name == "cap":
                mod.queries.copy_(torch.randn(mod.queries.shape) * 1e-2)


def build_model(cfg: ModelConfig, state_dict: dict[str, Any]) -> PerFeatureTransformer:
    """Instantiate the model and load ``state_dict`` with the reference's ``strict=False``
    (loading.py:540): extra keys ignored, missing modality-head tensors keep their (seeded)
    initialisation with a warning, a missing trunk tensor is an error."""
    model = PerFeatureTransformer(cfg)
    names = [n for n, _ in state_dict_spec(cfg)]
    missing = [n for n in names if n not in state_dict]
    trunk = [n for n in missing if not n.startswith(MIXER_PREFIXES)]
    if trunk:
        raise ValueError(f"checkpoint lacks {len(trunk)} trunk parameter(s) the model needs, e.g. {trunk[:5]}")
    if missing:
        init_mixer_(model, cfg.model_seed)
        heads = sorted({n.split(".")[0] for n in missing})
        warnings.warn(f"checkpoint has no weights for the modality head(s) {heads} ({len(missing)} tensors): "
                      f"they keep their initialisation (seeded by model_seed={cfg.model_seed}), as the "
                      "reference's strict=False load leaves them", stacklevel=3)
    model.load_state_dict({n: torch.as_tensor(state_dict[n]) for n in names if n in state_dict}, strict=False)
    model.cache_trainset_representation = True  # loading.py:497
    model.eval()
    return model


def load_model(*, path: Path, model_seed: int, mixer_type: str, mgm_heads: int, cap_heads: int,
               features_per_group: int) -> tuple[PerFeatureTransformer, nn.Module, dict]:
    """``loading.py:401-542``: returns (model, loss criterion, config dict)."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    assert "state_dict" in ckpt
    assert "config" in ckpt
    config = dict(ckpt["config"])
    cfg = model_config_from_checkpoint(config, model_seed=model_seed, mixer_type=mixer_type, mgm_heads=mgm_heads,
                                       cap_heads=cap_heads, features_per_group=features_per_group)
    state = {k: v for k, v in ckpt["state_dict"].items() if not k.startswith("criterion.")}
    model = build_model(cfg, state)
    criterion: nn.Module = (nn.BCEWithLogitsLoss(reduction="none") if cfg.max_num_classes == 2
                            else nn.CrossEntropyLoss(reduction="none"))
    return model, criterion, config
