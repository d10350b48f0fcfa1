"""Drop-in ``PerFeatureTransformer``: the model seam of the reference inference engine.

Mirrors ``mmpfn/models/mmpfn/model/transformer.py:182-545`` at its interface:

* parameters are registered under the reference's exact ``state_dict`` names
  (checkpoint ABI, ``model/spec.py``), so ``load_state_dict`` of a reference
  checkpoint works unchanged (``loading.py:540``);
* ``model(None, X_full[S,1,F], image_full[S,n_mod,768], y_train[N],
  only_return_standard_out=True, categorical_inds=..., single_eval_pos=N)``
  returns ``[Q, 1, n_out]`` like the reference call at ``inference.py:343-348``;
* attributes the surrounding code touches exist with the same meaning:
  ``ninp``, ``features_per_group``, ``transformer_encoder.layers``,
  ``reset_save_peak_mem_factor``, ``cache_trainset_representation`` and the
  ``encoder`` steps whose ``InputNormalizationEncoderStep`` carries
  ``remove_outliers`` / ``remove_outliers_sigma`` (``utils.py:703-745``).

The torch modules here are weight containers only -- the forward runs in the
HIP engine (``libmmpfn_hip.so``).  There is no CPU/torch compute path: without a
ROCm GPU (or without the built library) the forward raises ``RuntimeError``.

Precision follows the reference's choice at call time: inside
``torch.autocast`` (the reference's "auto" on GPU, ``base.py:126-165``) the engine
runs its bf16-MFMA performance mode; otherwise (or with a forced float32 dtype)
the fp32 parity mode.
"""

from __future__ import annotations

import copy
from typing import Any

import torch
from torch import nn

from multimodalpfn_amd import _lib
from multimodalpfn_amd.model.spec import ModelConfig

# ----------------------------------------------------------------------------- containers


class RemoveEmptyFeaturesEncoderStep(nn.Module):
    """encoders.py:496-527 (executed by the HIP encoder kernel)."""


class RemoveDuplicateFeaturesEncoderStep(nn.Module):
    """encoders.py:530-576 (inert in the reference: returns its input)."""


class NanHandlingEncoderStep(nn.Module):
    """encoders.py:428-493."""

    def __init__(self, keep_nans: bool = True):
        super().__init__()
        self.keep_nans = keep_nans


class VariableNumFeaturesEncoderStep(nn.Module):
    """encoders.py:579-655."""

    def __init__(self, num_features: int, normalize_by_used_features: bool = True):
        super().__init__()
        self.num_features = num_features
        self.normalize_by_used_features = normalize_by_used_features


class InputNormalizationEncoderStep(nn.Module):
    """encoders.py:658-782; ``remove_outliers`` is switched on by ``update_encoder_outlier_params``."""

    def __init__(self, remove_outliers: bool = False, remove_outliers_sigma: float = 4.0):
        super().__init__()
        self.normalize_on_train_only = True
        self.normalize_to_ranking = False
        self.normalize_x = True
        self.remove_outliers = remove_outliers
        self.remove_outliers_sigma = remove_outliers_sigma
        self.seed = 0

    def reset_seed(self) -> None:
        """encoders.py:699-700 (no-op in the reference too)."""


class LinearInputEncoderStep(nn.Module):
    """encoders.py:382-425."""

    def __init__(self, num_features: int, emsize: int, bias: bool):
        super().__init__()
        self.layer = nn.Linear(num_features, emsize, bias=bias)


class MulticlassClassificationTargetEncoder(nn.Module):
    """encoders.py:949-974."""


class SequentialEncoder(nn.Sequential):
    """encoders.py:187-228."""


class MultiHeadAttentionWeights(nn.Module):
    """Parameter layout of ``MultiHeadAttention`` (multi_head_attention.py:201-271)."""

    def __init__(self, E: int, H: int, d: int, two_sets_of_queries: bool = False):
        super().__init__()
        self._w_out = nn.Parameter(torch.empty(H, d, E))
        if two_sets_of_queries:
            self._w_q = nn.Parameter(torch.empty(2, H, d, E))
            self._w_kv = nn.Parameter(torch.empty(2, H, d, E))
        else:
            self._w_qkv = nn.Parameter(torch.empty(3, H, d, E))


class MLPWeights(nn.Module):
    """mlp.py:59-91 (two bias-free Linear layers)."""

    def __init__(self, E: int, Fh: int):
        super().__init__()
        self.linear1 = nn.Linear(E, Fh, bias=False)
        self.linear2 = nn.Linear(Fh, E, bias=False)


class PerFeatureEncoderLayer(nn.Module):
    """layer.py:95-266 parameters (LayerNorms have no affine -> no parameters)."""

    def __init__(self, cfg: ModelConfig):
        super().__init__()
        E, H, d = cfg.emsize, cfg.nhead, cfg.d_head
        self.self_attn_between_features = MultiHeadAttentionWeights(E, H, d)
        self.self_attn_between_items = MultiHeadAttentionWeights(E, H, d, cfg.two_sets_of_queries)
        self.mlp = MLPWeights(E, cfg.nhid)
        self.save_peak_mem_factor: int | None = None  # accepted, the engine needs no chunking


class LayerStack(nn.Module):
    """transformer.py:131-179."""

    def __init__(self, cfg: ModelConfig):
        super().__init__()
        self.layers = nn.ModuleList([PerFeatureEncoderLayer(cfg) for _ in range(cfg.nlayers)])
        self.num_layers = cfg.nlayers


class MultiheadGatedMLP(nn.Module):
    """transformer.py:33-57."""

    def __init__(self, in_dim: int, out_dim: int, mgm_heads: int):
        super().__init__()
        self.projs = nn.ModuleList(
            [
                nn.Sequential(
                    nn.LayerNorm(in_dim), nn.Linear(in_dim, in_dim), nn.GLU(), nn.Dropout(0.0),
                    nn.Linear(in_dim // 2, out_dim),
                )
                for _ in range(mgm_heads)
            ]
        )


class CrossAttentionPooler(nn.Module):
    """transformer.py:60-88."""

    def __init__(self, src_dim: int, cap_heads: int):
        super().__init__()
        self.queries = nn.Parameter(torch.empty(cap_heads, src_dim))
        self.q_proj = nn.Linear(src_dim, src_dim, bias=False)
        self.mha = nn.MultiheadAttention(src_dim, cap_heads, batch_first=False)
        self.k_norm = nn.LayerNorm(src_dim)
        self.q_norm = nn.LayerNorm(src_dim)
        self.out_norm = nn.LayerNorm(src_dim)
        self.ffn = nn.Sequential(
            nn.Linear(src_dim, src_dim * 2), nn.GELU(), nn.Dropout(0.0), nn.Linear(src_dim * 2, src_dim)
        )


class MoE(nn.Module):
    """transformer.py:91-128."""

    def __init__(self, in_dim: int, out_dim: int, n_experts: int):
        super().__init__()
        self.experts = nn.ModuleList(
            [
                nn.Sequential(
                    nn.LayerNorm(in_dim), nn.Linear(in_dim, in_dim // 2), nn.GELU(), nn.Dropout(0.0),
                    nn.Linear(in_dim // 2, out_dim),
                )
                for _ in range(n_experts)
            ]
        )
        self.gate = nn.Linear(in_dim, n_experts)


# ----------------------------------------------------------------------------- the model


class PerFeatureTransformer(nn.Module):
    """HIP-engine-backed drop-in for the reference ``PerFeatureTransformer``."""

    def __init__(self, cfg: ModelConfig):
        super().__init__()
        self.cfg = cfg
        E = cfg.emsize
        self.mixer_type = cfg.mixer_type
        if cfg.mixer_type in ("MGM", "MGM+CAP"):
            self.mgm = MultiheadGatedMLP(cfg.mixer_in_dim, E, cfg.mgm_heads)
        if cfg.mixer_type == "MGM+CAP":
            self.cap = CrossAttentionPooler(E, cfg.cap_heads)
        if cfg.mixer_type == "MoE":
            self.moe = MoE(cfg.mixer_in_dim, E, cfg.mgm_heads)
        nf = cfg.encoder_features
        steps = [RemoveEmptyFeaturesEncoderStep()]
        if cfg.remove_duplicate_features:
            steps.append(RemoveDuplicateFeaturesEncoderStep())
        steps += [
            NanHandlingEncoderStep(True),
            VariableNumFeaturesEncoderStep(nf, normalize_by_used_features=False),
            InputNormalizationEncoderStep(
                remove_outliers=cfg.remove_outliers_sigma is not None,
                remove_outliers_sigma=cfg.remove_outliers_sigma if cfg.remove_outliers_sigma is not None else 4.0,
            ),
            VariableNumFeaturesEncoderStep(nf, normalize_by_used_features=True),
            LinearInputEncoderStep(2 * nf, E, bias=False),
        ]
        self.encoder = SequentialEncoder(*steps)
        self.y_encoder = SequentialEncoder(
            NanHandlingEncoderStep(True), MulticlassClassificationTargetEncoder(), LinearInputEncoderStep(2, E, True)
        )
        self.transformer_encoder = LayerStack(cfg)
        self.decoder_dict = nn.ModuleDict(
            {"standard": nn.Sequential(nn.Linear(E, cfg.nhid), nn.GELU(), nn.Linear(cfg.nhid, cfg.n_out))}
        )
        self.feature_positional_embedding_embeddings = nn.Linear(E // 4, E)
        self.feature_positional_embedding = "subspace"
        self.ninp = E
        self.nhead = cfg.nhead
        self.nhid = cfg.nhid
        self.features_per_group = cfg.features_per_group
        self.cache_trainset_representation = False
        self.seed = cfg.model_seed
        self._target_device = torch.device("cpu")
        self._forced_dtype: torch.dtype | None = None
        self._engines: dict[Any, Any] = {}
        self._weights_version = 0
        self._train_cache = None  # device train-KV cache of the last train-only forward (fit_with_cache)

    def __deepcopy__(self, memo):
        """``deepcopy(model)`` (InferenceEngineCacheKV.prepare, inference.py:421): parameters are
        copied; the packed device weights are shared with the original (same values), the train-KV
        cache is not (each copy caches its own member)."""
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            if k == "_engines":
                # the engines are shared (same weights), the dict is not: each holder counts as one
                # reference, so invalidating or re-keying one copy leaves the others' engines open
                new.__dict__[k] = dict(v)
                for eng in v.values():
                    eng.refs += 1
            elif k == "_train_cache":
                new.__dict__[k] = None
            else:
                new.__dict__[k] = copy.deepcopy(v, memo)
        return new

    # ------------------------------------------------------------------ module plumbing
    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):  # noqa: D102
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self.invalidate_engine()
        return res

    def invalidate_engine(self) -> None:
        """Drop packed device weights (call after modifying parameters in place)."""
        for eng in self._engines.values():
            eng.release()
        self._engines.clear()
        self._weights_version += 1

    def to(self, *args, **kwargs):  # noqa: D102
        device, dtype, _, _ = torch._C._nn._parse_to(*args, **kwargs)
        if device is not None:
            self._target_device = torch.device(device)
        if dtype is not None:
            self._forced_dtype = dtype
        return self

    def cuda(self, device=None):  # noqa: D102
        self._target_device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device or "cuda")
        return self

    def cpu(self):  # noqa: D102
        self._target_device = torch.device("cpu")
        return self

    def type(self, dst_type):  # noqa: D102
        self._forced_dtype = dst_type if isinstance(dst_type, torch.dtype) else None
        return self

    def reset_save_peak_mem_factor(self, factor: int | None = None) -> None:
        """memory.py:386-389 -- accepted for API parity; the engine streams without chunking."""
        for layer in self.transformer_encoder.layers:
            layer.save_peak_mem_factor = factor

    # ------------------------------------------------------------------ engine
    def _effective_config(self) -> ModelConfig:
        norm = next(e for e in self.encoder if isinstance(e, InputNormalizationEncoderStep))
        cfg = ModelConfig(**{k: getattr(self.cfg, k) for k in self.cfg.__dataclass_fields__})
        cfg.remove_outliers_sigma = float(norm.remove_outliers_sigma) if norm.remove_outliers else None
        cfg.features_per_group = self.features_per_group
        cfg.model_seed = self.seed if isinstance(self.seed, int) else 0
        return cfg

    def _device(self) -> torch.device:
        if not torch.cuda.is_available():
            raise RuntimeError(
                "multimodalpfn_amd runs the PerFeatureTransformer forward on MI355X through its HIP engine; "
                "no ROCm GPU is visible (there is no CPU path)"
            )
        dev = self._target_device
        if dev.type != "cuda":
            dev = torch.device("cuda", torch.cuda.current_device())
        elif dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        return dev

    def engine(self, device: torch.device | None = None):
        """The HIP engine for ``device`` (built lazily, weights uploaded once)."""
        from multimodalpfn_amd.engine import HipEngine

        dev = torch.device(device) if device is not None else self._device()
        if dev.type == "cuda" and dev.index is None:  # "cuda" and "cuda:<current>" are one engine
            dev = torch.device("cuda", torch.cuda.current_device())
        cfg = self._effective_config()
        key = (str(dev), cfg.remove_outliers_sigma, cfg.features_per_group, cfg.model_seed)
        eng = self._engines.get(key)
        if eng is None:
            for old in list(self._engines):
                if old[0] == str(dev):
                    self._engines.pop(old).release()
            eng = HipEngine(cfg, self.state_dict(), dev)
            self._engines[key] = eng
        return eng

    def precision(self, device: torch.device) -> int:
        if self._forced_dtype is not None:
            return _lib.precision_of_dtype(self._forced_dtype)
        if torch.is_autocast_enabled(device.type):
            return _lib.autocast_precision()
        return _lib.f32_precision()

    # ------------------------------------------------------------------ forward
    def forward(self, *args: Any, **kwargs: Any) -> torch.Tensor:
        """Inference call forms of transformer.py:462-545 (4-tuple and 3-tuple)."""
        supported = {"only_return_standard_out", "style", "data_dags", "categorical_inds", "single_eval_pos",
                     "mixer_tokens", "precision"}
        spurious = set(kwargs) - supported
        assert not spurious, spurious
        if len(args) == 4:
            style, x, image, y = args
        elif len(args) == 3:
            style, x, y = args
            image = None
        else:
            raise ValueError("Unrecognized input. Please follow the doc string.")
        assert style is None
        if not kwargs.get("only_return_standard_out", True):
            raise NotImplementedError("only the standard decoder output is served by the engine")
        sep = kwargs.get("single_eval_pos")
        dev = self._device()
        eng = self.engine(dev)
        prec = kwargs.get("precision")
        if prec is None:
            prec = self.precision(dev)
        tokens = kwargs.get("mixer_tokens")
        if tokens is None and image is not None and self.mixer_type in ("MGM", "MGM+CAP", "MoE"):
            img = image
            if img.dim() > 3:  # [n_mod, S, D] style (transformer.py:587-588)
                img = torch.movedim(img, 0, 1)
            tokens = eng.mixer_tokens(img, prec)
        if x is not None and x.dim() == 3:
            x = x[:, 0, :]
        if not sep:
            # test rows only against the cached train representation (transformer.py:593-595,779-784;
            # layer.py:311,391-394): the call form of InferenceEngineCacheKV.iter_outputs
            # (inference.py:499-507)
            if not self.cache_trainset_representation:
                raise ValueError("single_eval_pos (number of train rows) is required")
            if y is not None:
                raise ValueError("a cached-trainset call takes no y (transformer.py:593-595)")
            cache = self._train_cache
            if cache is None or cache.engine is not eng or not cache.handle:
                raise RuntimeError(
                    "single_eval_pos=None needs a train-KV cache: call the model once on the train rows only "
                    "(single_eval_pos=len(X_train), as InferenceEngineCacheKV.prepare does) with "
                    "cache_trainset_representation=True")
            return eng.cache_predict(cache, x, tokens).unsqueeze(1)
        if y.dim() > 1:
            y = y.reshape(-1)
        y = y[:sep]
        S = x.shape[0] if x is not None else tokens.shape[0]
        if self.cache_trainset_representation and sep == S:
            # train rows only (InferenceEngineCacheKV.prepare, inference.py:425-436): keep this
            # member's head-0 K/V per layer and encoder statistics on the device; the reference
            # returns the (empty) test-row output
            if self._train_cache is not None:
                self._train_cache.free()
            self._train_cache = eng.cache_build(x, tokens, y, prec)
            return torch.empty((0, 1, self.cfg.n_out), device=dev, dtype=torch.float32)
        logits = eng.forward(x, tokens, y, prec)
        return logits.unsqueeze(1)

    def empty_trainset_representation_cache(self) -> None:
        """transformer.py:999-1001: drop the train-KV cache."""
        if self._train_cache is not None:
            self._train_cache.free()
            self._train_cache = None
