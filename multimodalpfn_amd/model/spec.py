"""Model hyper-parameters and the checkpoint ABI (state-dict names and shapes).

The names and shapes are those of the reference ``PerFeatureTransformer`` built by
``load_model`` (``mmpfn/models/mmpfn/model/loading.py:401-542``) so that a
reference ``{"state_dict", "config"}`` checkpoint loads unchanged.
"""

from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class ModelConfig:
    """Hyper-parameters of one PerFeatureTransformer.

    Mirrors the fields of the reference ``InferenceConfig``
    (``model/config.py:18-84``) that shape the forward, plus the mixer arguments
    passed to ``load_model`` (``loading.py:401-408``).
    """

    emsize: int = 192
    nhead: int = 6
    nlayers: int = 12
    nhid_factor: int = 4
    features_per_group: int = 2  # model grouping (PerFeatureTransformer arg, yaml)
    encoder_features: int = 2  # checkpoint config.features_per_group (get_encoder num_features)
    max_num_classes: int = 10
    mixer_type: str = "MGM+CAP"  # "MGM" | "MGM+CAP" | "MoE"
    mgm_heads: int = 64
    cap_heads: int = 24
    two_sets_of_queries: bool = False
    # an (inert) RemoveDuplicateFeatures step shifts the Linear step to index 6
    # (loading.py:328-329,361-369)
    remove_duplicate_features: bool = False
    # set by update_encoder_outlier_params (utils.py:703-745); classification default 12
    remove_outliers_sigma: float | None = 12.0
    model_seed: int = 0
    ln_eps: float = 1e-5
    extra: dict = field(default_factory=dict)

    @property
    def nhid(self) -> int:
        return self.emsize * self.nhid_factor

    @property
    def d_head(self) -> int:
        return self.emsize // self.nhead

    @property
    def n_out(self) -> int:
        # loading.py:460-468 (classifier: max_num_classes > 2 -> n_out = max_num_classes)
        return 1 if self.max_num_classes == 2 else self.max_num_classes

    @property
    def mixer_in_dim(self) -> int:
        # PerFeatureTransformer uses nhid as the modality-embedding width (transformer.py:295)
        return self.nhid


def encoder_linear_name(cfg: ModelConfig) -> str:
    return f"encoder.{6 if cfg.remove_duplicate_features else 5}.layer.weight"


def state_dict_spec(cfg: ModelConfig) -> list[tuple[str, tuple[int, ...]]]:
    """Ordered list of ``(name, shape)`` the reference state_dict contains."""
    E, H, d, Fh = cfg.emsize, cfg.nhead, cfg.d_head, cfg.nhid
    nf = cfg.encoder_features
    spec: list[tuple[str, tuple[int, ...]]] = []
    D = cfg.mixer_in_dim
    if cfg.mixer_type in ("MGM", "MGM+CAP"):
        for h in range(cfg.mgm_heads):
            p = f"mgm.projs.{h}"
            spec += [
                (p + ".0.weight", (D,)),
                (p + ".0.bias", (D,)),
                (p + ".1.weight", (D, D)),
                (p + ".1.bias", (D,)),
                (p + ".4.weight", (E, D // 2)),
                (p + ".4.bias", (E,)),
            ]
    if cfg.mixer_type == "MGM+CAP":
        spec += [
            ("cap.queries", (cfg.cap_heads, E)),
            ("cap.q_proj.weight", (E, E)),
            ("cap.mha.in_proj_weight", (3 * E, E)),
            ("cap.mha.in_proj_bias", (3 * E,)),
            ("cap.mha.out_proj.weight", (E, E)),
            ("cap.mha.out_proj.bias", (E,)),
            ("cap.k_norm.weight", (E,)),
            ("cap.k_norm.bias", (E,)),
            ("cap.q_norm.weight", (E,)),
            ("cap.q_norm.bias", (E,)),
            ("cap.out_norm.weight", (E,)),
            ("cap.out_norm.bias", (E,)),
            ("cap.ffn.0.weight", (2 * E, E)),
            ("cap.ffn.0.bias", (2 * E,)),
            ("cap.ffn.3.weight", (E, 2 * E)),
            ("cap.ffn.3.bias", (E,)),
        ]
    if cfg.mixer_type == "MoE":
        for i in range(cfg.mgm_heads):
            p = f"moe.experts.{i}"
            spec += [
                (p + ".0.weight", (D,)),
                (p + ".0.bias", (D,)),
                (p + ".1.weight", (D // 2, D)),
                (p + ".1.bias", (D // 2,)),
                (p + ".4.weight", (E, D // 2)),
                (p + ".4.bias", (E,)),
            ]
        spec += [("moe.gate.weight", (cfg.mgm_heads, D)), ("moe.gate.bias", (cfg.mgm_heads,))]
    spec += [
        (encoder_linear_name(cfg), (E, 2 * nf)),
        ("y_encoder.2.layer.weight", (E, 2)),
        ("y_encoder.2.layer.bias", (E,)),
    ]
    for l in range(cfg.nlayers):
        p = f"transformer_encoder.layers.{l}"
        spec += [
            (p + ".self_attn_between_features._w_out", (H, d, E)),
            (p + ".self_attn_between_features._w_qkv", (3, H, d, E)),
            (p + ".self_attn_between_items._w_out", (H, d, E)),
        ]
        if cfg.two_sets_of_queries:
            spec += [
                (p + ".self_attn_between_items._w_q", (2, H, d, E)),
                (p + ".self_attn_between_items._w_kv", (2, H, d, E)),
            ]
        else:
            spec += [(p + ".self_attn_between_items._w_qkv", (3, H, d, E))]
        spec += [
            (p + ".mlp.linear1.weight", (Fh, E)),
            (p + ".mlp.linear2.weight", (E, Fh)),
        ]
    spec += [
        ("decoder_dict.standard.0.weight", (Fh, E)),
        ("decoder_dict.standard.0.bias", (Fh,)),
        ("decoder_dict.standard.2.weight", (cfg.n_out, Fh)),
        ("decoder_dict.standard.2.bias", (cfg.n_out,)),
        ("feature_positional_embedding_embeddings.weight", (E, E // 4)),
        ("feature_positional_embedding_embeddings.bias", (E,)),
    ]
    return spec
