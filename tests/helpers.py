"""Test helpers: fixtures -> configs, weights and inputs (shared by CPU and GPU tests)."""

from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import torch

from synth import synth_state_dict

from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec
from oracle.forward import OracleSpec

GOLDEN = Path(__file__).resolve().parent / "golden"
CASES = sorted(p.stem for p in GOLDEN.glob("*.npz") if not p.stem.startswith(("api_", "modality_")))


def load_case(name: str):
    z = np.load(GOLDEN / f"{name}.npz")
    meta = json.loads(str(z["meta"]))
    cfg = ModelConfig(**meta["cfg"])
    sd = synth_state_dict(state_dict_spec(cfg), meta["wseed"])
    return z, meta, cfg, sd


def oracle_spec(cfg: ModelConfig) -> OracleSpec:
    return OracleSpec(
        emsize=cfg.emsize, nhead=cfg.nhead, nlayers=cfg.nlayers, nhid=cfg.nhid,
        features_per_group=cfg.features_per_group, encoder_features=cfg.encoder_features, n_out=cfg.n_out,
        mixer_type=cfg.mixer_type, mgm_heads=cfg.mgm_heads, cap_heads=cfg.cap_heads,
        remove_outliers_sigma=cfg.remove_outliers_sigma, model_seed=cfg.model_seed,
        two_sets_of_queries=cfg.two_sets_of_queries, ln_eps=cfg.ln_eps,
    )


def torch_sd(sd: dict) -> dict:
    return {k: torch.from_numpy(v) for k, v in sd.items()}


def rel_err(a, b) -> float:
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(1.0, np.abs(b).max()))
