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

# numbers a test wants in the run's tail (conftest.pytest_terminal_summary prints them after the result line,
# so `pytest -q` on the GPU box carries them even for passing tests)
REPORT: list[str] = []


def report(line: str) -> None:
    print(line)
    REPORT.append(line)
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


def check_argmax(out, ref, min_agree: float, label: str = "") -> float:
    """Argmax agreement of ``out`` with ``ref`` (rows x classes); prints every disagreeing row's
    reference top-2 margin (a flip on a near-tie is rounding, a flip on a wide margin is a bug)."""
    out = np.asarray(out, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    a, b = out.argmax(1), ref.argmax(1)
    bad = np.nonzero(a != b)[0]
    agree = 1.0 - len(bad) / max(1, len(a))
    if len(bad):
        srt = np.sort(ref, axis=1)
        margins = srt[:, -1] - srt[:, -2]
        print(f"{label}: argmax agreement {agree:.4f}; disagreeing rows (row, ref margin, out margin):",
              [(int(i), float(margins[i]), float(out[i, a[i]] - out[i, b[i]])) for i in bad[:20]])
    assert agree >= min_agree, (label, agree, min_agree)
    return agree
