"""Deterministic synthetic weights and inputs (shared by fixture generation and tests).

Weights: every tensor named in the checkpoint ABI is drawn from its own numpy
PCG64 stream (seed mixed with the CRC32 of its name), so the values do not depend
on enumeration order.  Scales are O(1/sqrt(fan_in)) so logits are O(1) with clear
argmax margins.  The reference zero-initialises ``_w_out`` and ``mlp.linear2``
(``transformer.py:225``); overwriting everything avoids a degenerate identity net.
"""

from __future__ import annotations

import math
import zlib

import numpy as np


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.default_rng([seed & 0xFFFFFFFF, zlib.crc32(name.encode())])


def _fan_in(name: str, shape: tuple[int, ...]) -> int:
    if name.endswith("._w_out"):
        return shape[0] * shape[1]
    if name.endswith(("._w_qkv", "._w_q", "._w_kv")):
        return shape[-1]
    return shape[-1]


def _is_layernorm(name: str) -> bool:
    return (
        name.endswith(("k_norm.weight", "q_norm.weight", "out_norm.weight"))
        or (name.startswith(("mgm.projs.", "moe.experts.")) and name.endswith(".0.weight"))
    )


def synth_weight(name: str, shape: tuple[int, ...], seed: int) -> np.ndarray:
    g = _rng(seed, name)
    z = g.standard_normal(shape)
    if _is_layernorm(name):
        v = 1.0 + 0.1 * z
    elif name.endswith("bias") or name.endswith("_bias"):
        v = 0.1 * z
    elif name == "cap.queries":
        v = z
    else:
        v = z / math.sqrt(_fan_in(name, shape))
    return v.astype(np.float32)


def synth_state_dict(spec: list[tuple[str, tuple[int, ...]]], seed: int) -> dict[str, np.ndarray]:
    return {n: synth_weight(n, tuple(s), seed) for n, s in spec}


def synth_table(
    S: int,
    F: int,
    seed: int,
    *,
    n_cat: int = 0,
    nan_frac: float = 0.0,
    add_inf: bool = False,
    add_constant: bool = False,
    add_outlier: bool = False,
) -> np.ndarray:
    """``[S, F]`` float32 table: first ``n_cat`` columns small ints, rest N(0,1)."""
    g = np.random.default_rng(seed)
    X = g.standard_normal((S, F))
    for j in range(min(n_cat, F)):
        k = int(g.integers(1, 6))
        X[:, j] = g.integers(0, k + 1, size=S)
    if nan_frac > 0:
        m = g.random((S, F)) < nan_frac
        X[m] = np.nan
    if add_constant and F > 1:
        X[:, F - 1] = 3.25
    if add_inf and F > 2:
        # +-inf in the last (query) rows: a train column holding both would give a
        # NaN train mean and the reference raises (transformer.py:790-796)
        X[S - 1, F - 2] = np.inf
        X[S - 2, F - 2] = -np.inf
    if add_outlier and F > 3:
        X[int(g.integers(0, S // 2)), F - 3] = 1e4
    return X.astype(np.float32)


def synth_labels(S: int, n_classes: int, seed: int) -> np.ndarray:
    g = np.random.default_rng(seed + 7)
    y = g.integers(0, n_classes, size=S)
    y[:n_classes] = np.arange(n_classes)  # every class present in train
    return y.astype(np.float32)


def synth_image(S: int, n_mod: int, seed: int, dim: int = 768) -> np.ndarray:
    """Modality embeddings ``[S, n_mod, dim]`` (L2-normalised like a DINOv2 CLS x sqrt(dim))."""
    g = np.random.default_rng(seed + 11)
    z = g.standard_normal((S, n_mod, dim))
    z = z / np.linalg.norm(z, axis=-1, keepdims=True) * math.sqrt(dim)
    return z.astype(np.float32)
