"""C-ABI boundary and checkpoint ABI (CPU-only checks; no compute without a GPU)."""

import re
from pathlib import Path

import pytest
import torch

from multimodalpfn_amd import _lib
from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec
from multimodalpfn_amd.model.transformer import PerFeatureTransformer

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "mmpfn_hip.h"


def header_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(mmpfn_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_binding_table():
    assert header_symbols() == sorted(n for n, _, _ in _lib.SIGNATURES)


def test_library_loads_and_exports_every_symbol():
    if not _lib.LIB_PATH.exists():
        pytest.fail(f"{_lib.LIB_PATH} not built (run __graft_entry__.build())")
    lib = _lib.load_library()
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert b"gfx950" in lib.mmpfn_version()


def test_library_rejects_bad_calls_without_gpu_compute():
    lib = _lib.load_library()
    assert lib.mmpfn_last_error(None) == b"null context"
    assert lib.mmpfn_set_stream(None, None) == _lib.MMPFN_ERR_INVALID
    assert lib.mmpfn_forward(None, None, 0, 0, None, 0, None, 0, None, 0, None, None, 0) == _lib.MMPFN_ERR_INVALID


@pytest.mark.parametrize(
    "kw",
    [
        dict(),
        dict(mixer_type="MGM", mgm_heads=3),
        dict(mixer_type="MoE", mgm_heads=4, cap_heads=2),
        dict(two_sets_of_queries=True, nlayers=2),
        dict(remove_duplicate_features=True, nlayers=1),
        dict(features_per_group=1, nlayers=1, mgm_heads=2),
    ],
)
def test_state_dict_names_match_checkpoint_abi(kw):
    cfg = ModelConfig(**kw)
    model = PerFeatureTransformer(cfg)
    got = sorted((k, tuple(v.shape)) for k, v in model.state_dict().items())
    assert got == sorted(state_dict_spec(cfg))


def test_forward_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    cfg = ModelConfig(nlayers=1, mgm_heads=2, cap_heads=2)
    model = PerFeatureTransformer(cfg)
    x = torch.zeros(8, 1, 3)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        model(None, x, None, torch.zeros(6), single_eval_pos=6)


def test_outlier_params_hook_like_reference():
    """utils.update_encoder_outlier_params finds the step by class name (utils.py:734-745)."""
    model = PerFeatureTransformer(ModelConfig(nlayers=1, mgm_heads=2, cap_heads=2))
    norm = next(e for e in model.encoder if "InputNormalizationEncoderStep" in str(e.__class__))
    norm.remove_outliers = True
    norm.remove_outliers_sigma = 7.0
    assert model._effective_config().remove_outliers_sigma == 7.0
    norm.remove_outliers = False
    assert model._effective_config().remove_outliers_sigma is None


def test_loader_refuses_variant_builds(tmp_path, monkeypatch):
    """A library carrying the variant marker (an A/B or stamps build) and any MMPFN_LIB override load
    only under MMPFN_DIAGNOSTICS=1, so the product path cannot pick up a build with changed kernels."""
    import shutil
    import subprocess

    from multimodalpfn_amd import _lib

    src = tmp_path / "m.c"
    src.write_text('const char *const mmpfn_variant_flags = "test: -DX";\n')
    so = tmp_path / "libvar.so"
    subprocess.run([shutil.which("gcc") or "gcc", "-shared", "-fPIC", str(src), "-o", str(so)], check=True)
    monkeypatch.delenv("MMPFN_DIAGNOSTICS", raising=False)
    with pytest.raises(RuntimeError, match="variant build"):
        _lib.load_library(so)
    monkeypatch.setenv("MMPFN_LIB", str(so))
    monkeypatch.setattr(_lib, "_LIB", None)
    with pytest.raises(RuntimeError, match="MMPFN_DIAGNOSTICS"):
        _lib.load_library()


def test_parity_attention_switch_defaults_off_and_round_trips():
    """mmpfn_set_parity_attention_min_keys: off (-1) by default -- no N keeps the cheap forms 2x under 1e-4
    (profiles/r06/parity_n0_sweep_form*.txt) -- and returns the previous value (no GPU call)."""
    lib = _lib.load_library()
    prev = lib.mmpfn_set_parity_attention_min_keys(512, 2)
    try:
        assert prev == -1
        assert lib.mmpfn_set_parity_attention_min_keys(0, 0) == 512
    finally:
        lib.mmpfn_set_parity_attention_min_keys(-1, 3)
    assert lib.mmpfn_set_parity_attention_min_keys(-1, 0) == -1
