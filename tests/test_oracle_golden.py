"""The CPU oracle reproduces the reference's golden vectors (pins the oracle)."""

import numpy as np
import pytest
import torch

from helpers import CASES, load_case, oracle_spec, rel_err, torch_sd
from oracle.forward import oracle_forward, oracle_mixer


@pytest.mark.parametrize("case", CASES)
def test_oracle_logits_match_reference(case):
    z, meta, cfg, sd = load_case(case)
    x = torch.from_numpy(z["x"]) if "x" in z else None
    im = torch.from_numpy(z["image"]) if "image" in z else None
    taps = {}
    out = oracle_forward(oracle_spec(cfg), torch_sd(sd), x, im, torch.from_numpy(z["y_train"]), taps=taps)
    assert rel_err(out.numpy(), z["logits"]) < 1e-5
    assert (out.numpy().argmax(1) == z["logits"].argmax(1)).all()
    if "embedded_input" in z:
        assert rel_err(taps["embedded_input"].numpy(), z["embedded_input"]) < 1e-5
        assert rel_err(taps["layer0"].numpy(), z["layer0"]) < 1e-5


@pytest.mark.parametrize("case", [c for c in CASES if c not in ("tab_small",)])
def test_oracle_mixer_matches_reference(case):
    z, meta, cfg, sd = load_case(case)
    if "mixer_tokens" not in z:
        pytest.skip("no image input")
    tok = oracle_mixer(oracle_spec(cfg), torch_sd(sd), torch.from_numpy(z["image"]).double())
    assert np.abs(tok.numpy() - z["mixer_tokens"]).max() < 1e-4


def test_oracle_float64_close_to_float32():
    z, meta, cfg, sd = load_case("pad_ufes_12l")
    args = (oracle_spec(cfg), torch_sd(sd), torch.from_numpy(z["x"]), torch.from_numpy(z["image"]),
            torch.from_numpy(z["y_train"]))
    a = oracle_forward(*args, dtype=torch.float32).numpy()
    b = oracle_forward(*args, dtype=torch.float64).numpy()
    assert rel_err(a, b) < 1e-5


def test_oracle_sdpa_branch_agrees():
    """The SDPA branch the reference takes on a GPU box agrees with the einsum branch."""
    z, meta, cfg, sd = load_case("mgmcap_edge")
    args = (oracle_spec(cfg), torch_sd(sd), torch.from_numpy(z["x"]), torch.from_numpy(z["image"]),
            torch.from_numpy(z["y_train"]))
    a = oracle_forward(*args).numpy()
    b = oracle_forward(*args, use_sdpa=True).numpy()
    assert rel_err(a, b) < 1e-5


def test_oracle_matches_reference_at_config_c_model():
    """Config C's model (12 layers, MGM 64 + CAP 24, F = 21 with 18 categorical) on 600 rows: the oracle against
    the reference's fp32 logits stored by make_f16_golden.py (pad_ufes_c_reduced)."""
    import json

    from synth import synth_state_dict

    from helpers import GOLDEN
    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    f = np.load(GOLDEN / "f16" / "pad_ufes_c_reduced.npz")
    meta = json.loads(str(f["meta"]))
    cfg = ModelConfig(**meta["cfg"])
    sd = synth_state_dict(state_dict_spec(cfg), meta["wseed"])
    out = oracle_forward(oracle_spec(cfg), torch_sd(sd), torch.from_numpy(f["x"]), torch.from_numpy(f["image"]),
                         torch.from_numpy(f["y_train"])).numpy()
    assert rel_err(out, f["logits_f32"]) < 1e-5
    assert (out.argmax(1) == f["logits_f32"].argmax(1)).all()
    # the reference's own fp16 autocast stays within a few 1e-3 of its fp32 forward (the fp16 mode's band)
    assert rel_err(f["logits_f16"], f["logits_f32"]) < 5e-3
