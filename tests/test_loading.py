"""Checkpoint loading semantics of ``load_model`` (loading.py:401-542): CPU only."""

import copy

import pytest
import torch

from api_cases import ckpt_config
from synth import synth_state_dict

from multimodalpfn_amd.model.loading import load_model
from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec


def _write_ckpt(tmp_path, cfg, drop_prefixes=()):
    sd = synth_state_dict(state_dict_spec(cfg), 3)
    sd = {k: torch.from_numpy(v) for k, v in sd.items() if not k.startswith(tuple(drop_prefixes))}
    path = tmp_path / "m.ckpt"
    torch.save({"state_dict": sd, "config": ckpt_config(cfg)}, path)
    return path, sd


def _load(path, seed=0, mixer="MGM+CAP", mgm=4, cap=2):
    return load_model(path=path, model_seed=seed, mixer_type=mixer, mgm_heads=mgm, cap_heads=cap,
                      features_per_group=2)[0]


def test_base_checkpoint_without_mixer_loads_like_strict_false(tmp_path):
    """A base TabPFN-format checkpoint (no mgm.* / cap.* tensors) loads; the heads keep a seeded
    init and the trunk comes from the file (reference load_state_dict(strict=False), :540)."""
    cfg = ModelConfig(nlayers=2, mgm_heads=4, cap_heads=2)
    path, sd = _write_ckpt(tmp_path, cfg, drop_prefixes=("mgm.", "cap."))
    with pytest.warns(UserWarning, match="modality head"):
        m1 = _load(path, seed=5)
    with pytest.warns(UserWarning):
        m2 = _load(path, seed=5)
    with pytest.warns(UserWarning):
        m3 = _load(path, seed=6)
    s1, s2, s3 = m1.state_dict(), m2.state_dict(), m3.state_dict()
    for k, v in sd.items():  # trunk from the file
        assert torch.equal(s1[k], v), k
    mixer = [k for k in s1 if k.startswith(("mgm.", "cap."))]
    assert mixer and all(torch.equal(s1[k], s2[k]) for k in mixer)  # reproducible per model_seed
    assert any(not torch.equal(s1[k], s3[k]) for k in mixer)
    # reference init rules: LayerNorm ones / zeros, CAP queries randn * 1e-2, MHA out_proj bias 0
    assert torch.equal(s1["mgm.projs.0.0.weight"], torch.ones_like(s1["mgm.projs.0.0.weight"]))
    assert torch.equal(s1["cap.mha.out_proj.bias"], torch.zeros_like(s1["cap.mha.out_proj.bias"]))
    assert s1["cap.queries"].abs().max() < 0.1
    assert torch.isfinite(torch.cat([s1[k].flatten() for k in mixer])).all()
    assert m1.cache_trainset_representation  # loading.py:497


def test_missing_trunk_tensor_is_an_error(tmp_path):
    cfg = ModelConfig(nlayers=2, mgm_heads=4, cap_heads=2)
    path, _ = _write_ckpt(tmp_path, cfg, drop_prefixes=("transformer_encoder.layers.1.mlp.",))
    with pytest.raises(ValueError, match="trunk"):
        _load(path)


def test_full_checkpoint_loads_without_warning(tmp_path, recwarn):
    cfg = ModelConfig(nlayers=1, mgm_heads=4, cap_heads=2)
    path, sd = _write_ckpt(tmp_path, cfg)
    m = _load(path)
    assert not [w for w in recwarn if "modality head" in str(w.message)]
    s = m.state_dict()
    assert all(torch.equal(s[k], v) for k, v in sd.items())


def test_deepcopy_shares_nothing_mutable(tmp_path):
    """InferenceEngineCacheKV.prepare deep-copies the model per member (inference.py:421)."""
    cfg = ModelConfig(nlayers=1, mgm_heads=4, cap_heads=2)
    path, _ = _write_ckpt(tmp_path, cfg)
    m = _load(path)
    c = copy.deepcopy(m)
    assert c is not m and c._train_cache is None
    for (k, a), (_, b) in zip(m.state_dict().items(), c.state_dict().items()):
        assert torch.equal(a, b) and a.data_ptr() != b.data_ptr(), k
