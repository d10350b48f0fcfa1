"""Generate golden vectors by running the REFERENCE model (build container only).

Run from the repo root:   python tests/golden/make_golden.py

It imports ``/root/reference`` read-only (with a stub for the unused ``seaborn``
import at ``transformer.py:20``), builds ``PerFeatureTransformer`` exactly as
``load_model`` does (``loading.py:470-541``), overwrites every parameter with the
deterministic synthetic weights of ``tests/golden/synth.py``, enables the 12-sigma
outlier removal like ``MMPFNClassifier.fit`` (``classifier.py:396-406``) and calls
the model the way the inference engine does (``inference.py:343-348``).  Outputs
(inputs, logits, taps) are written to ``tests/golden/<case>.npz``; the reference
itself never travels to the GPU box.
"""

from __future__ import annotations

import json
import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(HERE))

from synth import synth_image, synth_labels, synth_state_dict, synth_table  # noqa: E402

from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec  # noqa: E402

# name, model config overrides, data spec
CASES = [
    dict(name="tab_small", cfg=dict(nlayers=2, mgm_heads=2, cap_heads=2), S=80, N=64, F=7,
         data=dict(n_cat=2), n_mod=0, n_classes=3, wseed=1, dseed=101),
    dict(name="mgmcap_edge", cfg=dict(nlayers=2, mgm_heads=4, cap_heads=4), S=96, N=72, F=20,
         data=dict(n_cat=5, nan_frac=0.05, add_inf=True, add_constant=True, add_outlier=True),
         n_mod=1, n_classes=4, wseed=2, dseed=102),
    dict(name="mgm_two_mod", cfg=dict(nlayers=1, mixer_type="MGM", mgm_heads=2, cap_heads=2), S=64, N=48,
         F=5, data=dict(), n_mod=2, n_classes=2, wseed=3, dseed=103),
    dict(name="moe", cfg=dict(nlayers=1, mixer_type="MoE", mgm_heads=4, cap_heads=2), S=64, N=40, F=6,
         data=dict(nan_frac=0.1), n_mod=1, n_classes=5, wseed=4, dseed=104),
    dict(name="image_only", cfg=dict(nlayers=2, mgm_heads=4, cap_heads=2), S=72, N=56, F=0,
         data=dict(), n_mod=1, n_classes=3, wseed=5, dseed=105),
    dict(name="two_queries", cfg=dict(nlayers=2, mgm_heads=2, cap_heads=2, two_sets_of_queries=True), S=70,
         N=50, F=9, data=dict(n_cat=3), n_mod=1, n_classes=3, wseed=6, dseed=106),
    dict(name="fpg1_seed", cfg=dict(nlayers=1, mgm_heads=2, cap_heads=2, features_per_group=1, model_seed=7),
         S=60, N=45, F=5, data=dict(add_constant=True), n_mod=1, n_classes=2, wseed=7, dseed=107),
    dict(name="pad_ufes_12l", cfg=dict(nlayers=12, mgm_heads=8, cap_heads=4), S=160, N=128, F=21,
         data=dict(n_cat=18), n_mod=1, n_classes=6, wseed=8, dseed=108, taps=True),
]


def _import_reference():
    sys.modules.setdefault("seaborn", types.ModuleType("seaborn"))
    sys.path.insert(0, "/root/reference")
    from mmpfn.models.mmpfn.model.loading import get_encoder, get_y_encoder
    from mmpfn.models.mmpfn.model.transformer import PerFeatureTransformer
    from mmpfn.models.mmpfn.utils import update_encoder_outlier_params

    return PerFeatureTransformer, get_encoder, get_y_encoder, update_encoder_outlier_params


def build_reference(cfg: ModelConfig):
    PerFeatureTransformer, get_encoder, get_y_encoder, update_outliers = _import_reference()
    model = PerFeatureTransformer(
        seed=cfg.model_seed,
        encoder=get_encoder(
            num_features=cfg.encoder_features, embedding_size=cfg.emsize, remove_empty_features=True,
            remove_duplicate_features=cfg.remove_duplicate_features, nan_handling_enabled=True,
            normalize_on_train_only=True, normalize_to_ranking=False, normalize_x=True,
            remove_outliers=False, normalize_by_used_features=True, encoder_use_bias=False,
        ),
        y_encoder=get_y_encoder(num_inputs=1, embedding_size=cfg.emsize, nan_handling_y_encoder=True,
                                max_num_classes=cfg.max_num_classes),
        nhead=cfg.nhead, ninp=cfg.emsize, nhid=cfg.nhid, nlayers=cfg.nlayers,
        features_per_group=cfg.features_per_group, cache_trainset_representation=True, init_method=None,
        decoder_dict={"standard": (None, cfg.n_out)}, use_encoder_compression_layer=False,
        recompute_attn=False, recompute_layer=True, feature_positional_embedding="subspace",
        use_separate_decoder=False, layer_norm_with_elementwise_affine=False, nlayers_decoder=None,
        pre_norm=False, multiquery_item_attention=False, multiquery_item_attention_for_test_set=True,
        attention_init_gain=1.0, two_sets_of_queries=cfg.two_sets_of_queries, mixer_type=cfg.mixer_type,
        mgm_heads=cfg.mgm_heads, cap_heads=cfg.cap_heads,
    )
    ref_spec = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    return model, ref_spec, update_outliers


def run_case(case: dict) -> dict:
    cfg = ModelConfig(**case["cfg"])
    model, ref_spec, update_outliers = build_reference(cfg)
    spec = state_dict_spec(cfg)
    assert sorted(ref_spec) == sorted(spec), (set(ref_spec) ^ set(spec))
    sd = synth_state_dict(spec, case["wseed"])
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.eval()
    update_outliers(model=model, remove_outliers_std=12.0, seed=cfg.model_seed, inplace=True)
    model.cache_trainset_representation = False  # fit_preprocessors (base.py:94, utils.py:359)

    S, N = case["S"], case["N"]
    x = synth_table(S, case["F"], case["dseed"], **case["data"]) if case["F"] else None
    y = synth_labels(S, case["n_classes"], case["dseed"])
    image = synth_image(S, case["n_mod"], case["dseed"]) if case["n_mod"] else None

    taps: dict[str, np.ndarray] = {}
    hooks = []
    if case.get("taps"):
        def enc_hook(_m, args, _kw, out):
            taps["embedded_input"] = args[0][0].detach().numpy().copy()
        hooks.append(model.transformer_encoder.register_forward_hook(enc_hook, with_kwargs=True))
        for li, layer in enumerate(model.transformer_encoder.layers):
            def lh(_m, _a, out, li=li):
                taps[f"layer{li}"] = out[0].detach().numpy().copy()
            if li == 0:
                hooks.append(layer.register_forward_hook(lh))
    if image is not None:
        mix = getattr(model, {"MGM+CAP": "cap", "MGM": "mgm", "MoE": "moe"}[cfg.mixer_type])
        def mh(_m, _a, out):
            taps["mixer_tokens"] = out[0].detach().numpy().copy()
        hooks.append(mix.register_forward_hook(mh))

    torch.manual_seed(0)
    with torch.inference_mode():
        out = model(
            None,
            torch.from_numpy(x[:, None, :]) if x is not None else None,
            torch.from_numpy(image) if image is not None else None,
            torch.from_numpy(y[:N]),
            only_return_standard_out=True,
            categorical_inds=list(range(case["data"].get("n_cat", 0))),
            single_eval_pos=N,
        )
    for h in hooks:
        h.remove()
    res = {
        "logits": out.squeeze(1).numpy().astype(np.float32),
        "y_train": y[:N],
        "meta": np.array(json.dumps({k: case[k] for k in case if k != "taps"} | {"cfg": case["cfg"]})),
    }
    if x is not None:
        res["x"] = x
    if image is not None:
        res["image"] = image
    res.update({k: v.astype(np.float32) for k, v in taps.items()})
    return res


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    only = set(sys.argv[1:])
    for case in CASES:
        if only and case["name"] not in only:
            continue
        res = run_case(case)
        path = HERE / f"{case['name']}.npz"
        np.savez_compressed(path, **res)
        print(f"{case['name']}: logits {res['logits'].shape} -> {path.name} ({path.stat().st_size/1e3:.0f} kB)")


if __name__ == "__main__":
    main()
