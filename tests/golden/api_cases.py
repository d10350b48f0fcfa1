"""Classifier-level test cases shared by ``make_api_golden.py`` and the API tests.

Each case fixes the model (checkpoint config + synthetic weight seed), the
classifier arguments, the ``ModelInterfaceConfig`` overrides and the data
generator.  Data are regenerated from seeds (only outputs are stored).
"""

from __future__ import annotations

import numpy as np

from synth import synth_image, synth_table

CASES = [
    # SURVEY 8d case A shape: 500 x 20 numeric, two classes, default preprocessing
    # (quantile + SVD member and raw member, fingerprint feature), tabular only
    dict(name="tab_default", model=dict(nlayers=2, mgm_heads=2, cap_heads=2), wseed=21,
         clf=dict(mixer_type="MGM+CAP", mgm_heads=2, cap_heads=2, features_per_group=2, n_estimators=4,
                  random_state=0),
         data=dict(kind="case_a", S=500, N=400, F=20, seed=0)),
    # PAD-UFES shape with run.py's no-preprocessing interface config, image modality
    dict(name="pad_none", model=dict(nlayers=2, mgm_heads=4, cap_heads=2), wseed=22,
         clf=dict(mixer_type="MGM+CAP", mgm_heads=4, cap_heads=2, features_per_group=2, n_estimators=4,
                  categorical_features_indices=list(range(18)), ignore_pretraining_limits=True, random_state=0),
         interface=dict(FINGERPRINT_FEATURE=False, PREPROCESS_TRANSFORMS=[dict(name="none")]),
         data=dict(kind="pad", S=300, N=240, F=21, n_cat=18, n_classes=6, n_mod=1, seed=2)),
    # rotate shifts, row sub-sampling, polynomial features, mixed transforms, leftover pick
    dict(name="variants", model=dict(nlayers=1, mixer_type="MGM", mgm_heads=2, cap_heads=2), wseed=23,
         clf=dict(mixer_type="MGM", mgm_heads=2, cap_heads=2, features_per_group=2, n_estimators=5,
                  categorical_features_indices=[0, 1, 2], softmax_temperature=0.8, average_before_softmax=True,
                  balance_probabilities=True, random_state=3),
         interface=dict(FEATURE_SHIFT_METHOD="rotate", CLASS_SHIFT_METHOD="rotate", SUBSAMPLE_SAMPLES=150,
                        POLYNOMIAL_FEATURES=4,
                        PREPROCESS_TRANSFORMS=[
                            dict(name="quantile_norm", categorical_name="onehot"),
                            dict(name="robust", categorical_name="ordinal_shuffled", append_original=True),
                            dict(name="power", categorical_name="numeric", global_transformer_name="scaler"),
                        ]),
         data=dict(kind="pad", S=260, N=200, F=9, n_cat=3, n_classes=4, n_mod=0, nan_frac=0.05, seed=5)),
    # image only (X is None), MoE mixer
    dict(name="image_only", model=dict(nlayers=1, mixer_type="MoE", mgm_heads=3, cap_heads=2), wseed=24,
         clf=dict(mixer_type="MoE", mgm_heads=3, cap_heads=2, features_per_group=2, n_estimators=3,
                  random_state=1),
         data=dict(kind="image_only", S=120, N=90, n_classes=3, n_mod=1, seed=7)),
]


def case_data(case: dict) -> dict:
    d = case["data"]
    S, N = d["S"], d["N"]
    g = np.random.default_rng(d["seed"])
    out: dict = {"X_train": None, "X_test": None, "image_train": None, "image_test": None}
    if d["kind"] == "case_a":
        X = g.standard_normal((S, d["F"]))
        y = (X[:, 0] + 0.5 * X[:, 1] > 0).astype(np.int64)
    else:
        n_cls = d["n_classes"]
        y = g.integers(0, n_cls, size=S)
        y[:n_cls] = np.arange(n_cls)
        X = None
        if d["kind"] == "pad":
            X = synth_table(S, d["F"], d["seed"], n_cat=d.get("n_cat", 0), nan_frac=d.get("nan_frac", 0.0))
            X = X.astype(np.float64)
        if d.get("n_mod", 0) or d["kind"] == "image_only":
            im = synth_image(S, max(1, d.get("n_mod", 1)), d["seed"])
            out["image_train"], out["image_test"] = im[:N], im[N:]
    if X is not None:
        out["X_train"], out["X_test"] = X[:N], X[N:]
    out["y_train"], out["y_test"] = y[:N], y[N:]
    return out


def ckpt_config(cfg) -> dict:
    """``InferenceConfig`` dict of a synthetic checkpoint (``model/config.py:18-108``)."""
    return {
        "adaptive_max_seq_len_to_max_full_table_size": 150000,
        "batch_size": 8,
        "aggregate_k_gradients": 1,
        "emsize": cfg.emsize,
        "features_per_group": cfg.encoder_features,
        "max_num_classes": cfg.max_num_classes,
        "nhead": cfg.nhead,
        "nlayers": cfg.nlayers,
        "remove_duplicate_features": cfg.remove_duplicate_features,
        "seq_len": 4000,
        "task_type": "multiclass",
        "num_buckets": 5000,
        "max_num_features": 85,
        "two_sets_of_queries": cfg.two_sets_of_queries,
    }
