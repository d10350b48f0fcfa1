"""Host side of the classifier against the reference's API-level goldens (CPU).

``tests/golden/api_*.npz`` hold, per ensemble member, what the reference
``MMPFNClassifier.fit`` produced (``make_api_golden.py``): preprocessed train /
test tables, permuted labels, categorical indices, class permutation, feature
shift.  Here the same checkpoint and data go through this package's ``fit``
(host work only, no GPU needed) and every member must match exactly.
"""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE / "golden"))

from api_cases import CASES, case_data, ckpt_config  # noqa: E402
from synth import synth_state_dict  # noqa: E402

from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec  # noqa: E402

NAMES = [c["name"] for c in CASES]


def _case(name):
    return next(c for c in CASES if c["name"] == name)


def write_ckpt(case, tmp: Path) -> Path:
    cfg = ModelConfig(**case["model"])
    sd = synth_state_dict(state_dict_spec(cfg), case["wseed"])
    p = tmp / f"{case['name']}.ckpt"
    torch.save({"state_dict": {k: torch.from_numpy(v) for k, v in sd.items()}, "config": ckpt_config(cfg)}, p)
    return p


def make_classifier(case, ckpt: Path, **over):
    from multimodalpfn_amd import MMPFNClassifier
    from multimodalpfn_amd.constants import ModelInterfaceConfig
    from multimodalpfn_amd.preprocessing import PreprocessorConfig

    ic = dict(case.get("interface", {}))
    if "PREPROCESS_TRANSFORMS" in ic:
        ic["PREPROCESS_TRANSFORMS"] = [PreprocessorConfig(**p) for p in ic["PREPROCESS_TRANSFORMS"]]
    kw = dict(case["clf"]) | over
    return MMPFNClassifier(model_path=str(ckpt), inference_config=ModelInterfaceConfig(**ic) if ic else None, **kw)


def _eq(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    if a.dtype.kind == "f" or b.dtype.kind == "f":
        np.testing.assert_allclose(a.astype(np.float64), b.astype(np.float64), rtol=1e-12, atol=1e-12,
                                   equal_nan=True, err_msg=what)
    else:
        np.testing.assert_array_equal(a, b, err_msg=what)


@pytest.mark.parametrize("name", NAMES)
def test_fit_members_match_reference(name, tmp_path):
    case = _case(name)
    z = np.load(HERE / "golden" / f"api_{name}.npz")
    d = case_data(case)
    clf = make_classifier(case, write_ckpt(case, tmp_path), device="cpu")
    clf.fit(d["X_train"], d["image_train"], d["y_train"])
    _eq(clf.classes_, z["classes"], "classes_")
    _eq(clf.inferred_categorical_indices_, z["inferred_cat"], "inferred categorical")
    ex = clf.executor_
    n = len(ex.ensemble_configs)
    assert n == case["clf"]["n_estimators"]
    for m, c in enumerate(ex.ensemble_configs):
        assert str(c.preprocess_config) == str(z[f"m{m}_pp"]), m
        assert int(c.feature_shift_count) == int(z[f"m{m}_feature_shift"]), m
        if f"m{m}_class_perm" in z:
            _eq(c.class_permutation, z[f"m{m}_class_perm"], f"m{m} class perm")
        else:
            assert c.class_permutation is None
        if f"m{m}_subsample" in z:
            _eq(c.subsample_ix, z[f"m{m}_subsample"], f"m{m} subsample")
        _eq(ex.y_trains[m], z[f"m{m}_y_train"], f"m{m} y_train")
        if f"m{m}_X_train" in z:
            _eq(ex.X_trains[m], z[f"m{m}_X_train"], f"m{m} X_train")
            _eq(ex.cat_ixs[m], z[f"m{m}_cat_ix"], f"m{m} cat_ix")
            from multimodalpfn_amd.utils import _fix_dtypes

            X_enc = clf.preprocessor_.transform(_fix_dtypes(d["X_test"], cat_indices=clf.categorical_features_indices))
            _eq(ex.preprocessors[m].transform(X_enc).X, z[f"m{m}_X_test"], f"m{m} X_test")
        else:
            assert ex.X_trains[m] is None


def test_fingerprint_matches_python_hash_seed0():
    """The vectorised SipHash equals CPython's ``hash(bytes)`` under PYTHONHASHSEED=0."""
    import os
    import subprocess

    from multimodalpfn_amd.model._siphash import siphash24_rows

    rows = np.random.default_rng(3).standard_normal((6, 5))
    rows[2] = rows[1]
    odd = np.frombuffer(b"abcdefghijklmnopqrstu", dtype=np.uint8).reshape(3, 7)
    code = (
        "import numpy as np,sys;"
        "r=np.random.default_rng(3).standard_normal((6,5));r[2]=r[1];"
        "o=np.frombuffer(b'abcdefghijklmnopqrstu',dtype=np.uint8).reshape(3,7);"
        "print(' '.join(str(hash(x.tobytes())) for x in list(r)+list(o)))"
    )
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, PYTHONHASHSEED="0"),
                         capture_output=True, text=True, check=True).stdout.split()
    mine = list(siphash24_rows(rows)) + list(siphash24_rows(odd))
    assert [int(v) for v in mine] == [int(v) for v in out]


def test_native_row_hash_equals_the_numpy_restatement():
    """The library's host hash (``mmpfn_siphash24_rows``) equals the numpy SipHash on every tail length."""
    from multimodalpfn_amd.model import _siphash

    if _siphash._native() is None:
        pytest.skip("library not built")
    rng = np.random.default_rng(5)
    for nb in range(0, 41):
        a = rng.integers(0, 256, (11, nb), dtype=np.uint8)
        assert (_siphash.siphash24_rows(a) == _siphash.siphash24_rows_numpy(a)).all(), nb
    a = rng.standard_normal((460, 36))
    a[3] = a[2]
    assert (_siphash.siphash24_rows(a) == _siphash.siphash24_rows_numpy(a)).all()
    assert _siphash.siphash24_rows(np.zeros((0, 3))).shape == (0,)


def test_interface_config_from_user_input():
    from multimodalpfn_amd.constants import ModelInterfaceConfig

    c = ModelInterfaceConfig.from_user_input(inference_config={"FINGERPRINT_FEATURE": False})
    assert c.FINGERPRINT_FEATURE is False and c.OUTLIER_REMOVAL_STD == "auto"
    with pytest.raises(ValueError, match="Unknown kwarg"):
        ModelInterfaceConfig.from_user_input(inference_config={"NOPE": 1})


def test_checkpoint_missing_weight_semantics(tmp_path):
    """strict=False (loading.py:540): a missing modality-head tensor keeps its init (warning);
    a missing trunk tensor is an error naming it."""
    from multimodalpfn_amd.model.loading import load_model

    case = _case("pad_none")
    p = write_ckpt(case, tmp_path)
    ck = torch.load(p, weights_only=True)
    del ck["state_dict"]["cap.queries"]
    torch.save(ck, p)
    with pytest.warns(UserWarning, match="cap"):
        load_model(path=p, model_seed=0, mixer_type="MGM+CAP", mgm_heads=4, cap_heads=2, features_per_group=2)
    del ck["state_dict"]["decoder_dict.standard.0.bias"]
    torch.save(ck, p)
    with pytest.raises(ValueError, match="decoder_dict.standard.0.bias"):
        load_model(path=p, model_seed=0, mixer_type="MGM+CAP", mgm_heads=4, cap_heads=2, features_per_group=2)


def test_predict_without_gpu_fails_loudly(tmp_path):
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    case = _case("pad_none")
    d = case_data(case)
    clf = make_classifier(case, write_ckpt(case, tmp_path))
    clf.fit(d["X_train"], d["image_train"], d["y_train"])
    with pytest.raises(RuntimeError, match="no ROCm GPU"):
        clf.predict_proba(d["X_test"], d["image_test"])


@pytest.mark.parametrize("name", NAMES)
def test_numpy_predict_encoding_matches_pandas_route(name, tmp_path):
    """The numpy fast path of predict-time encoding equals _fix_dtypes + ColumnTransformer."""
    from multimodalpfn_amd.utils import _fix_dtypes, validate_X_predict

    case = _case(name)
    d = case_data(case)
    if d["X_train"] is None:
        pytest.skip("image-only case")
    clf = make_classifier(case, write_ckpt(case, tmp_path), device="cpu")
    clf.fit(d["X_train"], d["image_train"], d["y_train"])
    assert clf._ordinal_plan_ is not None
    Xt = d["X_test"].copy()
    g = np.random.default_rng(0)
    Xt[g.random(Xt.shape) < 0.05] = np.nan  # missing values
    Xt[0, :] = 97.0  # unseen categories
    Xt[1, :] = -0.0  # signed zero (equal to a fitted 0.0)
    if len(Xt) > 3:  # the categories of the next column (the vectorised search must keep columns apart)
        Xt[2, :-1] = Xt[3, 1:]
    fast = clf._encode_predict_X(Xt)
    slow = clf.preprocessor_.transform(_fix_dtypes(validate_X_predict(Xt, clf),
                                                   cat_indices=clf.categorical_features_indices))
    np.testing.assert_array_equal(fast, np.asarray(slow, dtype=np.float64))


@pytest.mark.parametrize("name", NAMES)
def test_passthrough_member_transform_fast_path(name, tmp_path):
    """A member table that only passes columns through ("none" with no global transformer) is taken as a column
    selection at predict (ReshapeFeatureDistributionsStep.select_cols_): the same values as its ColumnTransformer."""
    from multimodalpfn_amd.model.preprocessing import ReshapeFeatureDistributionsStep

    case = _case(name)
    d = case_data(case)
    if d["X_train"] is None:
        pytest.skip("image-only case")
    clf = make_classifier(case, write_ckpt(case, tmp_path), device="cpu")
    clf.fit(d["X_train"], d["image_train"], d["y_train"])
    Xe = clf._encode_predict_X(d["X_test"])
    seen = 0
    for pre in clf.executor_.preprocessors:
        X = Xe
        for step in pre:
            if isinstance(step, ReshapeFeatureDistributionsStep):
                fast = step._transform(X, is_test=True)
                slow = step.transformer_.transform(X[:, step.subsampled_features_])
                np.testing.assert_array_equal(fast, slow)
                assert fast.dtype == slow.dtype
                seen += step.select_cols_ is not None
            X = step.transform(X).X
    if name == "pad_none":
        assert seen > 0  # run.py's members take the fast path


@pytest.mark.parametrize("scale", [1.0, 0.5])
def test_numpy_predict_encoding_with_missing_categories_at_fit(tmp_path, scale):
    """Categorical columns that held NaN at fit (missing is then a fitted category: NaN stays NaN) and columns that
    did not (missing -> -1), through the numpy path against the ColumnTransformer route: integer categories take the
    lookup table, half-integer ones (scale 0.5) the per-column search."""
    from multimodalpfn_amd.utils import _fix_dtypes, validate_X_predict

    case = _case("pad_none")
    d = case_data(case)
    clf = make_classifier(case, write_ckpt(case, tmp_path), device="cpu")
    Xtr = d["X_train"].copy() * scale
    Xtr[::7, 0] = np.nan
    Xtr[::5, 3] = np.nan
    clf.fit(Xtr, d["image_train"], d["y_train"])
    if clf._ordinal_plan_ is None:
        pytest.skip("encoder plan not numeric")
    assert (clf._ordinal_plan_[3] is None) == (scale != 1.0)
    Xt = d["X_test"].copy() * scale
    Xt[::3, :] = np.nan
    Xt[1, :] = 55.0
    Xt[2, :] = 0.5
    fast = clf._encode_predict_X(Xt)
    slow = clf.preprocessor_.transform(_fix_dtypes(validate_X_predict(Xt, clf),
                                                   cat_indices=clf.categorical_features_indices))
    np.testing.assert_array_equal(fast, np.asarray(slow, dtype=np.float64))
