"""End-to-end classifier parity on the GPU against the reference's API-level goldens.

Same checkpoint, data and interface config as ``make_api_golden.py``; the
reference ran fit/predict_proba on CPU in fp32.  fp32 mode (forced
``inference_precision=torch.float32``) must reproduce every member's logits to
1e-4 relative and the ensemble probabilities to 1e-5 absolute; the bf16 mode
(the default "auto" on a GPU) is held to a loose band and argmax agreement.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from helpers import check_argmax

from test_api_host import HERE, NAMES, _case, case_data, make_classifier, write_ckpt

pytestmark = pytest.mark.gpu

LOGIT_RTOL = 1e-4
PROBA_ATOL = 1e-5


def _spy(clf):
    captured = []
    orig = clf.executor_.iter_outputs

    def spy(*a, **k):
        for out, c in orig(*a, **k):
            captured.append(out.detach().float().cpu().numpy())
            yield out, c

    clf.executor_.iter_outputs = spy
    return captured


@pytest.mark.parametrize("name", NAMES)
def test_predict_proba_fp32_matches_reference(name, tmp_path):
    case = _case(name)
    z = np.load(HERE / "golden" / f"api_{name}.npz")
    d = case_data(case)
    clf = make_classifier(case, write_ckpt(case, tmp_path), inference_precision=torch.float32)
    clf.fit(d["X_train"], d["image_train"], d["y_train"])
    got = _spy(clf)
    proba = clf.predict_proba(d["X_test"], d["image_test"])
    for m, lg in enumerate(got):
        ref = z[f"m{m}_logits"]
        err = np.abs(lg - ref).max() / max(np.abs(ref).max(), 1e-6)
        assert err < LOGIT_RTOL, (m, err)
    np.testing.assert_allclose(proba, z["proba"], atol=PROBA_ATOL, rtol=0)
    np.testing.assert_array_equal(clf.predict(d["X_test"], d["image_test"]), z["pred"])


@pytest.mark.parametrize("mode", ["f16", "bf16"])
@pytest.mark.parametrize("name", NAMES)
def test_predict_proba_16bit_close(name, mode, tmp_path, monkeypatch):
    """inference_precision="auto" on a GPU = the reference's fp16 autocast: MMPFN_PREC_F16 (default), or the
    bf16-operand mode under MMPFN_AUTOCAST=bf16."""
    monkeypatch.setenv("MMPFN_AUTOCAST", mode)
    case = _case(name)
    z = np.load(HERE / "golden" / f"api_{name}.npz")
    d = case_data(case)
    clf = make_classifier(case, write_ckpt(case, tmp_path))  # "auto" -> autocast -> the 16-bit engine mode
    clf.fit(d["X_train"], d["image_train"], d["y_train"])
    assert clf.use_autocast_
    proba = clf.predict_proba(d["X_test"], d["image_test"])
    err = np.abs(proba - z["proba"]).max()
    print(f"{name}: {mode} proba max |err| {err:.3e}")
    assert err < (3e-2 if mode == "bf16" else 5e-3), err
    check_argmax(proba, z["proba"], 0.995, f"api {name} {mode}")


@pytest.mark.parametrize("fit_mode", ["fit_preprocessors", "low_memory"])
def test_early_mixer_launch(fit_mode, tmp_path, monkeypatch):
    """predict_proba enqueues the test rows' modality tokens before it validates / encodes X
    (``InferenceEngine.launch_mixer_early``); the member loop must take exactly those tokens, and the result must
    equal the predict without the early launch bitwise.  An image of the wrong width is left to the regular path
    and its error."""
    from multimodalpfn_amd import inference

    case = _case("pad_none")
    d = case_data(case)
    clf = make_classifier(case, write_ckpt(case, tmp_path), inference_precision=torch.float32, fit_mode=fit_mode)
    clf.fit(d["X_train"], d["image_train"], d["y_train"])
    calls = []
    orig = inference._mixer_tokens
    monkeypatch.setattr(inference, "_mixer_tokens", lambda *a, **k: calls.append(1) or orig(*a, **k))
    a = clf.predict_proba(d["X_test"], d["image_test"])
    assert len(calls) == 1 and clf.executor_._early_tokens is None
    monkeypatch.setattr(type(clf.executor_), "launch_mixer_early", lambda self, *a, **k: None)
    b = clf.predict_proba(d["X_test"], d["image_test"])
    assert len(calls) == 2
    np.testing.assert_array_equal(a, b)
    monkeypatch.undo()
    bad = np.concatenate([d["image_test"], d["image_test"][..., :1]], axis=-1)
    with pytest.raises(ValueError):
        clf.predict_proba(d["X_test"], bad)


def test_deferred_status_survives_a_failed_aggregation(tmp_path, monkeypatch):
    """predict_proba waits for the member loop (and checks its NaN flags) after the aggregation is enqueued
    (``InferenceEngine.check_status``).  An error between the loop and the aggregation must still run that check
    -- no pending wait is left behind for the next predict -- and the next predict equals a clean one."""
    from multimodalpfn_amd.engine import HipEngine

    case = _case("pad_none")
    d = case_data(case)
    clf = make_classifier(case, write_ckpt(case, tmp_path), inference_precision=torch.float32)
    clf.fit(d["X_train"], d["image_train"], d["y_train"])
    ref = clf.predict_proba(d["X_test"], d["image_test"])

    def boom(*a, **k):
        raise RuntimeError("injected")

    monkeypatch.setattr(HipEngine, "aggregate", boom)
    with pytest.raises(RuntimeError, match="injected"):
        clf.predict_proba(d["X_test"], d["image_test"])
    assert clf.executor_._pending_status is None and not clf.executor_._defer_status
    monkeypatch.undo()
    np.testing.assert_array_equal(clf.predict_proba(d["X_test"], d["image_test"]), ref)

    # an error inside the member loop's consumer (after _run_members deferred its check) and one in X's
    # validation (after the early mixer was queued): no pending check, no early tokens left behind
    ex = clf.executor_
    real_iter = type(ex).iter_outputs

    def bad_iter(self, *a, **k):
        for out, cfg in real_iter(self, *a, **k):
            yield out[None], cfg  # 3-D: the loop body's shape assertion fires
    monkeypatch.setattr(type(ex), "iter_outputs", bad_iter)
    with pytest.raises(AssertionError):
        clf.predict_proba(d["X_test"], d["image_test"])
    assert ex._pending_status is None and not ex._defer_status and ex._early_tokens is None
    monkeypatch.undo()
    with pytest.raises(ValueError):
        clf.predict_proba(d["X_test"][:, :1], d["image_test"])  # wrong width: X validation raises
    assert ex._pending_status is None and ex._early_tokens is None
    np.testing.assert_array_equal(clf.predict_proba(d["X_test"], d["image_test"]), ref)


def test_low_memory_mode_is_reproducible(tmp_path):
    """``low_memory`` re-fits members at every predict from one fixed seed (inference.py:148)."""
    case = _case("pad_none")
    d = case_data(case)
    clf = make_classifier(case, write_ckpt(case, tmp_path), inference_precision=torch.float32,
                          fit_mode="low_memory")
    clf.fit(d["X_train"], d["image_train"], d["y_train"])
    a = clf.predict_proba(d["X_test"], d["image_test"])
    b = clf.predict_proba(d["X_test"], d["image_test"])
    np.testing.assert_array_equal(a, b)
    np.testing.assert_allclose(a.sum(1), 1.0, atol=1e-6)


@pytest.mark.parametrize("name", NAMES)
def test_fit_with_cache_matches_reference(name, tmp_path):
    """``fit_mode="fit_with_cache"``: train rows forwarded once at fit (train-KV cache on the
    device), predict forwards the test rows only; same member logits as the reference's
    fit_preprocessors goldens, twice in a row from one cache."""
    case = _case(name)
    z = np.load(HERE / "golden" / f"api_{name}.npz")
    d = case_data(case)
    clf = make_classifier(case, write_ckpt(case, tmp_path), inference_precision=torch.float32,
                          fit_mode="fit_with_cache")
    clf.fit(d["X_train"], d["image_train"], d["y_train"])
    got = _spy(clf)
    proba = clf.predict_proba(d["X_test"], d["image_test"])
    for m, lg in enumerate(got):
        ref = z[f"m{m}_logits"]
        err = np.abs(lg - ref).max() / max(np.abs(ref).max(), 1e-6)
        assert err < LOGIT_RTOL, (m, err)
    np.testing.assert_allclose(proba, z["proba"], atol=PROBA_ATOL, rtol=0)
    np.testing.assert_array_equal(clf.predict_proba(d["X_test"], d["image_test"]), proba)


_FIT_MATRIX = [(fs, cs, fm, ip, ro)
               for fs in ("shuffle", "rotate")
               for cs in ("shuffle", "rotate")
               for fm in ("low_memory", "fit_preprocessors", "fit_with_cache")
               for ip in ("auto", "autocast", torch.float64)
               for ro in (None, 12)]


@pytest.fixture(scope="module")
def iris_ckpt(tmp_path_factory):
    return write_ckpt(_case("tab_default"), tmp_path_factory.mktemp("iris"))


@pytest.mark.parametrize("feature_shift,class_shift,fit_mode,precision,outlier_std", _FIT_MATRIX)
def test_fit_matrix(feature_shift, class_shift, fit_mode, precision, outlier_std, iris_ckpt):
    """The reference's ``tests/test_classifier_interface.py:47-94`` matrix (shift decoders x
    fit modes x inference precision x outlier removal) on iris, tabular only: ``fit`` returns
    the estimator, it is fitted, probabilities are ``[n, n_classes]`` rows summing to 1 and
    ``predict`` is ``[n]`` of the train labels."""
    import sklearn.datasets
    from sklearn.utils.validation import check_is_fitted

    from multimodalpfn_amd import MMPFNClassifier

    X, y = sklearn.datasets.load_iris(return_X_y=True)
    clf = MMPFNClassifier(model_path=str(iris_ckpt), device="cuda", fit_mode=fit_mode,
                          inference_precision=precision, mixer_type="MGM+CAP", mgm_heads=2, cap_heads=2,
                          features_per_group=2,
                          inference_config={"OUTLIER_REMOVAL_STD": outlier_std,
                                            "CLASS_SHIFT_METHOD": class_shift,
                                            "FEATURE_SHIFT_METHOD": feature_shift})
    assert clf.fit(X, None, y) is clf
    check_is_fitted(clf)
    assert clf.use_autocast_ == (precision != torch.float64)
    proba = clf.predict_proba(X, None)
    assert proba.shape == (X.shape[0], len(np.unique(y)))
    assert np.isfinite(proba).all()
    np.testing.assert_allclose(proba.sum(1), 1.0, atol=1e-5)
    pred = clf.predict(X, None)
    assert pred.shape == (X.shape[0],)
    assert set(np.unique(pred)) <= set(np.unique(y))
