"""``MMPFNClassifier``: the reference's scikit-learn interface over the HIP engine.

Same constructor (``mmpfn/models/mmpfn/classifier.py:112-137``), same ``fit(X,
image, y)`` / ``predict(X, X_image)`` / ``predict_proba(X, image_test)`` and
fitted attributes.  Host-side work (validation, ordinal encoding, categorical
inference, member preprocessing) is the reference's algorithm on numpy /
scikit-learn; every forward runs in ``libmmpfn_hip.so`` on an MI355X, and the
ensemble post-processing (temperature, class un-permutation, softmax, member
mean, class balancing; ``classifier.py:541-566``) runs in one HIP kernel on the
logits already resident in HBM.  There is no CPU forward: without a ROCm GPU
``fit`` succeeds (host work only) and ``predict_proba`` raises ``RuntimeError``.
"""

from __future__ import annotations

from collections.abc import Sequence
from pathlib import Path
from typing import Any, Literal

import os

import numpy as np
import torch
from sklearn.base import BaseEstimator, ClassifierMixin, check_is_fitted
from sklearn.preprocessing import LabelEncoder

from multimodalpfn_amd.base import create_inference_engine, determine_precision, initialize_mmpfn_model
from multimodalpfn_amd.constants import (
    PROBABILITY_EPSILON_ROUND_ZERO,
    SKLEARN_16_DECIMAL_PRECISION,
    ModelInterfaceConfig,
)
from multimodalpfn_amd.preprocessing import EnsembleConfig, default_classifier_preprocessor_configs
from multimodalpfn_amd.utils import (
    _fix_dtypes,
    _get_ordinal_encoder,
    infer_categorical_features,
    infer_device_and_type,
    infer_random_state,
    update_encoder_outlier_params,
    validate_X_predict,
    validate_Xy_fit,
)


class MMPFNClassifier(ClassifierMixin, BaseEstimator):
    """Multimodal PFN classifier (tabular + image/text embeddings), MI355X engine."""

    def __init__(
        self,
        *,
        mixer_type: str,
        mgm_heads: int,
        cap_heads: int,
        features_per_group: int,
        n_estimators: int = 4,
        categorical_features_indices: Sequence[int] | None = None,
        softmax_temperature: float = 0.9,
        balance_probabilities: bool = False,
        average_before_softmax: bool = False,
        model_path: str | Path | Literal["auto"] = "auto",
        device: str | torch.device | Literal["auto"] = "auto",
        ignore_pretraining_limits: bool = False,
        inference_precision: torch.dtype | Literal["autocast", "auto"] = "auto",
        fit_mode: Literal["low_memory", "fit_preprocessors", "fit_with_cache"] = "fit_preprocessors",
        memory_saving_mode: bool | Literal["auto"] | float | int = "auto",
        random_state: int | np.random.RandomState | np.random.Generator | None = 0,
        n_jobs: int = -1,
        inference_config: dict | ModelInterfaceConfig | None = None,
    ) -> None:
        super().__init__()
        self.n_estimators = n_estimators
        self.categorical_features_indices = categorical_features_indices
        self.softmax_temperature = softmax_temperature
        self.balance_probabilities = balance_probabilities
        self.average_before_softmax = average_before_softmax
        self.model_path = model_path
        self.device = device
        self.ignore_pretraining_limits = ignore_pretraining_limits
        self.inference_precision = inference_precision
        self.fit_mode = fit_mode
        self.memory_saving_mode = memory_saving_mode
        self.random_state = random_state
        self.n_jobs = n_jobs
        self.inference_config = inference_config
        self.mixer_type = mixer_type
        self.mgm_heads = mgm_heads
        self.cap_heads = cap_heads
        self.features_per_group = features_per_group

    def _more_tags(self) -> dict[str, Any]:
        return {"allow_nan": True, "multilabel": False}

    def __sklearn_tags__(self):
        tags = super().__sklearn_tags__()
        tags.input_tags.allow_nan = True
        tags.estimator_type = "classifier"
        return tags

    # ------------------------------------------------------------------ fit
    def fit(self, X, image: np.ndarray | None, y):
        """``classifier.py:364-502``: load the model, encode inputs, build and fit the members."""
        static_seed, rng = infer_random_state(self.random_state)
        self.model_, self.config_, _ = initialize_mmpfn_model(
            model_path=self.model_path,
            which="classifier",
            fit_mode=self.fit_mode,
            static_seed=static_seed,
            mixer_type=self.mixer_type,
            mgm_heads=self.mgm_heads,
            cap_heads=self.cap_heads,
            features_per_group=self.features_per_group,
        )
        self.device_ = infer_device_and_type(self.device)
        self.use_autocast_, self.forced_inference_dtype_, byte_size = determine_precision(
            self.inference_precision, self.device_
        )
        self.interface_config_ = ModelInterfaceConfig.from_user_input(inference_config=self.inference_config)
        sigma = self.interface_config_.OUTLIER_REMOVAL_STD
        if sigma == "auto":
            sigma = self.interface_config_._CLASSIFICATION_DEFAULT_OUTLIER_REMOVAL_STD
        update_encoder_outlier_params(model=self.model_, remove_outliers_std=sigma, seed=static_seed, inplace=True)

        if X is not None:
            X, y, names, n_in = validate_Xy_fit(
                X,
                y,
                estimator=self,
                ensure_y_numeric=False,
                max_num_samples=self.interface_config_.MAX_NUMBER_OF_SAMPLES,
                max_num_features=self.interface_config_.MAX_NUMBER_OF_FEATURES,
                ignore_pretraining_limits=self.ignore_pretraining_limits,
            )
            if names is not None:
                self.feature_names_in_ = names
            self.n_features_in_ = n_in

        _, counts = np.unique(y, return_counts=True)
        self.class_counts_ = counts
        self.label_encoder_ = LabelEncoder()
        y = self.label_encoder_.fit_transform(y)
        self.classes_ = self.label_encoder_.classes_
        self.n_classes_ = len(self.classes_)
        if self.n_classes_ > self.interface_config_.MAX_NUMBER_OF_CLASSES:
            raise ValueError(
                f"Number of classes {self.n_classes_} exceeds the maximal number of classes supported by TabPFN. "
                "Consider using a strategy to reduce the number of classes (e.g., OneVsRest)."
            )

        if X is not None:
            X = _fix_dtypes(X, cat_indices=self.categorical_features_indices)
            enc = _get_ordinal_encoder()
            X = enc.fit_transform(X)
            assert isinstance(X, np.ndarray)
            self.preprocessor_ = enc
            self._plan_ordinal()
            ic = self.interface_config_
            self.inferred_categorical_indices_ = infer_categorical_features(
                X=X,
                provided=self.categorical_features_indices,
                min_samples_for_inference=ic.MIN_NUMBER_SAMPLES_FOR_CATEGORICAL_INFERENCE,
                max_unique_for_category=ic.MAX_UNIQUE_FOR_CATEGORICAL_FEATURES,
                min_unique_for_numerical=ic.MIN_UNIQUE_FOR_NUMERICAL_FEATURES,
            )
            max_index = len(X)
        else:
            self.inferred_categorical_indices_ = []
            max_index = len(image)

        ic = self.interface_config_
        configs = EnsembleConfig.generate_for_classification(
            n=self.n_estimators,
            subsample_size=ic.SUBSAMPLE_SAMPLES,
            add_fingerprint_feature=ic.FINGERPRINT_FEATURE,
            feature_shift_decoder=ic.FEATURE_SHIFT_METHOD,
            polynomial_features=ic.POLYNOMIAL_FEATURES,
            max_index=max_index,
            preprocessor_configs=(
                ic.PREPROCESS_TRANSFORMS if ic.PREPROCESS_TRANSFORMS is not None
                else default_classifier_preprocessor_configs()
            ),
            class_shift_method=ic.CLASS_SHIFT_METHOD,
            n_classes=self.n_classes_,
            random_state=rng,
        )
        assert len(configs) == self.n_estimators
        self.executor_ = create_inference_engine(
            X_train=X,
            y_train=y,
            image_train=image,
            model=self.model_,
            ensemble_configs=configs,
            cat_ix=self.inferred_categorical_indices_,
            fit_mode=self.fit_mode,
            device_=self.device_,
            rng=rng,
            n_jobs=self.n_jobs,
            byte_size=byte_size,
            forced_inference_dtype_=self.forced_inference_dtype_,
            memory_saving_mode=self.memory_saving_mode,
            use_autocast_=self.use_autocast_,
        )
        return self

    # ------------------------------------------------------------------ predict
    def _encode_predict_X(self, X) -> np.ndarray:
        """validate -> _fix_dtypes -> fitted ordinal encoder (``classifier.py:529-532``).

        A plain numeric ndarray (the run.py case) takes a numpy path computing the same
        table as the pandas / ColumnTransformer route in ~1/20 of its time: categorical
        columns map to their index in the fitted sorted categories (unseen -> -1,
        missing -> NaN), encoded columns first, then the remainder in order
        (``tests/test_api_host.py`` checks the two routes agree).
        """
        X = validate_X_predict(X, self)
        fast = getattr(self, "_ordinal_plan_", None)
        if fast is not None and isinstance(X, np.ndarray) and X.dtype.kind in "biuf" and X.ndim == 2:
            Xf = X.astype(np.float64, copy=False)
            cols, cats, miss, lut, rem = fast
            out = np.empty((Xf.shape[0], len(cols) + len(rem)), dtype=np.float64)
            if cols:
                v = Xf[:, cols]
                if lut is not None:
                    # integer categories in a small range (the usual case): one table lookup for every encoded
                    # column at once; a value that is not an integer of the column's range is unseen (-1)
                    lo, table = lut
                    vi = np.floor(v)
                    pos = vi - lo
                    ok = (vi == v) & (pos >= 0) & (pos < table.shape[1])
                    idx = np.where(ok, pos, 0).astype(np.intp)
                    enc = np.where(ok, table[np.arange(len(cols)), idx], -1.0)
                else:
                    enc = np.empty(v.shape)
                    for k, c in enumerate(cats):
                        idx = np.searchsorted(c, v[:, k])
                        hit = c[np.minimum(idx, len(c) - 1)] == v[:, k] if len(c) else np.zeros(len(v), bool)
                        enc[:, k] = np.where(hit, idx, -1.0)
                # missing -> NaN only if missing was a fitted category, else it is unseen (-1)
                out[:, :len(cols)] = np.where(np.isnan(v), miss, enc)
            if rem:
                out[:, len(cols):] = Xf[:, rem]
            return out
        X = _fix_dtypes(X, cat_indices=self.categorical_features_indices)
        return self.preprocessor_.transform(X)

    def _plan_ordinal(self) -> None:
        """Record the fitted encoder's column plan for the numpy predict path (or None)."""
        self._ordinal_plan_ = None
        enc = self.preprocessor_
        ts = [(n, t, c) for n, t, c in enc.transformers_ if not (n == "remainder" and t == "drop")]
        if not ts or ts[0][0] != "encoder" or any(n not in ("encoder", "remainder") for n, _, _ in ts):
            return
        cols = [int(c) for c in ts[0][2]]
        oe = ts[0][1]
        if len(cols) and not hasattr(oe, "categories_"):
            return
        cats, nan_seen = [], []
        for c in (oe.categories_ if len(cols) else []):
            c = np.asarray(c)
            if c.dtype.kind not in "biuf":
                return
            c = c.astype(np.float64)
            nan_seen.append(bool(np.isnan(c).any()))
            cats.append(np.sort(c[~np.isnan(c)]))
        rem = [int(c) for c in ts[1][2]] if len(ts) > 1 else []
        miss = np.array([np.nan if n else -1.0 for n in nan_seen])
        # integer categories spanning < 4096 values: a [column][value - lo] table of category indices (-1: unseen)
        lut = None
        allc = np.concatenate(cats) if cats else np.zeros(0)
        if cats and len(allc) and np.all(allc == np.floor(allc)) and allc.max() - allc.min() < 4096:
            lo = float(allc.min())
            table = np.full((len(cats), int(allc.max() - lo) + 1), -1.0)
            for k, c in enumerate(cats):
                table[k, (c - lo).astype(np.intp)] = np.arange(len(c))
            lut = (lo, table)
        self._ordinal_plan_ = (cols, cats, miss, lut, rem)

    def predict(self, X, X_image: np.ndarray | None) -> np.ndarray:
        """Arg-max class labels (``classifier.py:504-515``)."""
        proba = self.predict_proba(X, X_image)
        return self.label_encoder_.inverse_transform(np.argmax(proba, axis=1))

    def predict_proba_device(self, X, image_test: np.ndarray | None) -> torch.Tensor:
        """Class probabilities ``[Q, n_classes]`` fp32 left on the GPU (no rounding)."""
        check_is_fitted(self)
        ex = self.executor_
        # the NaN / error check after the aggregation is enqueued (MMPFN_DEFER_STATUS=0: before it; A/B switch)
        defer = hasattr(ex, "check_status") and os.environ.get("MMPFN_DEFER_STATUS", "1") != "0"
        try:
            if image_test is not None and hasattr(ex, "launch_mixer_early"):
                # the mixer first: it does not need X, so the host's validation / encoding of X runs under it
                ex.launch_mixer_early(image_test, device=self.device_, autocast=self.use_autocast_)
            if X is not None:
                X = self._encode_predict_X(X)
            logits, perms = [], []
            if defer:
                ex._defer_status = True
            try:
                for out, config in ex.iter_outputs(X, image_test=image_test, device=self.device_,
                                                   autocast=self.use_autocast_):
                    assert out.ndim == 2
                    logits.append(out)
                    perms.append(config.class_permutation)
            finally:
                if defer:
                    ex._defer_status = False
            if any(p is None for p in perms) and not all(p is None for p in perms):
                raise ValueError("members must either all or none carry a class permutation")
            perm_arr = None if perms[0] is None else np.stack([np.asarray(p) for p in perms])
            weights = None
            if self.balance_probabilities:
                weights = (self.class_counts_ / self.class_counts_.sum()).astype(np.float32)
            eng = self.model_.engine(logits[0].device)
            return eng.aggregate(torch.stack(logits), perm_arr, self.n_classes_, float(self.softmax_temperature),
                                 bool(self.average_before_softmax), weights)
        finally:
            # whatever raised (X validation, the member loop, the aggregation): no early mixer tokens stay
            # referenced, and the deferred NaN / HIP check of a member loop that ran still runs (a NaN input's
            # ValueError takes precedence over the error in flight, as before)
            if hasattr(ex, "_early_tokens"):
                ex._early_tokens = None
            if defer:
                ex.check_status()

    def predict_proba(self, X, image_test: np.ndarray | None) -> np.ndarray:
        """``classifier.py:517-576``: ensemble-averaged class probabilities ``[Q, n_classes]``."""
        out = self.predict_proba_device(X, image_test).cpu().numpy()
        if self.interface_config_.USE_SKLEARN_16_DECIMAL_PRECISION:
            out = np.around(out, decimals=SKLEARN_16_DECIMAL_PRECISION)
            out = np.where(out < PROBABILITY_EPSILON_ROUND_ZERO, 0.0, out)
        return out / out.sum(axis=1, keepdims=True)
