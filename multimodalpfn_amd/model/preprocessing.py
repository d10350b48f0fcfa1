"""Per-member feature preprocessing steps (host side, numpy / scikit-learn).

Behavioural mirror of ``mmpfn/models/mmpfn/model/preprocessing.py``: every step
keeps the reference's class name, constructor arguments, random-stream usage
(each step seeds its own ``np.random.default_rng(static_seed)``) and output column
order, so a member's preprocessed table is identical to the reference's for the
same seed (pinned by ``tests/golden/api_*.npz``).  These run once per member at
``fit`` on the host, as in the reference; the forward that consumes their output
runs in the HIP engine.

Deliberate deviations (documented in DESIGN.md):

* KDI transforms need the third-party ``kditransform`` package, absent from this
  image.  The reference silently drops them there too (``preprocessing.py:40-45,
  105-125``); here asking for one raises a ``ValueError`` naming the package.
* ``SafePowerTransformer`` reverts every flagged column.  The reference's guard
  ``if self.revert_indices_ and (self.revert_indices_) > 0`` (``:184-193``)
  evaluates the truth value of a numpy array, which raises under numpy 2 unless
  exactly one column is flagged.
* The fingerprint column equals the reference's under ``PYTHONHASHSEED=0`` (the
  only setting in which the reference is reproducible), in every process.
"""

from __future__ import annotations

import warnings
from collections import UserList
from collections.abc import Sequence
from typing import Any, Literal, NamedTuple

import numpy as np
import scipy
from scipy.stats import shapiro
from sklearn.compose import ColumnTransformer, make_column_selector
from sklearn.decomposition import TruncatedSVD
from sklearn.impute import SimpleImputer
from sklearn.pipeline import FeatureUnion, Pipeline
from sklearn.preprocessing import (
    FunctionTransformer,
    MinMaxScaler,
    OneHotEncoder,
    OrdinalEncoder,
    PowerTransformer,
    QuantileTransformer,
    RobustScaler,
    StandardScaler,
)

from multimodalpfn_amd.model._siphash import siphash24_rows
from multimodalpfn_amd.utils import infer_random_state

# ----------------------------------------------------------------------------- transformers


class SafePowerTransformer(PowerTransformer):
    """Power transform that falls back to the input for columns it breaks (``:128-204``).

    A column is reverted when its transformed variance is not within
    ``variance_threshold`` of 1 or any transformed value exceeds
    ``large_value_threshold``; a Yeo-Johnson fit whose bracket search fails
    leaves the column untransformed.
    """

    def __init__(self, variance_threshold: float = 1e-3, large_value_threshold: float = 100, **kwargs: Any):
        super().__init__(**kwargs)
        self.variance_threshold = variance_threshold
        self.large_value_threshold = large_value_threshold
        self.revert_indices_ = None

    def _yeo_johnson_optimize(self, x: np.ndarray) -> float:
        try:
            with warnings.catch_warnings():
                warnings.filterwarnings("ignore", message=r"overflow encountered", category=RuntimeWarning)
                return super()._yeo_johnson_optimize(x)  # type: ignore[misc]
        except scipy.optimize._optimize.BracketError:
            return np.nan

    def _yeo_johnson_transform(self, x: np.ndarray, lmbda: float) -> np.ndarray:
        return x if np.isnan(lmbda) else super()._yeo_johnson_transform(x, lmbda)  # type: ignore[misc]

    def fit(self, X: np.ndarray, y: Any = None):
        super().fit(X, y)
        Xt = super().transform(X)
        bad_var = np.where(np.abs(np.nanvar(Xt, axis=0) - 1) > self.variance_threshold)[0]
        bad_big = np.nonzero(np.any(Xt > self.large_value_threshold, axis=0))[0]
        self.revert_indices_ = np.unique(np.concatenate([bad_var, bad_big]))
        return self

    def transform(self, X: np.ndarray) -> np.ndarray:
        Xt = super().transform(X)
        if self.revert_indices_ is not None and self.revert_indices_.size > 0:
            Xt[:, self.revert_indices_] = X[:, self.revert_indices_]
        return Xt


def skew(x: np.ndarray) -> float:
    """Pearson's second skewness, 3 (mean - median) / std (``:207-209``)."""
    return float(3 * (np.nanmean(x, 0) - np.nanmedian(x, 0)) / np.std(x, 0))


def _inf_to_nan_func(x: np.ndarray) -> np.ndarray:
    return np.nan_to_num(x, nan=np.nan, neginf=np.nan, posinf=np.nan)


def _exp_minus_1(x: np.ndarray) -> np.ndarray:
    return np.exp(x) - 1


def _identity(x):
    return x


def _finite_guard() -> list[tuple[str, Any]]:
    """inf -> nan, then mean-impute nan (the reference's ``_make_finite_transformer``)."""
    imputer = SimpleImputer(missing_values=np.nan, strategy="mean", keep_empty_features=True)
    imputer.inverse_transform = _identity  # type: ignore[method-assign]
    return [
        ("inf_to_nan", FunctionTransformer(func=_inf_to_nan_func, inverse_func=_identity, check_inverse=False)),
        ("nan_impute", imputer),
    ]


def make_standard_scaler_safe(_name_scaler_tuple: tuple[str, Any], *, no_name: bool = False) -> Pipeline:
    """Scaler sandwiched between finite guards (``:248-262``)."""
    pre = [(n + "_pre ", t) for n, t in _finite_guard()]
    post = [(n + "_post", t) for n, t in _finite_guard()]
    mid = ("placeholder", _name_scaler_tuple) if no_name else _name_scaler_tuple
    return Pipeline(steps=[*pre, mid, *post])


def make_box_cox_safe(input_transformer: Any) -> Pipeline:
    """MinMax into [0.1, 1] (clipped) so Box-Cox sees positive data (``:265-277``)."""
    return Pipeline(steps=[("mm", MinMaxScaler(feature_range=(0.1, 1), clip=True)), ("box_cox", input_transformer)])


def add_safe_standard_to_safe_power_without_standard(input_transformer: Any) -> Pipeline:
    """Power transform followed by a guarded StandardScaler (``:280-291``)."""
    return Pipeline(
        steps=[
            ("input_transformer", input_transformer),
            ("standard", make_standard_scaler_safe(("standard", StandardScaler()))),
        ]
    )


class NoneTransformer(FunctionTransformer):
    def __init__(self) -> None:
        super().__init__(func=_identity, inverse_func=_identity, check_inverse=False)


# ----------------------------------------------------------------------------- step protocol


class _TransformResult(NamedTuple):
    X: np.ndarray
    categorical_features: list[int]


class FeaturePreprocessingTransformerStep:
    """A transform that also tracks which output columns are categorical (``:300-368``)."""

    categorical_features_after_transform_: list[int]

    def fit_transform(self, X: np.ndarray, categorical_features: list[int]) -> _TransformResult:
        self.fit(X, categorical_features)
        return _TransformResult(self._transform(X, is_test=False), self.categorical_features_after_transform_)

    def _fit(self, X: np.ndarray, categorical_features: list[int]) -> list[int]:
        raise NotImplementedError

    def fit(self, X: np.ndarray, categorical_features: list[int]):
        self.categorical_features_after_transform_ = self._fit(X, categorical_features)
        assert self.categorical_features_after_transform_ is not None
        return self

    def _transform(self, X: np.ndarray, *, is_test: bool = False) -> np.ndarray:
        raise NotImplementedError

    def transform(self, X: np.ndarray) -> _TransformResult:
        return _TransformResult(self._transform(X, is_test=True), self.categorical_features_after_transform_)


class SequentialFeatureTransformer(UserList):
    """Chain of steps threading the categorical index list through (``:371-440``)."""

    def __init__(self, steps: Sequence[FeaturePreprocessingTransformerStep]):
        super().__init__(steps)
        self.steps = steps
        self.categorical_features_: list[int] | None = None

    def fit_transform(self, X: np.ndarray, categorical_features: list[int]) -> _TransformResult:
        for step in self.steps:
            X, categorical_features = step.fit_transform(X, categorical_features)
            assert isinstance(categorical_features, list), f"{step=} returned {categorical_features}"
        self.categorical_features_ = categorical_features
        return _TransformResult(X, categorical_features)

    def fit(self, X: np.ndarray, categorical_features: list[int]):
        assert len(self) > 0
        self.fit_transform(X, categorical_features)
        return self

    def transform(self, X: np.ndarray) -> _TransformResult:
        assert len(self) > 0
        assert self.categorical_features_ is not None, "fit before transform"
        cats: list[int] = []
        for step in self:
            X, cats = step.transform(X)
        assert cats == self.categorical_features_, (cats, self.categorical_features_)
        return _TransformResult(X, cats)


# ----------------------------------------------------------------------------- steps


class RemoveConstantFeaturesStep(FeaturePreprocessingTransformerStep):
    """Drop columns whose every training value equals the first row's (``:443-473``).

    A column of NaNs is kept (NaN != NaN), as in the reference.
    """

    def __init__(self) -> None:
        super().__init__()
        self.sel_: list[bool] | None = None

    def _fit(self, X: np.ndarray, categorical_features: list[int]) -> list[int]:
        sel = ((X[0:1, :] == X).mean(axis=0) < 1.0).tolist()
        if not any(sel):
            raise ValueError("All features are constant and would have been removed! Unable to predict using TabPFN.")
        self.sel_ = sel
        kept = np.where(sel)[0]
        return [new for new, old in enumerate(kept) if old in categorical_features]

    def _transform(self, X: np.ndarray, *, is_test: bool = False) -> np.ndarray:
        assert self.sel_ is not None, "You must call fit first"
        return X[:, self.sel_]


_CONSTANT = 10**12


def float_hash_rows(rows: np.ndarray) -> np.ndarray:
    """Row fingerprints in [0, 1) of a 2-D array (``:476-479``, vectorised over rows).

    The reference uses Python's ``hash`` of the row bytes, which is reproducible
    only under ``PYTHONHASHSEED=0``; this computes those ``PYTHONHASHSEED=0``
    values whatever the interpreter's seed (``_siphash.py``).
    """
    return np.mod(siphash24_rows(rows), _CONSTANT) / _CONSTANT


def float_hash_arr(arr: np.ndarray) -> float:
    return float(float_hash_rows(np.asarray(arr)[None, :])[0])


class AddFingerprintFeaturesStep(FeaturePreprocessingTransformerStep):
    """Append a per-row hash column (``:482-523``).

    Training rows resolve collisions by re-hashing ``row + k`` for k = 1, 2, ...
    (in row order); test rows keep the first hash and, as in the reference, add
    the salt twice.
    """

    def __init__(self, random_state: int | np.random.Generator | None = None):
        super().__init__()
        self.random_state = random_state

    def _fit(self, X: np.ndarray, categorical_features: list[int]) -> list[int]:
        _, rng = infer_random_state(self.random_state)
        self.rnd_salt_ = int(rng.integers(0, 2**16))
        return [*categorical_features]

    def _transform(self, X: np.ndarray, *, is_test: bool = False) -> np.ndarray:
        salted = X + self.rnd_salt_
        if is_test:
            fp = float_hash_rows(salted + self.rnd_salt_).astype(X.dtype)
        else:
            first = float_hash_rows(salted)
            fp = np.zeros(X.shape[0], dtype=X.dtype)
            seen: set[float] = set()
            for i in range(X.shape[0]):
                h = float(first[i])
                k = 0
                while h in seen:
                    k += 1
                    h = float_hash_arr(salted[i] + k)
                fp[i] = h
                seen.add(h)
        return np.concatenate([X, fp.reshape(-1, 1)], axis=1)


class ShuffleFeaturesStep(FeaturePreprocessingTransformerStep):
    """Column permutation of the member: rotate by ``shuffle_index`` or a seeded shuffle (``:526-571``)."""

    def __init__(
        self,
        shuffle_method: Literal["shuffle", "rotate"] | None = "rotate",
        shuffle_index: int = 0,
        random_state: int | np.random.Generator | None = None,
    ):
        super().__init__()
        self.random_state = random_state
        self.shuffle_method = shuffle_method
        self.shuffle_index = shuffle_index
        self.index_permutation_: list[int] | None = None

    def _fit(self, X: np.ndarray, categorical_features: list[int]) -> list[int]:
        _, rng = infer_random_state(self.random_state)
        n = X.shape[1]
        if self.shuffle_method == "rotate":
            perm = np.roll(np.arange(n), self.shuffle_index).tolist()
        elif self.shuffle_method == "shuffle":
            perm = rng.permutation(n).tolist()
        elif self.shuffle_method is None:
            perm = np.arange(n).tolist()
        else:
            raise ValueError(f"Unknown shuffle method {self.shuffle_method}")
        self.index_permutation_ = perm
        return [new for new, old in enumerate(perm) if old in categorical_features]

    def _transform(self, X: np.ndarray, *, is_test: bool = False) -> np.ndarray:
        assert self.index_permutation_ is not None, "You must call fit first"
        assert len(self.index_permutation_) == X.shape[1], "The number of features must not change after fit"
        return X[:, self.index_permutation_]


_KDI_NAMES = {"kdi", "kdi_uni", "kdi_random_alpha", "kdi_random_alpha_uni", "norm_and_kdi"}


class ReshapeFeatureDistributionsStep(FeaturePreprocessingTransformerStep):
    """Per-column distribution transform plus optional global transform (``:579-995``)."""

    @staticmethod
    def get_column_types(X: np.ndarray) -> list[str]:
        """Column type tags used by the adaptive transformer (``:582-606``)."""
        out = []
        for c in range(X.shape[1]):
            col = X[:, c]
            if np.unique(col).size < 10:
                out.append(f"ordinal_{c}")
            elif skew(col) > 1.1 and np.min(col) >= 0 and np.max(col) <= 1:
                out.append(f"skewed_pos_1_0_{c}")
            elif skew(col) > 1.1 and np.min(col) > 0:
                out.append(f"skewed_pos_{c}")
            elif skew(col) > 1.1:
                out.append(f"skewed_{c}")
            elif shapiro(X[0:3000, c]).statistic > 0.95:
                out.append(f"normal_{c}")
            else:
                out.append(f"other_{c}")
        return out

    @staticmethod
    def get_all_preprocessors(num_examples: int, random_state: int | None = None) -> dict[str, Any]:
        """Name -> column transformer table (``:684-779``), without the KDI family."""

        def quantile(dist: str, nq: int) -> QuantileTransformer:
            return QuantileTransformer(output_distribution=dist, n_quantiles=nq, random_state=random_state)

        coarse, mid = max(num_examples // 10, 2), max(num_examples // 5, 2)
        table: dict[str, Any] = {
            "power": add_safe_standard_to_safe_power_without_standard(PowerTransformer(standardize=False)),
            "safepower": add_safe_standard_to_safe_power_without_standard(SafePowerTransformer(standardize=False)),
            "power_box": make_box_cox_safe(
                add_safe_standard_to_safe_power_without_standard(PowerTransformer(standardize=False, method="box-cox"))
            ),
            "safepower_box": make_box_cox_safe(
                add_safe_standard_to_safe_power_without_standard(
                    SafePowerTransformer(standardize=False, method="box-cox")
                )
            ),
            "log": FunctionTransformer(func=np.log, inverse_func=np.exp, check_inverse=False),
            "1_plus_log": FunctionTransformer(func=np.log1p, inverse_func=_exp_minus_1, check_inverse=False),
            "exp": FunctionTransformer(func=np.exp, inverse_func=np.log, check_inverse=False),
            "quantile_uni_coarse": quantile("uniform", coarse),
            "quantile_norm_coarse": quantile("normal", coarse),
            "quantile_uni": quantile("uniform", mid),
            "quantile_norm": quantile("normal", mid),
            "quantile_uni_fine": quantile("uniform", num_examples),
            "quantile_norm_fine": quantile("normal", num_examples),
            "robust": RobustScaler(unit_variance=True),
            "none": FunctionTransformer(_identity),
        }
        table["adaptive"] = ColumnTransformer(
            [
                ("skewed_pos_1_0", FunctionTransformer(func=np.exp, inverse_func=np.log, check_inverse=False),
                 make_column_selector("skewed_pos_1_0*")),
                ("skewed_pos", make_box_cox_safe(add_safe_standard_to_safe_power_without_standard(
                    SafePowerTransformer(standardize=False, method="box-cox"))), make_column_selector("skewed_pos*")),
                ("skewed", add_safe_standard_to_safe_power_without_standard(
                    SafePowerTransformer(standardize=False, method="yeo-johnson")), make_column_selector("skewed*")),
                ("other", QuantileTransformer(output_distribution="normal", n_quantiles=num_examples // 10,
                                              random_state=random_state), make_column_selector("other*")),
                ("ordinal", NoneTransformer(), make_column_selector("ordinal*")),
                ("normal", NoneTransformer(), make_column_selector("normal*")),
            ],
            remainder="passthrough",
        )
        return table

    def get_all_global_transformers(self, num_examples: int, num_features: int, random_state: int | None = None):
        """``scaler`` and ``svd`` (identity + truncated SVD of the scaled table), ``:782-821``."""
        n_comp = max(1, min(num_examples // 10 + 1, num_features // 2))
        return {
            "scaler": make_standard_scaler_safe(("standard", StandardScaler())),
            "svd": FeatureUnion(
                [
                    ("passthrough", FunctionTransformer(func=_identity)),
                    (
                        "svd",
                        Pipeline(
                            steps=[
                                ("save_standard", make_standard_scaler_safe(("standard", StandardScaler(with_mean=False)))),
                                ("svd", TruncatedSVD(algorithm="arpack", n_components=n_comp, random_state=random_state)),
                            ]
                        ),
                    ),
                ]
            ),
        }

    def __init__(
        self,
        *,
        transform_name: str = "safepower",
        apply_to_categorical: bool = False,
        append_to_original: bool = False,
        subsample_features: float = -1,
        global_transformer_name: str | None = None,
        random_state: int | np.random.Generator | None = None,
    ):
        super().__init__()
        self.transform_name = transform_name
        self.apply_to_categorical = apply_to_categorical
        self.append_to_original = append_to_original
        self.random_state = random_state
        self.subsample_features = float(subsample_features)
        self.global_transformer_name = global_transformer_name
        self.transformer_: Any = None

    def _set_transformer_and_cat_ix(self, n_samples: int, n_features: int, categorical_features: list[int]):
        if "adaptive" in self.transform_name:
            raise NotImplementedError("Adaptive preprocessing raw removed.")
        if self.transform_name in _KDI_NAMES or self.transform_name.startswith("kdi_alpha_"):
            raise ValueError(
                f"preprocessor '{self.transform_name}' needs the 'kditransform' package, which is not installed"
            )
        static_seed, rng = infer_random_state(self.random_state)

        gname = self.global_transformer_name
        global_tf = None
        if gname is not None and gname != "None" and not (gname == "svd" and n_features < 2):
            global_tf = self.get_all_global_transformers(n_samples, n_features, random_state=static_seed)[gname]

        table = self.get_all_preprocessors(n_samples, random_state=static_seed)
        if self.subsample_features > 0:
            k = int(self.subsample_features * n_features) + 1
            self.subsampled_features_ = rng.choice(list(range(n_features)), k, replace=k > n_features)
            categorical_features = [
                new for new, old in enumerate(self.subsampled_features_) if old in categorical_features
            ]
            n_features = k
        else:
            self.subsampled_features_ = np.arange(n_features)

        everything = list(range(n_features))
        numeric = [i for i in everything if i not in categorical_features]
        parts: list[tuple[str, Any, list[int]]] = []
        if self.append_to_original:
            # the untouched table comes first, categorical columns stay where they were
            parts.append(("original", "passthrough", everything))
            targets = categorical_features + numeric if self.apply_to_categorical else numeric
            cat_ix = categorical_features
        elif self.apply_to_categorical:
            targets = categorical_features + numeric
            cat_ix = []
        else:
            parts.append(("cats", "passthrough", categorical_features))
            targets = numeric
            cat_ix = list(range(len(categorical_features)))

        if self.transform_name != "per_feature":
            parts.append(("feat_transform", table[self.transform_name], targets))
        else:
            choices = list(table.values())
            parts.extend((f"transformer_{i}", rng.choice(choices), [i]) for i in targets)

        tf: Any = ColumnTransformer(parts, remainder="drop", sparse_threshold=0.0)
        # a table that only passes columns through ("none" with no global transformer: run.py's members) is a
        # column selection; predict takes it straight (identical values, ~1/50 of the ColumnTransformer's per-call
        # cost, which sits in front of the first member's launch -- DESIGN 7)
        ident = self.transform_name == "none" and not global_tf
        self.select_cols_ = (self.subsampled_features_[np.concatenate([np.asarray(c, dtype=np.int64) for _, _, c in parts])]
                             if ident and parts else None)
        if global_tf:
            tf = Pipeline([("preprocess", tf), ("global_transformer", global_tf)])
        self.transformer_ = tf
        return tf, cat_ix

    def _fit(self, X: np.ndarray, categorical_features: list[int]) -> list[int]:
        tf, cat_ix = self._set_transformer_and_cat_ix(X.shape[0], X.shape[1], categorical_features)
        tf.fit(X[:, self.subsampled_features_])
        self.categorical_features_after_transform_ = cat_ix
        return cat_ix

    def fit_transform(self, X: np.ndarray, categorical_features: list[int]) -> _TransformResult:
        tf, cat_ix = self._set_transformer_and_cat_ix(X.shape[0], X.shape[1], categorical_features)
        Xt = tf.fit_transform(X[:, self.subsampled_features_])
        self.categorical_features_after_transform_ = cat_ix
        return _TransformResult(Xt, cat_ix)

    def _transform(self, X: np.ndarray, *, is_test: bool = False) -> np.ndarray:
        assert self.transformer_ is not None, "You must call fit first"
        sel = getattr(self, "select_cols_", None)
        if sel is not None and isinstance(X, np.ndarray) and X.ndim == 2:
            return X[:, sel]
        return self.transformer_.transform(X[:, self.subsampled_features_])


class EncodeCategoricalFeaturesStep(FeaturePreprocessingTransformerStep):
    """Re-encode categorical columns: ordinal (optionally shuffled) or one-hot (``:998-1200``)."""

    def __init__(self, categorical_transform_name: str = "ordinal", random_state=None):
        super().__init__()
        self.categorical_transform_name = categorical_transform_name
        self.random_state = random_state
        self.categorical_transformer_ = None

    @staticmethod
    def get_least_common_category_count(x_column: np.ndarray) -> int:
        if len(x_column) == 0:
            return 0
        return int(np.unique(x_column, return_counts=True)[1].min())

    def _get_transformer(self, X: np.ndarray, categorical_features: list[int]):
        name = self.categorical_transform_name
        if name.startswith("ordinal"):
            rest = name[len("ordinal"):]
            if rest.startswith("_common_categories"):
                rest = rest[len("_common_categories"):]
                categorical_features = [
                    i for i, col in enumerate(X.T)
                    if i in categorical_features and self.get_least_common_category_count(col) >= 10
                ]
            elif rest.startswith("_very_common_categories"):
                rest = rest[len("_very_common_categories"):]
                categorical_features = [
                    i for i, col in enumerate(X.T)
                    if i in categorical_features
                    and self.get_least_common_category_count(col) >= 10
                    and len(np.unique(col)) < (len(X) // 10)
                ]
            assert rest in ("_shuffled", ""), f"unknown categorical transform {name}"
            ct = ColumnTransformer(
                [("ordinal_encoder", OrdinalEncoder(handle_unknown="use_encoded_value", unknown_value=np.nan),
                  categorical_features)],
                remainder="passthrough",
            )
            return ct, categorical_features
        if name == "onehot":
            ct = ColumnTransformer(
                [("one_hot_encoder", OneHotEncoder(drop="if_binary", sparse_output=False, handle_unknown="ignore"),
                  categorical_features)],
                remainder="passthrough",
            )
            return ct, categorical_features
        if name in ("numeric", "none"):
            return None, categorical_features
        raise ValueError(f"Unknown categorical transform {name}")

    def _shuffle_maps(self, ct, categorical_features: list[int], rng, Xt: np.ndarray | None) -> None:
        self.random_mappings_ = {}
        if not self.categorical_transform_name.endswith("_shuffled"):
            return
        for c in categorical_features:
            perm = rng.permutation(len(ct.named_transformers_["ordinal_encoder"].categories_[c]))
            self.random_mappings_[c] = perm
            if Xt is not None:
                col = Xt[:, c]
                ok = ~np.isnan(col)
                col[ok] = perm[col[ok].astype(int)].astype(col.dtype)

    def _fit(self, X: np.ndarray, categorical_features: list[int]) -> list[int]:
        Xt, cats = self._fit_transform(X, categorical_features)
        return cats

    def _fit_transform(self, X: np.ndarray, categorical_features: list[int]):
        ct, categorical_features = self._get_transformer(X, categorical_features)
        if ct is None:
            self.categorical_transformer_ = None
            return X, categorical_features
        _, rng = infer_random_state(self.random_state)
        if self.categorical_transform_name.startswith("ordinal"):
            Xt = ct.fit_transform(X)
            categorical_features = list(range(len(categorical_features)))
            self._shuffle_maps(ct, categorical_features, rng, Xt)
        elif self.categorical_transform_name == "onehot":
            Xt = ct.fit_transform(X)
            if Xt.size >= 1_000_000:
                ct, Xt = None, X
            else:
                categorical_features = list(range(Xt.shape[1]))[ct.output_indices_["one_hot_encoder"]]
        else:
            raise ValueError(f"Unknown categorical transform {self.categorical_transform_name}")
        self.categorical_transformer_ = ct
        return Xt, categorical_features

    def fit_transform(self, X: np.ndarray, categorical_features: list[int]) -> _TransformResult:
        Xt, cats = self._fit_transform(X, categorical_features)
        self.categorical_features_after_transform_ = cats
        return _TransformResult(Xt, cats)

    def _transform(self, X: np.ndarray, *, is_test: bool = False) -> np.ndarray:
        if self.categorical_transformer_ is None:
            return X
        Xt = self.categorical_transformer_.transform(X)
        if self.categorical_transform_name.endswith("_shuffled"):
            for c, perm in self.random_mappings_.items():
                col = Xt[:, c]
                ok = ~np.isnan(col)
                col[ok] = perm[col[ok].astype(int)].astype(col.dtype)
        return Xt


class NanHandlingPolynomialFeaturesStep(FeaturePreprocessingTransformerStep):
    """Append products of random feature pairs of the scaled table (``:1203-1278``)."""

    def __init__(self, *, max_features: int | None, random_state=None):
        super().__init__()
        self.max_poly_features = max_features
        self.random_state = random_state
        self.poly_factor_1_idx: np.ndarray | None = None
        self.poly_factor_2_idx: np.ndarray | None = None
        self.standardizer = StandardScaler(with_mean=False)

    def _fit(self, X: np.ndarray, categorical_features: list[int]) -> list[int]:
        assert X.ndim == 2
        _, rng = infer_random_state(self.random_state)
        if X.shape[0] == 0 or X.shape[1] == 0:
            return [*categorical_features]
        nf = X.shape[1]
        n_poly = nf * (nf - 1) // 2 + nf
        n_poly = min(self.max_poly_features, n_poly) if self.max_poly_features else n_poly
        X = self.standardizer.fit_transform(X)
        first = rng.choice(np.arange(0, nf), size=n_poly, replace=True)
        second = np.ones_like(first) * -1
        for i in range(len(first)):
            while second[i] == -1:
                a = first[i]
                taken = second[first == a]
                free = set(range(a, nf)) - set(taken.tolist())
                if not free:
                    first[i] = rng.choice(np.arange(0, nf), size=1)[0]
                    continue
                second[i] = rng.choice(list(free), size=1)[0]
        self.poly_factor_1_idx, self.poly_factor_2_idx = first, second
        return categorical_features

    def _transform(self, X: np.ndarray, *, is_test: bool = False) -> np.ndarray:
        assert X.ndim == 2
        if X.shape[0] == 0 or X.shape[1] == 0:
            return X
        X = self.standardizer.transform(X)
        return np.hstack((X, X[:, self.poly_factor_1_idx] * X[:, self.poly_factor_2_idx]))
