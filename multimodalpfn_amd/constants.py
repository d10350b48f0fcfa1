"""Interface constants of the classifier (mirror of ``mmpfn/models/mmpfn/constants.py``).

``ModelInterfaceConfig`` keeps the reference's field names, defaults and
``from_user_input`` semantics (``constants.py:35-211``) so user code such as
``run.py:113-116``::

    ModelInterfaceConfig(FINGERPRINT_FEATURE=False,
                         PREPROCESS_TRANSFORMS=[PreprocessorConfig(name="none")])

works unchanged.
"""

from __future__ import annotations

from copy import deepcopy
from dataclasses import dataclass
from typing import TYPE_CHECKING, Any, Literal

import numpy as np

if TYPE_CHECKING:
    from multimodalpfn_amd.preprocessing import PreprocessorConfig

XType = Any
YType = Any


@dataclass
class ModelInterfaceConfig:
    """Expert knobs of the interface; field meanings as in ``constants.py:35-196``."""

    MAX_UNIQUE_FOR_CATEGORICAL_FEATURES: int = 30
    MIN_UNIQUE_FOR_NUMERICAL_FEATURES: int = 4
    MIN_NUMBER_SAMPLES_FOR_CATEGORICAL_INFERENCE: int = 100
    OUTLIER_REMOVAL_STD: float | None | Literal["auto"] = "auto"
    FEATURE_SHIFT_METHOD: Literal["shuffle", "rotate"] | None = "shuffle"
    CLASS_SHIFT_METHOD: Literal["rotate", "shuffle"] | None = "shuffle"
    FINGERPRINT_FEATURE: bool = True
    POLYNOMIAL_FEATURES: Literal["no", "all"] | int = "no"
    SUBSAMPLE_SAMPLES: int | float | None = None
    PREPROCESS_TRANSFORMS: list[PreprocessorConfig] | None = None
    REGRESSION_Y_PREPROCESS_TRANSFORMS: tuple[Literal["safepower", "power", "quantile_norm", None], ...] = (
        None,
        "safepower",
    )
    USE_SKLEARN_16_DECIMAL_PRECISION: bool = False
    MAX_NUMBER_OF_CLASSES: int = 10
    MAX_NUMBER_OF_FEATURES: int = 500
    MAX_NUMBER_OF_SAMPLES: int = 10_000
    FIX_NAN_BORDERS_AFTER_TARGET_TRANSFORM: bool = True
    _REGRESSION_DEFAULT_OUTLIER_REMOVAL_STD: None = None
    _CLASSIFICATION_DEFAULT_OUTLIER_REMOVAL_STD: float = 12.0

    @staticmethod
    def from_user_input(*, inference_config: dict | ModelInterfaceConfig | None) -> ModelInterfaceConfig:
        """None -> defaults; a config -> deep copy; a dict -> defaults overridden key by key."""
        if inference_config is None:
            return ModelInterfaceConfig()
        if isinstance(inference_config, ModelInterfaceConfig):
            return deepcopy(inference_config)
        if isinstance(inference_config, dict):
            cfg = ModelInterfaceConfig()
            for key, value in inference_config.items():
                if not hasattr(cfg, key):
                    raise ValueError(f"Unknown kwarg passed to model construction: {key}")
                setattr(cfg, key, value)
            return cfg
        raise ValueError(f"Unknown {inference_config=} passed to model.")


SKLEARN_16_DECIMAL_PRECISION = 16
PROBABILITY_EPSILON_ROUND_ZERO = 1e-3
AUTOCAST_DTYPE_BYTE_SIZE = 2
DEFAULT_DTYPE_BYTE_SIZE = 4
DEFAULT_NUMPY_PREPROCESSING_DTYPE = np.float64
ENSEMBLE_CONFIGURATION_MAX_STEP = 2
MAXIMUM_FEATURE_SHIFT = 1_000
CLASS_SHUFFLE_OVERESTIMATE_FACTOR = 3
