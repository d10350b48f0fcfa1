"""Inference engines of the classifier: how ensemble members reach the HIP forward.

Mirror of ``mmpfn/models/mmpfn/inference.py``.  ``InferenceEngineCachePreprocessing``
(``fit_mode="fit_preprocessors"``, the default and the path of ``run.py``) fits
each member's preprocessing at ``fit`` and at ``predict`` transforms the test
rows and runs one forward per member (``inference.py:217-351``);
``InferenceEngineOnDemand`` (``"low_memory"``) re-fits the preprocessing at every
predict (``:73-213``); ``InferenceEngineCacheKV`` (``"fit_with_cache"``) runs the train rows
through the model once at ``fit`` and keeps each member's train-KV cache on the device, so a
predict forwards the test rows only (``:352-512``; unlike the reference it also serves images).

MI355X-specific: the modality projection (MGM / CAP / MoE) depends only on the
image rows, which every member shares, so it runs once per predict instead of
once per member (the reference recomputes it inside every forward); members are
queued back-to-back on the engine's stream with one NaN-status check at the end;
with ``torch.distributed`` initialised and more than one rank, members are split
across ranks (longest-processing-time) and the logits all-gathered (RCCL).
"""

from __future__ import annotations


from collections.abc import Iterator, Sequence
from dataclasses import dataclass, field
from typing import Any, Literal

import numpy as np
import torch

from multimodalpfn_amd import _lib
from multimodalpfn_amd.preprocessing import fit_preprocessing
from multimodalpfn_amd.utils import infer_random_state




def _precision(model, device: torch.device, autocast: bool, forced: torch.dtype | None) -> int:
    if forced is not None:
        return _lib.precision_of_dtype(forced)
    return _lib.autocast_precision() if (autocast and device.type == "cuda") else _lib.f32_precision()


def _h2d(a, device: torch.device) -> torch.Tensor:
    """fp32 host array -> device on the current stream, through pinned memory and without a host wait (a
    pageable copy is host-synchronous, so the launches that follow it would trail the GPU)."""
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    if device.type == "cuda":
        return t.pin_memory().to(device, non_blocking=True)
    return t.to(device)


def _mixer_tokens(model, eng, image_train, image_test, prec: int, cache: dict | None = None):
    """Shared modality tokens of all members (``transformer.py:560-600``), or None.

    The projection heads are row-wise (MGM: per-row LN + gated MLP; CAP: each row's queries
    attend that row's MGM tokens; MoE: per-row gate and experts), so the train rows' tokens do
    not depend on the test rows: with ``cache`` they are computed at the first predict and kept
    on the device, and every predict projects only its test rows."""
    if image_train is None or image_test is None or model.mixer_type not in ("MGM", "MGM+CAP", "MoE"):
        return None
    # the test image rows (1.4 MB at PAD-UFES size) through pinned memory, asynchronously on the stream
    # the mixer runs on (a pageable copy is staged by the runtime in host-synchronous chunks)
    img = torch.from_numpy(np.ascontiguousarray(image_test, dtype=np.float32))
    if eng.device.type == "cuda":
        img = img.pin_memory().to(eng.device, non_blocking=True)
    test = eng.mixer_tokens(img, prec)
    key = ("train_tokens", str(eng.device), prec)
    train = None if cache is None else cache.get(key)
    if train is None:
        train = eng.mixer_tokens(torch.from_numpy(np.asarray(image_train, dtype=np.float32)), prec)
        if cache is not None:
            cache[key] = train
    return torch.cat([train, test], 0)


def _n_mixer_tokens(model, image) -> int:
    """Image tokens the mixer appends per row (C of SURVEY.md 8a: cap_heads for MGM+CAP, mgm_heads * n_mod
    for MGM, the expert count for MoE)."""
    if image is None or model.mixer_type not in ("MGM", "MGM+CAP", "MoE"):
        return 0
    n_mod = np.shape(image)[1] if np.ndim(image) == 3 else 1
    cfg = model.cfg
    return {"MGM": cfg.mgm_heads * n_mod, "MGM+CAP": cfg.cap_heads, "MoE": cfg.mgm_heads}[model.mixer_type]


@dataclass
class _Member:
    config: Any
    preprocessor: Any
    X_train: np.ndarray | None
    y_train: np.ndarray
    cat_ix: list[int] | None


@dataclass
class InferenceEngine:
    """Base: ``iter_outputs`` yields ``(logits [Q, n_out], member config)`` per member."""

    save_peak_mem: bool | Literal["auto"] | float | int
    dtype_byte_size: int
    # device copies of what every predict re-uses: the train rows' modality tokens and each
    # member's preprocessed train table (the reference re-uploads both per member and predict)
    _device_cache: dict = field(default_factory=dict, repr=False)

    _early_tokens: tuple | None = field(default=None, repr=False)
    _pending_status: Any = field(default=None, repr=False)
    _defer_status: bool = field(default=False, repr=False)  # set by a caller that calls check_status() itself
    _early_mixer = False  # executors whose predict runs _run_members with self.model / self.image_train

    def iter_outputs(self, X, image_test, *, device: torch.device, autocast: bool) -> Iterator[tuple]:
        raise NotImplementedError

    def launch_mixer_early(self, image_test, *, device: torch.device, autocast: bool) -> None:
        """Enqueue the test rows' modality tokens before the caller validates and encodes X: the mixer is the
        first GPU work of a predict and does not depend on X, so the GPU starts ~0.3 ms earlier (the host's X
        path then runs under it).  ``_run_members`` takes the tokens if it is called with this same image array
        and precision; anything else (no image, a mixer-less model, an image that is not a [Q, n_mod, D] /
        [Q, D] float array of the model's width) is left to the regular path and its errors."""
        self._early_tokens = None
        model, image_train = getattr(self, "model", None), getattr(self, "image_train", None)
        if (not self._early_mixer or model is None or image_train is None or device.type != "cuda"
                or model.mixer_type not in ("MGM", "MGM+CAP", "MoE") or not isinstance(image_test, np.ndarray)
                or image_test.ndim not in (2, 3) or image_test.dtype.kind not in "fiu"
                or image_test.shape[-1] != model.cfg.mixer_in_dim):
            return
        eng = model.engine(device)
        prec = _precision(model, eng.device, autocast, getattr(self, "force_inference_dtype", None))
        cache = self._fresh_cache(model, eng) if self._cacheable else None
        self._early_tokens = (image_test, prec, _mixer_tokens(model, eng, image_train, image_test, prec, cache))

    def _fresh_cache(self, model, eng) -> dict:
        """The device cache, emptied if it was made with other weights (load_state_dict / invalidate_engine
        after fit) or by another engine."""
        cache = self._device_cache
        tag = (model._weights_version, eng.serial)
        if cache.get("_tag") != tag:
            cache.clear()
            cache["_tag"] = tag
        return cache

    # -- shared member loop -------------------------------------------------------
    def _run_members(self, members: Sequence[_Member], X, image_train, image_test, *, device, autocast,
                     forced_dtype, model) -> list[torch.Tensor]:
        from multimodalpfn_amd.parallel import member_shard

        eng = model.engine(model._device() if device.type != "cuda" else device)
        prec = _precision(model, eng.device, autocast, forced_dtype)
        mine, gather = member_shard(len(members), [self._member_cost(m, X, image_test, model) for m in members],
                                    keys=[self._member_key(m) for m in members], unit=eng.batch)
        cache = self._fresh_cache(model, eng) if self._cacheable else None
        early, self._early_tokens = self._early_tokens, None
        if early is not None and early[0] is image_test and early[1] == prec and mine:
            tokens = early[2]  # launch_mixer_early's, already queued on this stream
        else:
            tokens = _mixer_tokens(model, eng, image_train, image_test, prec, cache) if mine else None
        # launch order: geometry groups (members the engine stacks into one batched forward) narrowest
        # first, so the GPU starts after the cheapest transforms and the wider members' transforms run
        # under the earlier units' forwards.  Each member is transformed in the main thread when its unit
        # is assembled: a worker thread (tried with one and with four) holds the GIL for sklearn's per-call
        # overhead exactly while the main thread enqueues the previous unit's kernels, and measured 2-3 ms
        # slower per predict at config C (19.1 / 17.5 vs 16.1 / 15.6 ms; default preprocessing 19.7 / 20.1 vs
        # 17.8 / 17.4 ms, profiles/r03/ab/api_transform_inline.txt)
        order = self._launch_order(members, mine)

        def items():  # a generator: forward_many launches each unit as soon as its members are ready
            for i in order:
                m = members[i]
                x_full = None
                if m.X_train is not None:
                    X_test = _h2d(m.preprocessor.transform(X).X, eng.device)
                    key = ("X_train", i, str(eng.device))
                    xtr = None if cache is None else cache.get(key)
                    if xtr is None:
                        xtr = _h2d(m.X_train, eng.device)
                        if cache is not None:
                            cache[key] = xtr
                    x_full = torch.cat([xtr, X_test], 0)
                yield x_full, tokens, np.asarray(m.y_train, np.float32)

        outs: dict[int, torch.Tensor] = dict(zip(order, eng.forward_many(items(), prec)))
        if mine:
            if self._defer_status:
                # the caller enqueues its own device work (the aggregation) first and then calls check_status():
                # the GPU does not idle while the host waits here
                self._pending_status = eng
            else:
                eng.status()  # NaN / HIP errors of every queued member (transformer.py:727-731,790-796)
        Q = len(X) if X is not None else len(image_test)
        return gather(outs, eng.device, Q, model.cfg.n_out)

    def check_status(self) -> None:
        """The deferred ``status`` of the last member loop (``_defer_status``): waits for its streams and raises
        ``ValueError`` on NaN input (transformer.py:727-731,790-796)."""
        eng, self._pending_status = self._pending_status, None
        if eng is not None:
            eng.status()

    _cacheable = True  # the members' train tables and train images are fixed after fit

    @classmethod
    def _launch_order(cls, members: Sequence[_Member], mine: list[int]) -> list[int]:
        """``mine`` grouped by batching key, groups by ascending width (host transform cost), index order
        inside a group."""
        groups: dict = {}
        for i in mine:
            groups.setdefault(cls._member_key(members[i]), []).append(i)

        def width(g):
            x = members[g[0]].X_train
            return (0 if x is None else np.asarray(x).shape[1], g[0])

        return [i for g in sorted(groups.values(), key=width) for i in g]

    @staticmethod
    def _member_cost(m: _Member, X, image_test, model) -> float:
        from multimodalpfn_amd.parallel import member_cost

        n_tr = len(m.y_train)
        n_te = len(X) if X is not None else len(image_test)
        fpg = model.features_per_group
        F = 0 if m.X_train is None else np.asarray(m.X_train).shape[1]
        C = _n_mixer_tokens(model, image_test)
        return member_cost((F + fpg - 1) // fpg + C + 1, n_tr + n_te, n_tr, model.cfg.emsize, model.cfg.nhid)

    @staticmethod
    def _member_key(m: _Member):
        """Members the engine can stack into one batched forward share this key (same F and N)."""
        return (None if m.X_train is None else np.asarray(m.X_train).shape[1], len(m.y_train))


@dataclass
class InferenceEngineCachePreprocessing(InferenceEngine):
    """Preprocessing fitted at ``fit``; one forward per member at predict (``inference.py:217-351``)."""

    _early_mixer = True

    X_trains: Sequence[np.ndarray | None] = ()
    y_trains: Sequence[np.ndarray] = ()
    image_train: np.ndarray | None = None
    cat_ixs: Sequence[list[int] | None] = ()
    ensemble_configs: Sequence[Any] = ()
    preprocessors: Sequence[Any] = ()
    model: Any = None
    force_inference_dtype: torch.dtype | None = None

    @classmethod
    def prepare(cls, X_train, y_train, image_train, *, cat_ix, model, ensemble_configs, n_workers, rng,
                dtype_byte_size, force_inference_dtype, save_peak_mem) -> InferenceEngineCachePreprocessing:
        itr = fit_preprocessing(configs=ensemble_configs, X_train=X_train, y_train=y_train, random_state=rng,
                                cat_ix=cat_ix, n_workers=n_workers, parallel_mode="block")
        configs, preprocessors, X_trains, y_trains, cat_ixs = list(zip(*itr))
        return cls(save_peak_mem=save_peak_mem, dtype_byte_size=dtype_byte_size, X_trains=X_trains,
                   y_trains=y_trains, image_train=image_train, cat_ixs=cat_ixs, ensemble_configs=configs,
                   preprocessors=preprocessors, model=model, force_inference_dtype=force_inference_dtype)

    def members(self) -> list[_Member]:
        return [_Member(c, p, xt, yt, ci) for c, p, xt, yt, ci in
                zip(self.ensemble_configs, self.preprocessors, self.X_trains, self.y_trains, self.cat_ixs)]

    def iter_outputs(self, X, image_test, *, device: torch.device, autocast: bool) -> Iterator[tuple]:
        self.model = self.model.to(device)
        outs = self._run_members(self.members(), X, self.image_train, image_test, device=device,
                                 autocast=autocast, forced_dtype=self.force_inference_dtype, model=self.model)
        for out, cfg in zip(outs, self.ensemble_configs):
            yield out, cfg


@dataclass
class InferenceEngineOnDemand(InferenceEngine):
    """Nothing cached: members' preprocessing re-fitted at every predict (``inference.py:73-213``)."""

    _cacheable = False
    _early_mixer = True

    X_train: np.ndarray | None = None
    y_train: np.ndarray | None = None
    image_train: np.ndarray | None = None
    ensemble_configs: Sequence[Any] = ()
    cat_ix: list[int] = field(default_factory=list)
    static_seed: int = 0
    n_workers: int = 1
    model: Any = None
    force_inference_dtype: torch.dtype | None = None

    @classmethod
    def prepare(cls, X_train, y_train, image_train=None, *, cat_ix, model, ensemble_configs, rng, n_workers,
                dtype_byte_size, force_inference_dtype, save_peak_mem) -> InferenceEngineOnDemand:
        static_seed = rng.integers(0, 2**31)  # fixed once so every predict re-fits identically
        return cls(save_peak_mem=save_peak_mem, dtype_byte_size=dtype_byte_size, X_train=X_train, y_train=y_train,
                   image_train=image_train, ensemble_configs=ensemble_configs, cat_ix=cat_ix,
                   static_seed=static_seed, n_workers=n_workers, model=model,
                   force_inference_dtype=force_inference_dtype)

    def iter_outputs(self, X, image_test, *, device: torch.device, autocast: bool) -> Iterator[tuple]:
        _, rng = infer_random_state(self.static_seed)
        itr = fit_preprocessing(configs=self.ensemble_configs, X_train=self.X_train, y_train=self.y_train,
                                random_state=rng, cat_ix=self.cat_ix, n_workers=self.n_workers,
                                parallel_mode="in-order")
        members = [_Member(c, p, xt, yt, ci) for c, p, xt, yt, ci in itr]
        self.model = self.model.to(device)
        outs = self._run_members(members, X, self.image_train, image_test, device=device, autocast=autocast,
                                 forced_dtype=self.force_inference_dtype, model=self.model)
        for out, m in zip(outs, members):
            yield out, m.config


@dataclass
class InferenceEngineCacheKV(InferenceEngine):
    """``fit_mode="fit_with_cache"`` (``inference.py:352-512``): at ``fit`` every member's train rows
    go through the model once and the engine keeps, on the device, head 0's K/V of the train rows
    per layer plus the encoders' train statistics; a predict then forwards only the test rows
    (``mmpfn_cache_build`` / ``mmpfn_cache_predict``).  The reference serves tabular inputs only
    here (its prepare passes no image, ``:425-436``); images are served: the modality tokens of
    the train rows are computed at fit and those of the test rows at predict (the mixers are
    row-wise).  Precision is fixed at fit.  Members are sharded over ranks like the other engines.
    """

    caches: dict = field(default_factory=dict)
    ensemble_configs: Sequence[Any] = ()
    preprocessors: Sequence[Any] = ()
    n_members: int = 0
    model: Any = None
    precision: int = _lib.PREC_F32
    mine: list = field(default_factory=list)
    gather: Any = None

    @classmethod
    def prepare(cls, X_train, y_train, image_train, *, cat_ix, model, ensemble_configs, n_workers, rng,
                dtype_byte_size, force_inference_dtype, save_peak_mem, device, autocast) -> InferenceEngineCacheKV:
        from multimodalpfn_amd.parallel import member_cost, member_shard

        itr = fit_preprocessing(configs=ensemble_configs, X_train=X_train, y_train=y_train, random_state=rng,
                                cat_ix=cat_ix, n_workers=n_workers, parallel_mode="block")
        configs, preprocessors, X_trains, y_trains, _ = list(zip(*itr))
        model = model.to(device)
        eng = model.engine(device)
        prec = _precision(model, eng.device, autocast, force_inference_dtype)
        # the flop model of the other engines (parallel.member_cost) on each member's cache build:
        # T tokens of N train rows against N keys (ragged widths make T differ between members)
        C = _n_mixer_tokens(model, image_train)
        fpg = model.features_per_group
        costs = []
        for xt, yt in zip(X_trains, y_trains):
            F = 0 if xt is None else np.asarray(xt).shape[1]
            costs.append(member_cost((F + fpg - 1) // fpg + C + 1, len(yt), len(yt), model.cfg.emsize,
                                     model.cfg.nhid))
        mine, gather = member_shard(len(configs), costs)
        tokens = None
        if image_train is not None and model.mixer_type in ("MGM", "MGM+CAP", "MoE") and mine:
            tokens = eng.mixer_tokens(torch.from_numpy(np.asarray(image_train, np.float32)), prec)
        caches = {}
        for i in mine:
            xt = None if X_trains[i] is None else torch.from_numpy(np.asarray(X_trains[i], np.float32))
            caches[i] = eng.cache_build(xt, tokens, np.asarray(y_trains[i], np.float32), prec)
        if mine:
            eng.status()  # NaN in the encoded train rows (transformer.py:727-731,790-796)
        return cls(save_peak_mem=save_peak_mem, dtype_byte_size=dtype_byte_size, caches=caches,
                   ensemble_configs=configs, preprocessors=preprocessors, n_members=len(configs), model=model,
                   precision=prec, mine=list(mine), gather=gather)

    def iter_outputs(self, X, image_test, *, device: torch.device, autocast: bool) -> Iterator[tuple]:
        eng = self.model.engine(self.model._device() if device.type != "cuda" else device)
        tokens = None
        if image_test is not None and self.model.mixer_type in ("MGM", "MGM+CAP", "MoE") and self.mine:
            tokens = eng.mixer_tokens(torch.from_numpy(np.asarray(image_test, np.float32)), self.precision)
        xts = []
        for i in self.mine:
            xt = None
            if X is not None and self.caches[i].F > 0:
                xt = torch.from_numpy(np.asarray(self.preprocessors[i].transform(X).X, np.float32))
            xts.append(xt)
        outs = dict(zip(self.mine, eng.cache_predict_many([self.caches[i] for i in self.mine], xts, tokens)))
        if self.mine:
            eng.status()
        Q = len(X) if X is not None else len(image_test)
        for out, cfg in zip(self.gather(outs, eng.device, Q, self.model.cfg.n_out), self.ensemble_configs):
            yield out, cfg

