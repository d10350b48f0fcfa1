"""Host-side handle on one HIP engine context (one per GPU / rank).

Owns the packed device weights (uploaded once through the checkpoint ABI) and
drives the C-ABI entry points on the caller's current HIP stream.  All compute
of the forward runs in ``libmmpfn_hip.so``; this module only moves pointers,
shapes and the few host-side constants the reference also computes on the host:

* the subspace positional-embedding draw ``torch.randn`` from the model's CPU
  generator (``transformer.py:421-424,925-931``) -- bit-exact with the reference's CPU
  forward (see ``pos_rand`` for the GPU stream);
* the sorted unique train labels of the target encoder (``encoders.py:956-958``).
"""

from __future__ import annotations

import ctypes
import itertools
import os

import numpy as np
import torch

from multimodalpfn_amd import _lib
from multimodalpfn_amd.model.spec import ModelConfig, encoder_linear_name


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def model_desc(cfg: ModelConfig) -> _lib.ModelDesc:
    d = _lib.ModelDesc()
    d.emsize = cfg.emsize
    d.nhead = cfg.nhead
    d.nlayers = cfg.nlayers
    d.nhid = cfg.nhid
    d.features_per_group = cfg.features_per_group
    d.encoder_features = cfg.encoder_features
    d.n_out = cfg.n_out
    d.mixer_type = _lib.MIXER_CODES[cfg.mixer_type]
    d.mgm_heads = cfg.mgm_heads
    d.cap_heads = cfg.cap_heads
    d.two_sets_of_queries = int(cfg.two_sets_of_queries)
    d.remove_duplicate_features = int(cfg.remove_duplicate_features)
    d.ln_eps = cfg.ln_eps
    d.outlier_sigma = float(cfg.remove_outliers_sigma) if cfg.remove_outliers_sigma else 0.0
    return d


POS_RNG = os.environ.get("MMPFN_POS_RNG", "cpu")  # "cpu" (default) or "device"


def pos_rand(cfg: ModelConfig, n_tokens: int, device: torch.device | None = None) -> torch.Tensor:
    """``randn((n_tokens, E//4))`` from a fresh generator seeded like ``_init_rnd`` (transformer.py:421-424).

    The reference draws on the generator of the device its input lives on (:887-892): on a CPU
    forward that is the CPU Mersenne-Twister stream, which is what the goldens pin, and the engine
    reproduces it bit for bit.  On a GPU the reference draws from that GPU's Philox generator in the
    autocast dtype of its embedded input; that stream depends on the device's grid geometry and dtype,
    so it is not a fixed target.  ``MMPFN_POS_RNG=device`` draws from a generator on ``device`` (fp32)
    instead -- the reference's GPU behaviour in kind, parity unpinned.
    """
    gdev = device if (POS_RNG == "device" and device is not None) else torch.device("cpu")
    gen = torch.Generator(device=gdev)
    if cfg.model_seed:  # `if self.seed:` (transformer.py:423)
        gen.manual_seed(cfg.model_seed)
    return torch.randn((n_tokens, cfg.emsize // 4), generator=gen, dtype=torch.float32, device=gdev)


def target_uniques(y_train: np.ndarray) -> np.ndarray:
    """Sorted unique train targets after the y NaN fill (encoders.py:461-493,954-958)."""
    y = np.asarray(y_train, dtype=np.float32)
    if np.isnan(y).any():
        y = np.where(np.isnan(y), np.float32(np.nanmean(y)), y)
    return np.unique(y).astype(np.float32)


# Lane streams are process-wide (one per device and lane index), shared by every engine: each HIP stream is bound to
# one of the device's few hardware queues (GPU_MAX_HW_QUEUES), and two lanes that land on the same queue run one after
# the other.  Which pool streams share a queue is not under the caller's control -- per-engine streams gave every second
# MMPFNClassifier of a process 15.0-15.9 instead of 13.6-13.8 ms per predict at config C -- so the first pair, made
# together at the first lanes' use, serves all engines (13.5-13.8 ms for all four classifiers of the same test;
# profiles/r06/api_lane_streams.txt; CU-masked streams 17-24 ms, a high-priority second lane 14.0-14.8 ms).
_LANE_STREAMS: dict = {}


def _lane_stream(device: torch.device, k: int) -> torch.cuda.Stream:
    key = (str(device), k)
    st = _LANE_STREAMS.get(key)
    if st is None:
        st = _LANE_STREAMS[key] = torch.cuda.Stream(device)
    return st


DEFAULT_LANES = int(os.environ.get("MMPFN_LANES", "2"))  # concurrent member lanes of forward_many
DEFAULT_BATCH = int(os.environ.get("MMPFN_BATCH", "1"))  # members per batched forward of forward_many (1: DESIGN 7)
_DEBUG_SYNC = os.environ.get("MMPFN_DEBUG_SYNC") == "1"  # diagnostics: serialise forward_many's units
_DEBUG_KEEP = os.environ.get("MMPFN_DEBUG_KEEP") == "1"  # diagnostics: keep every prepared input alive
_KEEP: list = []
_SERIAL = itertools.count(1)  # engine serial numbers: cache tags that a freed engine's id() could alias


class HipEngine:
    """One ``mmpfn_ctx`` bound to a CUDA(HIP) device."""

    def __init__(self, cfg: ModelConfig, state_dict: dict, device: torch.device):
        if not torch.cuda.is_available():
            raise RuntimeError("the MMPFN HIP engine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _lib.load_library()
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError(f"HipEngine needs a cuda device, got {self.device}")
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        self.ctx = self.lib.mmpfn_create(idx, ctypes.c_void_p(self._stream()))
        if not self.ctx:
            raise _lib.EngineError(f"mmpfn_create failed on device {idx}")
        self.desc = model_desc(cfg)
        self._check(self.lib.mmpfn_set_model(self.ctx, ctypes.byref(self.desc)), "mmpfn_set_model")
        names = set()
        for name, t in state_dict.items():
            if isinstance(t, torch.Tensor):
                a = t.detach().to("cpu", torch.float32).contiguous().numpy()
            else:
                a = np.ascontiguousarray(t, dtype=np.float32)
            self._check(
                self.lib.mmpfn_load_weight(self.ctx, name.encode(), a.ctypes.data_as(ctypes.c_void_p), a.size),
                f"mmpfn_load_weight({name})",
            )
            names.add(name)
        if encoder_linear_name(cfg) not in names:
            raise _lib.EngineError(f"state_dict lacks {encoder_linear_name(cfg)}")
        self._check(self.lib.mmpfn_finalize_weights(self.ctx), "mmpfn_finalize_weights")
        self._pos_cache: dict[int, torch.Tensor] = {}
        self._streams: list = []
        self.lanes = DEFAULT_LANES
        self.batch = DEFAULT_BATCH
        self.refs = 1  # model copies holding this engine (PerFeatureTransformer.__deepcopy__ shares it)
        self.serial = next(_SERIAL)

    # ------------------------------------------------------------------ plumbing
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _check(self, rc: int, what: str) -> None:
        _lib.check(self.lib, self.ctx, rc, what)

    def _bind_stream(self) -> None:
        self._check(self.lib.mmpfn_set_stream(self.ctx, ctypes.c_void_p(self._stream())), "mmpfn_set_stream")

    def release(self) -> None:
        """Drop one holder's reference; the context is destroyed with the last one."""
        self.refs -= 1
        if self.refs <= 0:
            self.close()

    def close(self) -> None:
        if getattr(self, "ctx", None):
            self.lib.mmpfn_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def _dev(self, t, dtype=torch.float32) -> torch.Tensor:
        """To the engine device on the current stream.  Host data goes through pinned memory without a
        host wait: a pageable host-to-device copy blocks the host until the stream has drained up to it,
        so every launch after it would trail the GPU (the predict path's per-member labels, the
        all-gather's member order and the aggregation's class permutations left ~0.5 ms of idle GPU
        per step that way)."""
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(np.asarray(t))
        if t.device.type == "cpu" and self.device.type == "cuda":
            return t.to(dtype).contiguous().pin_memory().to(self.device, non_blocking=True)
        return t.to(self.device, dtype).contiguous()

    def _pos(self, n: int) -> torch.Tensor:
        if n not in self._pos_cache:
            t = pos_rand(self.cfg, n, self.device).to(self.device)
            # drawn / copied on whichever stream (lane) asked first, read later from every lane: wait for
            # it here once, so no lane can read the cached table before it is complete
            torch.cuda.current_stream(self.device).synchronize()
            self._pos_cache[n] = t
        return self._pos_cache[n]

    # ------------------------------------------------------------------ compute
    def mixer_tokens(self, image, precision: int) -> torch.Tensor:
        """Modality projection heads: ``[S, n_mod, D]`` -> ``[S, C, E]`` tokens."""
        img = self._dev(image)
        if img.dim() == 2:
            img = img.unsqueeze(1)
        S, n_mod, D = img.shape
        if D != self.cfg.mixer_in_dim:
            raise ValueError(f"image embedding width {D} != {self.cfg.mixer_in_dim}")
        C = self.lib.mmpfn_mixer_tokens(self.ctx, n_mod)
        out = torch.empty((S, C, self.cfg.emsize), device=self.device, dtype=torch.float32)
        self._bind_stream()
        self._check(
            self.lib.mmpfn_mixer_forward(self.ctx, _ptr(img), S, n_mod, _ptr(out), precision), "mmpfn_mixer_forward"
        )
        return out

    def _prepare(self, x, tokens, y_train):
        y_np = y_train.detach().float().cpu().numpy() if isinstance(y_train, torch.Tensor) else np.asarray(y_train)
        y_np = y_np.reshape(-1).astype(np.float32)
        N = y_np.shape[0]
        xd = None if x is None else self._dev(x)
        if xd is not None and xd.dim() == 3:  # [S, 1, F] seam layout
            xd = xd.reshape(xd.shape[0], xd.shape[-1])
        td = None if tokens is None else self._dev(tokens)
        S = xd.shape[0] if xd is not None else td.shape[0]
        F = xd.shape[1] if xd is not None else 0
        C = td.shape[1] if td is not None else 0
        if td is not None and td.shape[0] != S:
            raise ValueError(f"tokens rows {td.shape[0]} != table rows {S}")
        fpg = self.cfg.features_per_group
        G = (F + fpg - 1) // fpg if xd is not None else 0
        uniq = self._dev(torch.from_numpy(target_uniques(y_np)))
        yd = self._dev(torch.from_numpy(y_np))
        if _DEBUG_KEEP:
            _KEEP.append((xd, td, yd, uniq))
        return xd, td, yd, uniq, S, F, C, N, G

    def forward(self, x, tokens, y_train, precision: int, check_nan: bool = True) -> torch.Tensor:
        """One ensemble member: logits ``[S - N, n_out]`` (fp32, on the engine device)."""
        xd, td, yd, uniq, S, F, C, N, G = self._prepare(x, tokens, y_train)
        if N < 1 or N > S:
            raise ValueError(f"single_eval_pos must be in [1, {S}], got {N}")
        pr = self._pos(G + C)
        out = torch.empty((S - N, self.cfg.n_out), device=self.device, dtype=torch.float32)
        self._bind_stream()
        self._check(
            self.lib.mmpfn_forward(
                self.ctx, _ptr(xd), S, F, _ptr(td), C, _ptr(yd), N, _ptr(uniq), uniq.numel(), _ptr(pr), _ptr(out),
                precision,
            ),
            "mmpfn_forward",
        )
        if check_nan:
            self.status()
        return out

    # ------------------------------------------------------------------ train-KV cache
    def cache_build(self, x, tokens, y_train, precision: int) -> "TrainCache":
        """``fit_mode="fit_with_cache"``: forward the train rows once and keep, per layer, head 0's
        K/V of the train rows plus the encoders' train statistics (``mmpfn_cache_build``;
        reference ``InferenceEngineCacheKV.prepare``, inference.py:403-445)."""
        xd, td, yd, uniq, S, F, C, N, G = self._prepare(x, tokens, y_train)
        if N != S:
            raise ValueError(f"cache_build takes the train rows only: {S} rows, {N} labels")
        pr = self._pos(G + C)
        h = ctypes.c_void_p()
        self._bind_stream()
        self._check(
            self.lib.mmpfn_cache_build(self.ctx, _ptr(xd), N, F, _ptr(td), C, _ptr(yd), _ptr(uniq), uniq.numel(),
                                       _ptr(pr), precision, ctypes.byref(h)),
            "mmpfn_cache_build",
        )
        return TrainCache(self, h.value, N=N, F=F, C=C, precision=precision)

    def cache_predict(self, cache: "TrainCache", x, tokens) -> torch.Tensor:
        """Test rows against a train-KV cache: logits ``[Q, n_out]`` (``mmpfn_cache_predict``;
        reference ``InferenceEngineCacheKV.iter_outputs``, inference.py:470-512)."""
        if cache.engine is not self or not cache.handle:
            raise ValueError("the cache belongs to another engine or was freed")
        xd = None if x is None else self._dev(x)
        if xd is not None and xd.dim() == 3:
            xd = xd.reshape(xd.shape[0], xd.shape[-1])
        td = None if tokens is None else self._dev(tokens)
        Q = xd.shape[0] if xd is not None else td.shape[0]
        F = xd.shape[1] if xd is not None else 0
        C = td.shape[1] if td is not None else 0
        if (F, C) != (cache.F, cache.C):
            raise ValueError(f"test rows have F={F}, C={C}; the cache was built with F={cache.F}, C={cache.C}")
        out = torch.empty((Q, self.cfg.n_out), device=self.device, dtype=torch.float32)
        self._bind_stream()
        self._check(
            self.lib.mmpfn_cache_predict(self.ctx, ctypes.c_void_p(cache.handle), _ptr(xd), Q, F, _ptr(td), C,
                                         _ptr(out)),
            "mmpfn_cache_predict",
        )
        return out

    def cache_predict_many(self, caches, xs, tokens, lanes: int | None = None) -> list[torch.Tensor]:
        """``cache_predict`` of several members, spread over concurrent lanes like ``forward_many``
        (2 lanes: 4.5 ms vs 6.7 ms for 4 members' 460 test rows; 4 lanes measured no better)."""
        n = len(caches)
        lanes = max(1, min(int(self.lanes if lanes is None else lanes), n, _lib.MMPFN_MAX_LANES))
        if lanes == 1:
            return [self.cache_predict(c, x, tokens) for c, x in zip(caches, xs)]
        main = torch.cuda.current_stream(self.device)
        streams = self._lane_streams(lanes)
        for st in streams:
            st.wait_stream(main)
        outs = []
        try:
            for k, (c, x) in enumerate(zip(caches, xs)):
                with torch.cuda.stream(streams[k % lanes]):
                    self._check(self.lib.mmpfn_select_lane(self.ctx, k % lanes), "mmpfn_select_lane")
                    outs.append(self.cache_predict(c, x, tokens))
        finally:
            self._check(self.lib.mmpfn_select_lane(self.ctx, 0), "mmpfn_select_lane")
            for st in streams:
                main.wait_stream(st)
        for o in outs:
            o.record_stream(main)
        return outs

    def forward_batch(self, items, precision: int) -> list[torch.Tensor]:
        """Members of ONE geometry (same S, N, F and tokens) in one batched forward
        (``mmpfn_forward_batch``: every layer kernel runs once over all members)."""
        prep = [self._prepare(x, t, y) for x, t, y in items]
        M = len(prep)
        xd0, td, _, _, S, F, C, N, G = prep[0]
        for p in prep[1:]:
            if (p[4], p[5], p[6], p[7]) != (S, F, C, N):
                raise ValueError("forward_batch members must share S, F, C and N")
        if N < 1 or N > S:
            raise ValueError(f"single_eval_pos must be in [1, {S}], got {N}")
        pr = self._pos(G + C)
        out = torch.empty((M, S - N, self.cfg.n_out), device=self.device, dtype=torch.float32)
        arr = ctypes.c_void_p * M
        xs = arr(*[_ptr(p[0]) for p in prep]) if F > 0 else None
        ys = arr(*[_ptr(p[2]) for p in prep])
        us = arr(*[_ptr(p[3]) for p in prep])
        ns = (ctypes.c_int * M)(*[p[3].numel() for p in prep])
        self._bind_stream()
        self._check(
            self.lib.mmpfn_forward_batch(self.ctx, M, xs, S, F, _ptr(td), C, ys, N, us, ns, _ptr(pr), _ptr(out),
                                         precision),
            "mmpfn_forward_batch",
        )
        return list(out.unbind(0))

    def forward_many(self, items, precision: int, lanes: int | None = None,
                     batch: int | None = None) -> list[torch.Tensor]:
        """Independent ensemble members ``[(x, tokens, y_train), ...]`` -> logits list.

        Members are spread over ``lanes`` forward lanes (per-member workspaces of the same
        context), each on its own HIP stream, so one member's kernels fill the tails and
        latency gaps of another's; members of one geometry are stacked ``batch`` at a time
        into one batched forward.  ``items`` may be a generator: a unit is launched as soon as
        its members have arrived, so the caller's host work for later members (the per-member
        preprocessing of a predict) overlaps the GPU work of earlier ones.  The caller's stream
        waits for all of them.  The reference runs its members one after another
        (inference.py:294-349); the results do not depend on lanes or batching.
        """
        batch = max(1, int(self.batch if batch is None else batch))
        if isinstance(items, (list, tuple)):
            n_units = len({self._geometry(*it) for it in items})  # lower bound on the unit count
            n_units = max(n_units, -(-len(items) // batch))
        else:
            n_units = _lib.MMPFN_MAX_LANES
        lanes = max(1, min(int(self.lanes if lanes is None else lanes), n_units, _lib.MMPFN_MAX_LANES))
        outs: dict[int, torch.Tensor] = {}
        store: dict[int, tuple] = {}

        def run(unit, stream=None):
            if len(unit) == 1:
                x, t, y = store[unit[0]]
                outs[unit[0]] = self.forward(x, t, y, precision, check_nan=False)
            else:
                for i, o in zip(unit, self.forward_batch([store[i] for i in unit], precision)):
                    outs[i] = o
            if stream is not None:
                # the unit's device inputs were made on the caller's stream (e.g. each member's
                # torch.cat of train and test rows): keep their blocks from being reused before the
                # lane's kernels have read them
                for i in unit:
                    for t in store[i]:
                        if isinstance(t, torch.Tensor) and t.is_cuda:
                            t.record_stream(stream)
            for i in unit:
                del store[i]

        main = torch.cuda.current_stream(self.device)
        streams = self._lane_streams(lanes) if lanes > 1 else [main]
        if lanes > 1:
            for st in streams:
                st.wait_stream(main)
        launched = 0

        def launch(unit):
            nonlocal launched
            if lanes == 1:
                run(unit)
            else:
                k = launched % lanes
                # the unit's inputs may have been produced on the caller's stream after the lanes forked
                # (a generator builds each member just before its unit launches): order the lane behind it
                streams[k].wait_stream(main)
                with torch.cuda.stream(streams[k]):
                    self._check(self.lib.mmpfn_select_lane(self.ctx, k), "mmpfn_select_lane")
                    run(unit, streams[k])
                    if _DEBUG_SYNC:
                        torch.cuda.synchronize(self.device)
            launched += 1

        pending: dict = {}  # geometry -> member indices waiting for a full unit
        n = 0
        try:
            for i, it in enumerate(items):
                n = i + 1
                store[i] = it
                g = self._geometry(*it)
                pending.setdefault(g, []).append(i)
                if len(pending[g]) == batch:
                    launch(pending.pop(g))
            for unit in sorted(pending.values(), key=lambda u: u[0]):
                launch(unit)
        finally:
            if lanes > 1:
                self._check(self.lib.mmpfn_select_lane(self.ctx, 0), "mmpfn_select_lane")
                for st in streams:
                    main.wait_stream(st)
        result = [outs[i] for i in range(n)]
        if lanes > 1:
            for o in result:  # allocated on a lane stream, consumed on the caller's
                o.record_stream(main)
        return result

    def _geometry(self, x, tokens, y_train) -> tuple:
        S = (x.shape[0] if x is not None else tokens.shape[0])
        F = 0 if x is None else x.shape[-1]
        C = 0 if tokens is None else tokens.shape[1]
        N = int(np.asarray(y_train.shape if isinstance(y_train, torch.Tensor) else np.shape(y_train)).prod())
        return (S, F, C, N, None if tokens is None else tokens.data_ptr())

    def _lane_streams(self, n: int) -> list:
        if len(self._streams) < n:
            self._streams += [_lane_stream(self.device, len(self._streams) + i) for i in range(n - len(self._streams))]
        return self._streams[:n]

    def aggregate(self, logits: torch.Tensor, perms, n_classes: int, temperature: float,
                  average_before_softmax: bool, class_weights=None) -> torch.Tensor:
        """Ensemble post-processing of classifier.py:541-566 on the device."""
        lg = logits.to(self.device, torch.float32).contiguous()
        M, Q, n_out = lg.shape
        pd = None
        if perms is not None:
            pd = self._dev(torch.as_tensor(np.asarray(perms, dtype=np.int32).reshape(M, n_classes)), torch.int32)
        C = n_classes if (temperature != 1 or perms is not None) else n_out
        cw = None
        if class_weights is not None:
            cw = self._dev(class_weights).reshape(-1)
            if cw.numel() != C:  # the reference's `output * class_prob_in_train` fails on this broadcast too
                raise RuntimeError(
                    f"The size of tensor a ({C}) must match the size of tensor b ({cw.numel()}) at non-singleton "
                    "dimension 1 (balance_probabilities with softmax_temperature == 1 and no class permutation)")
        out = torch.empty((Q, C), device=self.device, dtype=torch.float32)
        self._bind_stream()
        self._check(
            self.lib.mmpfn_aggregate(self.ctx, _ptr(lg), M, Q, n_out, _ptr(pd), n_classes, float(temperature),
                                     int(average_before_softmax), _ptr(cw), _ptr(out)),
            "mmpfn_aggregate",
        )
        return out

    def status(self) -> None:
        """Wait for every stream the context ran on and raise ``ValueError`` if any forward since the
        last call saw NaNs in its embedded input (transformer.py:727-731,790-796)."""
        self._bind_stream()
        self._check(self.lib.mmpfn_status(self.ctx), "mmpfn_forward")

    # ------------------------------------------------------------------ parity taps
    def embed_state(self, x, tokens, y_train, precision: int) -> torch.Tensor:
        """Embedded transformer input in reference order ``[S, T, E]``."""
        xd, td, yd, uniq, S, F, C, N, G = self._prepare(x, tokens, y_train)
        pr = self._pos(G + C)
        self._S = S
        self._bind_stream()
        self._check(
            self.lib.mmpfn_embed(
                self.ctx, _ptr(xd), S, F, _ptr(td), C, _ptr(yd), N, _ptr(uniq), uniq.numel(), _ptr(pr), precision
            ),
            "mmpfn_embed",
        )
        return self.copy_state()

    def run_layers(self, l0: int, l1: int) -> torch.Tensor:
        self._bind_stream()
        self._check(self.lib.mmpfn_run_layers(self.ctx, l0, l1), "mmpfn_run_layers")
        return self.copy_state()

    def copy_state(self) -> torch.Tensor:
        T = self.lib.mmpfn_state_tokens(self.ctx)
        out = torch.empty((self._S, T, self.cfg.emsize), device=self.device, dtype=torch.float32)
        self._check(self.lib.mmpfn_copy_state(self.ctx, _ptr(out), out.numel()), "mmpfn_copy_state")
        torch.cuda.current_stream(self.device).synchronize()
        return out

    # ------------------------------------------------------------------ per-sublayer taps
    def _state_tap(self, X: torch.Tensor, fn, argf) -> torch.Tensor:
        """Run a C-ABI sublayer tap on a reference-order state ``[S, T, E]`` (copied to the
        engine's token-major ``[T, S, E]``, updated in place, copied back).  The working copy is always a
        new tensor: with S == 1 or T == 1 the transposed view is already contiguous, and ``.contiguous()``
        would hand the caller's own storage to the kernel."""
        Xd = self._dev(X)
        Xt = torch.empty((Xd.shape[1], Xd.shape[0]) + tuple(Xd.shape[2:]), dtype=Xd.dtype, device=Xd.device)
        Xt.copy_(Xd.transpose(0, 1))
        T, S, _ = Xt.shape
        self._bind_stream()
        self._check(fn(self.ctx, *argf(Xt, S, T)), fn.__name__)
        return Xt.transpose(0, 1).contiguous()

    def feature_attention(self, layer: int, X: torch.Tensor, precision: int) -> torch.Tensor:
        """``LN(X + FeatAttn_layer(X))`` (layer.py:332-339) through ``mmpfn_feature_attention``."""
        return self._state_tap(X, self.lib.mmpfn_feature_attention,
                               lambda Xt, S, T: (layer, _ptr(Xt), S, T, precision))

    def item_attention_block(self, layer: int, X: torch.Tensor, n_train: int, precision: int) -> torch.Tensor:
        """``LN(X + ItemAttn_layer(X))`` (layer.py:341-379) through ``mmpfn_item_attention_block``."""
        return self._state_tap(X, self.lib.mmpfn_item_attention_block,
                               lambda Xt, S, T: (layer, _ptr(Xt), S, T, n_train, precision))

    def mlp_ln(self, layer: int, X: torch.Tensor, precision: int) -> torch.Tensor:
        """``LN(X + MLP_layer(X))`` (mlp.py:93-138) through ``mmpfn_mlp_ln`` (row-wise: any order)."""
        Xd = self._dev(X).contiguous().clone()
        self._bind_stream()
        self._check(self.lib.mmpfn_mlp_ln(self.ctx, layer, _ptr(Xd), Xd.numel() // self.cfg.emsize, precision),
                    "mmpfn_mlp_ln")
        return Xd

    def mgm(self, image, precision: int) -> torch.Tensor:
        """MultiheadGatedMLP tokens ``[S, mgm * n_mod, E]`` (transformer.py:33-57)."""
        img = self._dev(image)
        if img.dim() == 2:
            img = img.unsqueeze(1)
        S, n_mod, _ = img.shape
        out = torch.empty((S, self.cfg.mgm_heads * n_mod, self.cfg.emsize), device=self.device)
        self._bind_stream()
        self._check(self.lib.mmpfn_mgm(self.ctx, _ptr(img), S, n_mod, _ptr(out), precision), "mmpfn_mgm")
        return out

    def cap(self, mgm_tokens, precision: int) -> torch.Tensor:
        """CrossAttentionPooler tokens ``[S, cap, E]`` (transformer.py:60-88)."""
        tok = self._dev(mgm_tokens)
        S, M, _ = tok.shape
        out = torch.empty((S, self.cfg.cap_heads, self.cfg.emsize), device=self.device)
        self._bind_stream()
        self._check(self.lib.mmpfn_cap(self.ctx, _ptr(tok), S, M, _ptr(out), precision), "mmpfn_cap")
        return out

    def decode(self, n_query: int) -> torch.Tensor:
        out = torch.empty((n_query, self.cfg.n_out), device=self.device, dtype=torch.float32)
        self._bind_stream()
        self._check(self.lib.mmpfn_decode(self.ctx, _ptr(out)), "mmpfn_decode")
        return out


class TrainCache:
    """Device-resident train-KV cache of one ensemble member (owned by its engine's context)."""

    def __init__(self, engine: HipEngine, handle: int, *, N: int, F: int, C: int, precision: int):
        self.engine, self.handle = engine, handle
        self.N, self.F, self.C, self.precision = N, F, C, precision

    @property
    def nbytes(self) -> int:
        return int(self.engine.lib.mmpfn_cache_bytes(ctypes.c_void_p(self.handle))) if self.handle else 0

    def free(self) -> None:
        if self.handle and getattr(self.engine, "ctx", None):
            self.engine.lib.mmpfn_cache_free(self.engine.ctx, ctypes.c_void_p(self.handle))
        self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
