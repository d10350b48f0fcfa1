"""GPU: BASELINE.json's headline configs at full size against the oracle, the config-D ensemble
(32 ragged members through the lane / batch scheduler), NaN reporting across queued forwards,
and the reference's cache-engine call form on the model seam.

Full-size parity (configs C, C at mgm = 256, D): the fp32 engine against the oracle evaluated in
fp32 on the same GPU (the oracle's torch code moved to the device; it is pinned by the reference
goldens on CPU).  Tolerances, written here:
  fp32 : max|d logits| <= 1e-4 * max(1, max|ref|), argmax identical on every row
  bf16 : max|d logits| <= BF16_BAND[config] * max(1, max|ref|), argmax agreement >= BF16_AGREE[config]
The bf16 bands are about twice the deviation measured on MI355X (profiles/r02/parity_bf16.jsonl,
printed by the test); the reference itself runs fp16 autocast on a GPU.
"""

import copy
import json
import os

import numpy as np
import pytest
import torch

from helpers import check_argmax, oracle_spec, rel_err, torch_sd
from oracle.forward import oracle_forward

pytestmark = pytest.mark.gpu

F32_TOL = 1e-4
S_ROWS, N_TRAIN, N_FEAT, N_CAT, N_CLS = 2298, 1838, 21, 18, 6
# name -> (mgm heads, cap heads, modalities, data seed)
FULL = {"C": (64, 24, 1, 2), "C-mgm256": (256, 24, 1, 2), "D": (64, 24, 2, 3)}
BF16_BAND = {"C": 3.5e-2, "C-mgm256": 3.5e-2, "D": 2e-2}  # measured 1.64e-2, 1.77e-2, 0.99e-2
BF16_AGREE = {"C": 0.995, "C-mgm256": 0.995, "D": 0.995}  # measured 1.00 on all three
F16_BAND = 2e-2  # fp16 mode (MMPFN_PREC_F16, the reference's autocast dtype), all three configs


def _model(cfg, sd):
    from multimodalpfn_amd.model.transformer import PerFeatureTransformer

    model = PerFeatureTransformer(cfg)
    model.load_state_dict(torch_sd(sd))
    norm = next(e for e in model.encoder if "InputNormalizationEncoderStep" in str(e.__class__))
    norm.remove_outliers, norm.remove_outliers_sigma = True, 12.0
    return model.to("cuda")


def _log(rec):
    print(json.dumps(rec))
    path = os.environ.get("MMPFN_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


@pytest.mark.parametrize("name", list(FULL))
def test_full_size_config_matches_oracle(name):
    """PAD-UFES-20 shape at full size (N = 1838, Q = 460, F = 21 with 18 categorical, 12 layers):
    C = image [S,1,768] MGM64 + CAP24 (the benchmarked config), C at MGM256 (the reference's best
    grid cell, charts/pad_ufes_20.csv), D = image + text [S,2,768] (CAP over 128 MGM tokens)."""
    from synth import synth_image, synth_labels, synth_state_dict, synth_table

    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    mgm, cap, n_mod, seed = FULL[name]
    torch.backends.cuda.matmul.allow_tf32 = False
    cfg = ModelConfig(mgm_heads=mgm, cap_heads=cap)
    sd = synth_state_dict(state_dict_spec(cfg), seed)
    model = _model(cfg, sd)
    x = torch.from_numpy(synth_table(S_ROWS, N_FEAT, seed, n_cat=N_CAT)).cuda()
    im = torch.from_numpy(synth_image(S_ROWS, n_mod, seed)).cuda()
    y = torch.from_numpy(synth_labels(S_ROWS, N_CLS, seed)[:N_TRAIN]).cuda()
    from multimodalpfn_amd import _lib

    with torch.inference_mode():
        f32 = model(None, x[:, None, :], im, y, single_eval_pos=N_TRAIN).squeeze(1).float().cpu().numpy()
        b16 = model(None, x[:, None, :], im, y, single_eval_pos=N_TRAIN,
                    precision=_lib.PREC_BF16).squeeze(1).float().cpu().numpy()
        h16 = model(None, x[:, None, :], im, y, single_eval_pos=N_TRAIN,
                    precision=_lib.PREC_F16).squeeze(1).float().cpu().numpy()
    model.invalidate_engine()
    w = {k: v.cuda() for k, v in torch_sd(sd).items()}
    ref = oracle_forward(oracle_spec(cfg), w, x, im, y).cpu().numpy()
    del w
    torch.cuda.empty_cache()
    assert ref.shape == (S_ROWS - N_TRAIN, cfg.n_out)
    assert np.isfinite(f32).all() and np.isfinite(b16).all()
    e32, eb, eh = rel_err(f32, ref), rel_err(b16, ref), rel_err(h16, ref)
    agree = float((b16.argmax(1) == ref.argmax(1)).mean())
    _log({"config": name, "S": S_ROWS, "N": N_TRAIN, "mgm": mgm, "cap": cap, "n_mod": n_mod,
          "f32_rel_err": e32, "f32_argmax_equal": bool((f32.argmax(1) == ref.argmax(1)).all()),
          "bf16_rel_err": eb, "bf16_argmax_agree": agree, "f16_rel_err": eh,
          "f16_argmax_agree": float((h16.argmax(1) == ref.argmax(1)).mean()), "ref_absmax": float(np.abs(ref).max())})
    assert e32 <= F32_TOL, (name, e32)
    assert (f32.argmax(1) == ref.argmax(1)).all()
    assert eb <= BF16_BAND[name], (name, eb)
    check_argmax(b16, ref, BF16_AGREE[name], f"bf16 {name}")
    assert np.isfinite(h16).all()
    assert eh <= F16_BAND, (name, eh)
    check_argmax(h16, ref, BF16_AGREE[name], f"f16 {name}")


def _ragged_members(n, seed, tok_n):
    """Members as default preprocessing makes them: different widths (quantile/SVD members
    append columns, 'none' members keep 21), a feature shuffle and a class permutation each."""
    from synth import synth_labels, synth_table

    rng = np.random.default_rng(seed)
    base = synth_table(S_ROWS, 51, seed, n_cat=N_CAT)
    y = synth_labels(S_ROWS, N_CLS, seed)[:N_TRAIN].astype(np.int64)
    items = []
    for m in range(n):
        F = (21, 51, 11, 31)[m % 4]
        xm = np.ascontiguousarray(base[:, rng.permutation(51)[:F]])
        ym = rng.permutation(N_CLS)[y].astype(np.float32)
        items.append((torch.from_numpy(xm), ym))
    return items


def test_config_d_32_ragged_members_scheduled_equal_single_forwards():
    """Config D's ensemble (32 members, image + text, MGM64 + CAP24) through forward_many with
    lanes and same-geometry batching equals each member forwarded alone, bitwise (inference.py:
    294-349 runs them one after another)."""
    from synth import synth_image, synth_state_dict

    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(mgm_heads=64, cap_heads=24)
    eng = _model(cfg, synth_state_dict(state_dict_spec(cfg), 3)).engine()
    im = torch.from_numpy(synth_image(S_ROWS, 2, 3)).cuda()
    members = _ragged_members(32, 3, None)
    with torch.inference_mode():
        tok = eng.mixer_tokens(im, _lib.PREC_BF16)
        items = [(xm.cuda(), tok, ym) for xm, ym in members]
        sched = eng.forward_many(items, _lib.PREC_BF16, lanes=2, batch=2)
        eng.status()
        single = [eng.forward(xm, t, ym, _lib.PREC_BF16) for xm, t, ym in items]
        torch.cuda.synchronize()
    assert len({it[0].shape[1] for it in items}) == 4
    for i, (a, b) in enumerate(zip(sched, single)):
        assert torch.isfinite(a).all(), i
        assert torch.equal(a.cpu(), b.cpu()), i


@pytest.mark.parametrize("lanes,batch", [(2, 1), (1, 1), (2, 2), (1, 4)])
def test_nan_in_an_early_member_is_reported(lanes, batch):
    """An all-NaN train column in member 0 of a 4-member forward_many raises ValueError, however
    the members are laid out on lanes and batches (reference: transformer.py:790-796)."""
    from synth import synth_labels, synth_state_dict, synth_table

    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(nlayers=2, mgm_heads=4, cap_heads=2)
    eng = _model(cfg, synth_state_dict(state_dict_spec(cfg), 8)).engine()
    S, N, F = 200, 150, 7
    x = synth_table(S, F, 8)
    y = synth_labels(S, 3, 8)[:N]
    items = [(torch.from_numpy(x.copy()).cuda(), None, y) for _ in range(4)]
    items[0][0][:N, 2] = float("nan")
    with torch.inference_mode():
        eng.forward_many(items, _lib.PREC_BF16, lanes=lanes, batch=batch)
        with pytest.raises(ValueError, match="NaN"):
            eng.status()
        eng.forward_many(items[1:], _lib.PREC_BF16, lanes=lanes, batch=batch)  # clean members: no stale flag
        eng.status()


def test_reference_cache_engine_call_form():
    """InferenceEngineCacheKV drives the model as: deepcopy per member, one train-only call
    model(None, X_train, y, single_eval_pos=len(X)) (inference.py:425-436), then
    model(None, X_test, None, single_eval_pos=None) (:499-507).  The test rows' logits equal the
    full forward's, bitwise."""
    from synth import synth_labels, synth_state_dict, synth_table

    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(nlayers=3, mgm_heads=4, cap_heads=2)
    base = _model(cfg, synth_state_dict(state_dict_spec(cfg), 12))
    base.cache_trainset_representation = True  # load_model sets it (loading.py:497)
    S, N, F = 400, 300, 9
    x = torch.from_numpy(synth_table(S, F, 12, n_cat=3, nan_frac=0.02)).cuda()[:, None, :]
    y = torch.from_numpy(synth_labels(S, 4, 12)[:N]).cuda()
    with torch.inference_mode():
        full = base(None, x, y, single_eval_pos=N)
        with pytest.raises(RuntimeError, match="train-KV cache"):
            copy.deepcopy(base)(None, x[N:], None, single_eval_pos=None)
        members = [copy.deepcopy(base) for _ in range(2)]
        for m in members:
            assert m(None, x[:N], y, single_eval_pos=N).shape == (0, 1, cfg.n_out)
        outs = [m(None, x[N:], None, single_eval_pos=None) for m in members]
        with torch.autocast("cuda"):
            m16 = copy.deepcopy(base)
            m16(None, x[:N], y, single_eval_pos=N)
            o16 = m16(None, x[N:], None, single_eval_pos=None)
            f16 = base(None, x, y, single_eval_pos=N)
    for o in outs:
        assert o.shape == full.shape
        assert torch.equal(o.cpu(), full.cpu())
    assert torch.equal(o16.cpu(), f16.cpu())
    for m in members:
        m.empty_trainset_representation_cache()


def test_engines_share_lane_streams_and_stay_exact():
    """Lane streams are process-wide (engine._lane_stream: a second engine's own pair could land on one hardware queue
    and run its lanes serially): two engines get the same lane streams, and members of both, launched
    alternately on those shared lanes, equal each engine's members forwarded alone, bitwise."""
    from synth import synth_image, synth_state_dict

    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(nlayers=2, mgm_heads=8, cap_heads=4)
    e1 = _model(cfg, synth_state_dict(state_dict_spec(cfg), 5)).engine()
    e2 = _model(cfg, synth_state_dict(state_dict_spec(cfg), 6)).engine()
    im = torch.from_numpy(synth_image(S_ROWS, 1, 5)).cuda()
    members = _ragged_members(4, 5, None)
    with torch.inference_mode():
        outs, refs = [], []
        for eng in (e1, e2):
            tok = eng.mixer_tokens(im, _lib.PREC_F16)
            items = [(xm.cuda(), tok, ym) for xm, ym in members]
            outs.append((eng, items, eng.forward_many(items, _lib.PREC_F16, lanes=2, batch=1)))
        assert e1._lane_streams(2) == e2._lane_streams(2)
        for eng, items, got in outs:
            eng.status()
            refs.append([eng.forward(x, t, y, _lib.PREC_F16) for x, t, y in items])
        torch.cuda.synchronize()
    for (eng, items, got), ref in zip(outs, refs):
        for a, b in zip(got, ref):
            assert torch.isfinite(a).all()
            assert torch.equal(a.cpu(), b.cpu())
