"""GPU parity: the HIP engine (through the C-ABI) against the oracle / reference goldens.

Tolerances (north star: fp32 logits within 1e-4 relative, argmax bit-exact):
  fp32 parity mode : max|d logits| <= 1e-4 * max(1, max|ref|), argmax identical
  bf16 perf mode   : max|d logits| <= 2e-2 * max(1, max|ref|) (about 2x the measured worst), argmax agreement >= 99.5 % (measured 100 % on every case)
"""

import math

import numpy as np
import pytest
import torch

from helpers import CASES, GOLDEN, check_argmax, load_case, oracle_spec, rel_err, report, torch_sd
from oracle.forward import layer_forward, oracle_forward

pytestmark = pytest.mark.gpu

F32_TOL = 1e-4
LARGE_BF16_TOL = {"B": 2.5e-2, "E": 3.5e-2}  # measured 1.28e-2 and 1.80e-2 (profiles/r02)
BF16_AGREE = 0.995  # argmax agreement; measured 1.00 on every golden and on B / E (profiles/r02)
F8_TOL = 5e-2  # config E with the fp8 P.V (MMPFN_PREC_BF16_F8 / _F8E5) against the oracle
F16_TOL = 1e-2  # fp16 mode (MMPFN_PREC_F16: fp16 state and operands, the reference's autocast dtype)
LARGE_F16_TOL = {"B": 2e-2, "E": 2e-2}
BF16_TOL = 2e-2  # measured 3.1e-3 .. 9.5e-3 over the goldens (profiles/r02/pytest_gpu_r02a.log)


def make_model(cfg, sd):
    from multimodalpfn_amd.model.transformer import PerFeatureTransformer

    model = PerFeatureTransformer(cfg)
    model.load_state_dict(torch_sd(sd))
    norm = next(e for e in model.encoder if "InputNormalizationEncoderStep" in str(e.__class__))
    norm.remove_outliers = cfg.remove_outliers_sigma is not None
    norm.remove_outliers_sigma = cfg.remove_outliers_sigma or 4.0
    return model.to("cuda")


def run_case(z, model, autocast=False, precision=None):
    x = torch.from_numpy(z["x"])[:, None, :].cuda() if "x" in z else None
    im = torch.from_numpy(z["image"]).cuda() if "image" in z else None
    y = torch.from_numpy(z["y_train"]).cuda()
    kw = {} if precision is None else {"precision": precision}
    with torch.autocast("cuda", enabled=autocast), torch.inference_mode():
        out = model(None, x, im, y, only_return_standard_out=True, categorical_inds=[], single_eval_pos=len(y), **kw)
    return out.squeeze(1).float().cpu().numpy()


@pytest.mark.parametrize("case", CASES)
def test_forward_fp32_matches_reference(case):
    z, meta, cfg, sd = load_case(case)
    out = run_case(z, make_model(cfg, sd))
    err = rel_err(out, z["logits"])
    print(f"fp32 (split-bf16) {case}: rel err {err:.3e}")
    assert err <= F32_TOL, err
    assert (out.argmax(1) == z["logits"].argmax(1)).all()


@pytest.mark.parametrize("form", [1, 2, 3])
def test_parity_attention_cheap_forms_are_opt_in(form):
    """The parity mode's cheap item-attention forms (fp16 S / two-product P.V; mmpfn_set_parity_attention_min_keys)
    run only when asked: off by default (the goldens above ran three products), on request they change the logits by
    no more than the sweep measured (profiles/r06/parity_n0_sweep_form*.txt: worst 4.3e-4 at N = 40, written here with
    its margin), argmax unchanged on the 12-layer case, and switching back restores the exact form bitwise."""
    from multimodalpfn_amd import _lib

    lib = _lib.load_library()
    z, meta, cfg, sd = load_case("pad_ufes_12l")
    model = make_model(cfg, sd)
    exact = run_case(z, model)
    prev = lib.mmpfn_set_parity_attention_min_keys(0, form)
    try:
        assert prev == -1
        cheap = run_case(z, model)
    finally:
        lib.mmpfn_set_parity_attention_min_keys(prev, 3)
    again = run_case(z, model)
    e = rel_err(cheap, z["logits"])
    report(f"parity cheap form {form} pad_ufes_12l: rel err {e:.3e} (exact {rel_err(exact, z['logits']):.3e})")
    assert not np.array_equal(cheap, exact)
    assert e <= 1e-3
    assert (cheap.argmax(1) == z["logits"].argmax(1)).all()
    np.testing.assert_array_equal(again, exact)


@pytest.mark.parametrize("case", CASES)
def test_forward_fp32_input_mfma_mode_matches_reference(case, monkeypatch):
    """MMPFN_F32_MODE=mfma: the parity mode on fp32-input MFMA (exact fp32 fma chains) still holds 1e-4."""
    monkeypatch.setenv("MMPFN_F32_MODE", "mfma")
    z, meta, cfg, sd = load_case(case)
    out = run_case(z, make_model(cfg, sd))
    err = rel_err(out, z["logits"])
    print(f"fp32-input MFMA {case}: rel err {err:.3e}")
    assert err <= F32_TOL, err
    assert (out.argmax(1) == z["logits"].argmax(1)).all()


@pytest.mark.parametrize("case", CASES)
def test_forward_bf16_close_to_reference(case):
    from multimodalpfn_amd import _lib

    z, meta, cfg, sd = load_case(case)
    out = run_case(z, make_model(cfg, sd), precision=_lib.PREC_BF16)
    assert np.isfinite(out).all()
    err = rel_err(out, z["logits"])
    print(f"bf16 {case}: rel err {err:.3e}")
    assert err <= BF16_TOL, err
    check_argmax(out, z["logits"], BF16_AGREE, f"bf16 {case}")


@pytest.mark.parametrize("case", CASES)
def test_forward_f16_close_to_reference(case):
    """MMPFN_PREC_F16 (the reference's fp16 autocast: fp16 state between kernels, fp16 MFMA operands)."""
    from multimodalpfn_amd import _lib

    z, meta, cfg, sd = load_case(case)
    model = make_model(cfg, sd)
    out = run_case(z, model, precision=_lib.PREC_F16)
    b16 = run_case(z, model, precision=_lib.PREC_BF16)
    assert np.array_equal(run_case(z, model, autocast=True), out)  # the reference's autocast = this mode
    assert np.isfinite(out).all()
    err, eb = rel_err(out, z["logits"]), rel_err(b16, z["logits"])
    print(f"f16 {case}: rel err {err:.3e} (bf16 {eb:.3e})")
    assert err <= F16_TOL, err
    check_argmax(out, z["logits"], BF16_AGREE, f"f16 {case}")


def test_embedding_and_layer_taps_fp32():
    from multimodalpfn_amd import _lib

    z, meta, cfg, sd = load_case("pad_ufes_12l")
    model = make_model(cfg, sd)
    eng = model.engine()
    tok = eng.mixer_tokens(torch.from_numpy(z["image"]).cuda(), _lib.PREC_F32)
    assert rel_err(tok.cpu().numpy(), z["mixer_tokens"]) < 1e-4
    X = eng.embed_state(torch.from_numpy(z["x"]).cuda(), tok, z["y_train"], _lib.PREC_F32)
    assert rel_err(X.cpu().numpy(), z["embedded_input"]) < 1e-5
    X1 = eng.run_layers(0, 1)
    assert rel_err(X1.cpu().numpy(), z["layer0"]) < 1e-4


def test_each_layer_matches_oracle_layer():
    """Feed the oracle's own layer input to one engine layer (isolates per-layer error)."""
    from multimodalpfn_amd import _lib

    z, meta, cfg, sd = load_case("mgmcap_edge")
    model = make_model(cfg, sd)
    eng = model.engine()
    spec = oracle_spec(cfg)
    w = torch_sd(sd)
    tok = eng.mixer_tokens(torch.from_numpy(z["image"]).cuda(), _lib.PREC_F32)
    X = eng.embed_state(torch.from_numpy(z["x"]).cuda(), tok, z["y_train"], _lib.PREC_F32).cpu()
    N = len(z["y_train"])
    for l in range(cfg.nlayers):
        ref = layer_forward(spec, w, l, X.double(), N).float()
        got = eng.run_layers(l, l + 1).cpu()
        assert rel_err(got.numpy(), ref.numpy()) < 2e-5, l
        X = got


@pytest.mark.parametrize("case", ["tab_small", "mgmcap_edge", "two_queries", "pad_ufes_12l"])
def test_each_layer_bf16_close_to_oracle_layer(case):
    """bf16 mode, one layer at a time from the oracle's input (fused feature-block kernel,
    bf16 item attention, fused MLP): bf16-rounding-level agreement with the fp64 oracle."""
    from multimodalpfn_amd import _lib

    z, meta, cfg, sd = load_case(case)
    model = make_model(cfg, sd)
    eng = model.engine()
    spec = oracle_spec(cfg)
    w = torch_sd(sd)
    tok = None
    if "image" in z:
        tok = eng.mixer_tokens(torch.from_numpy(z["image"]).cuda(), _lib.PREC_F32)
    xin = torch.from_numpy(z["x"]).cuda() if "x" in z else None
    X = eng.embed_state(xin, tok, z["y_train"], _lib.PREC_BF16).cpu()
    N = len(z["y_train"])
    for l in range(min(cfg.nlayers, 3)):
        ref = layer_forward(spec, w, l, X.double(), N).float()
        got = eng.run_layers(l, l + 1).cpu()
        assert torch.isfinite(got).all()
        err = rel_err(got.numpy(), ref.numpy())
        assert err < 4e-2, (l, err)
        X = got


def _attn_ref(q, k, v):
    s = (q.double() @ k.double().transpose(-1, -2)) / math.sqrt(q.shape[-1])
    return torch.softmax(s, -1) @ v.double()


# parity (split bf16), bf16, fp32-input MFMA, fp8 P.V with P e4m3 / e5m2 (V^T e4m3); |O| <= ~1
# (fp8: x max(1, max |V|) in test_item_attention_layer_fp8; measured max 0.125 at N = 1, |V| <= 3.6)
QK_BF16 = 0x100  # _lib.ATTN_QK_BF16: the fp16 forward's form of the layer tap (bf16 Q / K, fp16 O)
ATTN_TOL = {0: 5e-5, 1: 2e-2, 2: 2e-5, 3: 1e-1, 4: 1e-1, 5: 2e-2, 6: 1e-1, 7: 1e-1}  # 3 / 4 / 6 / 7: the
# overflow / re-run tests (exact path); the fp8 results themselves: _f8_layer_ref, F8_QBAND


@pytest.mark.parametrize("prec", [0, 1, 2])
@pytest.mark.parametrize(
    "S,N,T", [(2298, 1838, 3), (70, 1, 2), (130, 64, 1), (200, 65, 2), (129, 127, 1), (300, 299, 1)]
)
def test_item_attention_kernel(prec, S, N, T):
    """Sample-axis attention kernel alone: train self-attn (own heads) + test MQA (head 0), in the three
    precision modes (prec 0: split-bf16 three-product MFMAs on fp32 operands)."""
    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.engine import HipEngine  # noqa: F401

    lib = _lib.load_library()
    ctx = lib.mmpfn_create(0, None)
    H, d = 6, 32
    Npad = (N + 63) // 64 * 64
    g = torch.Generator().manual_seed(S * 7 + N)
    dt = torch.bfloat16 if prec == 1 else torch.float32
    q = torch.randn(T, H, S, d, generator=g)
    k = torch.randn(T, H, N, d, generator=g)
    v = torch.randn(T, H, N, d, generator=g)
    kp = torch.full((T, H, Npad, d), float("nan"))
    kp[:, :, :N] = k
    vt = torch.full((T, H, d, Npad), float("nan"))  # NaN padding must never leak
    vt[:, :, :, :N] = v.transpose(-1, -2)
    qd, kd, vd = q.to("cuda", dt), kp.to("cuda", dt), vt.to("cuda", dt)
    out = torch.zeros(T, S, H * d, device="cuda", dtype=dt)
    assert lib.mmpfn_item_attention(ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), S, T, H, Npad,
                                    0, N, N, -1, prec) == 0
    if N < S:
        assert lib.mmpfn_item_attention(ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), S, T, H,
                                        Npad, N, S - N, N, 0, prec) == 0
    torch.cuda.synchronize()
    lib.mmpfn_destroy(ctx)
    qr, kr, vr = q.to(dt).float(), k.to(dt).float(), v.to(dt).float()
    ref_tr = _attn_ref(qr[:, :, :N], kr, vr)
    ref_te = _attn_ref(qr[:, :, N:], kr[:, :1].expand_as(kr), vr[:, :1].expand_as(vr))
    ref = torch.cat([ref_tr, ref_te], 2).permute(0, 2, 1, 3).reshape(T, S, H * d)
    got = out.float().cpu()
    err = (got.double() - ref).abs().max().item()
    print(f"item attention prec {prec} S={S} N={N} T={T}: max abs err {err:.3e}")
    assert torch.isfinite(got).all()
    assert err < ATTN_TOL[prec]


def _qkv_case(S, N, T, H=6, d=32, seed=0):
    Npad = (N + 63) // 64 * 64
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(T, H, S, d, generator=g)
    k = torch.randn(T, H, N, d, generator=g)
    v = torch.randn(T, H, N, d, generator=g)
    return q, k, v, Npad


def _launch_layer(q, k, v, Npad, N, prec=1):
    """prec 1: the engine's one-launch bf16 layer tap; prec 0: the parity-mode kernel on fp32 operands
    (train rows, then test rows, through mmpfn_item_attention)."""
    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.engine import HipEngine  # noqa: F401

    T, H, S, d = q.shape
    kp = torch.full((T, H, Npad, d), float("nan"))
    kp[:, :, :N] = k
    vt = torch.full((T, H, d, Npad), float("nan"))  # NaN padding must never leak
    vt[:, :, :, :N] = v.transpose(-1, -2)
    lib = _lib.load_library()
    ctx = lib.mmpfn_create(0, None)
    dt = torch.bfloat16 if prec & 0xff in (1, 3, 4, 5, 6, 7) else torch.float32
    qd, kd, vd = q.to("cuda", dt), kp.to("cuda", dt), vt.to("cuda", dt)
    out = torch.zeros(T, S, H * d, device="cuda", dtype=dt)
    if prec == 1:
        assert lib.mmpfn_item_attention_layer(ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), S, T,
                                              H, Npad, N) == 0
    elif prec & 0xff in (3, 4, 5, 6, 7):  # fp8 P.V (P e4m3: 3 / 6, e5m2: 4 / 7); 5-7: fp16 Q / K / O
        if prec & 0xff >= 5:  # (| ATTN_QK_BF16: the fp16 forward's form, bf16 Q / K and fp16 O)
            if not prec & _lib.ATTN_QK_BF16:
                qd, kd = q.to("cuda", torch.float16), kp.to("cuda", torch.float16)
            out = out.to(torch.float16)
        assert lib.mmpfn_item_attention_layer_ex(ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), S,
                                                 T, H, Npad, N, prec) == 0
    else:
        assert lib.mmpfn_item_attention(ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), S, T, H,
                                        Npad, 0, N, N, -1, prec) == 0
        if N < S:
            assert lib.mmpfn_item_attention(ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), S, T,
                                            H, Npad, N, S - N, N, 0, prec) == 0
    torch.cuda.synchronize()
    lib.mmpfn_destroy(ctx)
    return out.float().cpu()


def _layer_ref(q, k, v, N, prec=1):
    T, H, S, d = q.shape
    qkb, prec = bool(prec & QK_BF16), prec & 0xff
    dt = torch.bfloat16 if prec in (1, 3, 4) else torch.float32
    qr, kr, vr = (t.to(dt).float() for t in (q, k, v))
    if prec >= 5:  # fp16 Q / K (bf16 in the fp16 forward's form), bf16 V
        qk = torch.bfloat16 if qkb else torch.float16
        qr, kr, vr = q.to(qk).float(), k.to(qk).float(), v.bfloat16().float()
    ref_tr = _attn_ref(qr[:, :, :N], kr, vr)
    ref_te = _attn_ref(qr[:, :, N:], kr[:, :1].expand_as(kr), vr[:, :1].expand_as(vr))
    return torch.cat([ref_tr, ref_te], 2).permute(0, 2, 1, 3).reshape(T, S, H * d)


@pytest.mark.parametrize("S,N,T", [(2298, 1838, 2), (70, 1, 2), (130, 64, 1), (200, 65, 3), (700, 333, 1)])
def test_item_attention_layer_fused(S, N, T):
    """One launch: train rows on their own heads + test rows of all heads on head 0 (MQA)."""
    q, k, v, Npad = _qkv_case(S, N, T, seed=S + N)
    got = _launch_layer(q, k, v, Npad, N)
    ref = _layer_ref(q, k, v, N)
    assert torch.isfinite(got).all()
    assert (got.double() - ref).abs().max().item() < 2e-2


F8_ETOP = {3: 0, 4: 6, 6: 0, 7: 6}     # attention_pipe.hip P8<1|2>::ETOP: where the first key tile's max lands
F8_EMAX = {3: 8, 4: 15, 6: 8, 7: 15}   # P8<>::EMAX
F8_FMT = {3: torch.float8_e4m3fn, 4: torch.float8_e5m2, 6: torch.float8_e4m3fn, 7: torch.float8_e5m2}
F8_QBAND = 1e-2  # x max|V|: accumulation order, exp2 ulps and the output rounding, against the quantising reference


def _f8_layer_ref(q, k, v, N, prec):
    """The fp8 P.V path's own arithmetic (float64 sums) (attention_pipe.hip: attn_pipe_kernel<F8, QF16> prologue and
    P8<F8>): Q rounded to the Q / K dtype, scaled by log2(e)/sqrt(32) and rounded again; s = Q K^T in log2 units;
    V^T saturated to +-448 and rounded to e4m3; per query a power-of-two scale 2^e from the max over the real keys of
    the FIRST tile processed (the partial last tile when N % 64 != 0, else tile 0), e = clamp(floor(max) - ETOP,
    -EMAX if partial else -100, 100); P' = fp8(exp2(s) / 2^e) in e4m3 / e5m2; O = sum P' V8 / sum P'."""
    T, H, S, d = q.shape
    qkb, prec = bool(prec & QK_BF16), prec & 0xff
    qk_dt = torch.float16 if prec >= 5 and not qkb else torch.bfloat16
    c = math.log2(math.e) / math.sqrt(d)
    qs = (q.to(qk_dt).float() * c).to(qk_dt).double()
    ks = k.to(qk_dt).double()
    v8 = v.to(torch.bfloat16).float().clamp(-448.0, 448.0).to(torch.float8_e4m3fn).double()
    nfull = N // 64
    partial = nfull * 64 != N
    first = slice(64 * nfull, N) if partial else slice(0, min(64, N))
    elo = -F8_EMAX[prec] if partial else -100

    def attend(qh, kh, vh):
        s = qh @ kh.transpose(-1, -2)
        m = s[..., first].amax(-1, keepdim=True)
        e = torch.clamp(torch.floor(m) - F8_ETOP[prec], elo, 100)
        p = (torch.exp2(s.float()).double() / torch.exp2(e)).float().to(F8_FMT[prec]).double()
        return (p @ vh) / p.sum(-1, keepdim=True)

    tr = attend(qs[:, :, :N], ks, v8)
    te = attend(qs[:, :, N:], ks[:, :1].expand_as(ks), v8[:, :1].expand_as(v8))
    return torch.cat([tr, te], 2).permute(0, 2, 1, 3).reshape(T, S, H * d)


def _f8_outcomes(got, q, k, v, N, prec):
    """Each (row, head) of an fp8 launch is one of two outcomes: the wave kept its fp8 pass (the quantising
    reference) or re-ran on the exact bf16 path (an overflow past the format, or the underflow guard).  Returns the
    per-(row, head) error against the nearer outcome and the fraction that re-ran."""
    T, H, S, d = q.shape
    got = got.double()
    e_q = (got - _f8_layer_ref(q, k, v, N, prec)).reshape(T, S, H, d).abs().amax(-1)
    e_x = (got - _layer_ref(q, k, v, N, (5 | (prec & QK_BF16)) if prec & 0xff >= 5 else 1)).reshape(T, S, H, d)
    e_x = e_x.abs().amax(-1)
    # (a P past the format converts to NaN / inf in the quantising reference too: that row's fp8 outcome does not
    # exist, the kernel re-ran it -- fmin takes the exact outcome there)
    return torch.fmin(e_q, e_x), (~(e_q <= e_x)).double().mean().item()


@pytest.mark.parametrize("prec", [3, 4, 6, 7, 6 | QK_BF16, 7 | QK_BF16])
@pytest.mark.parametrize("S,N,T", [(2298, 1838, 2), (70, 1, 2), (130, 64, 1), (200, 65, 3), (700, 333, 1),
                                   (12000, 10000, 1)])
def test_item_attention_layer_fp8(S, N, T, prec):
    """Config E's fp8 path (MMPFN_PREC_{BF16,F16}_F8 / _F8E5): P.V and the row sums on block-scaled fp8 MFMA, the
    per-query scale from the first key tile, the partial tile's padded keys cancelled at P'(0) -- against a
    reference that quantises V^T and P exactly as the kernel does, within 1e-2 max|V|; a wave
    whose fp8 row sums fail the overflow / underflow checks re-runs exactly (small N: L < nk 2^(EMIN+6) often)."""
    q, k, v, Npad = _qkv_case(S, N, T, seed=S + N + prec)
    got = _launch_layer(q, k, v, Npad, N, prec)
    assert torch.isfinite(got).all()
    err, rerun = _f8_outcomes(got, q, k, v, N, prec)
    vmax = v.abs().max().item()
    print(f"attention fp8 prec {prec} S={S} N={N} T={T}: max {err.max():.3e} (max|V| {vmax:.2f}), re-run {rerun:.3f}")
    assert err.max().item() < F8_QBAND * vmax
    if N >= 1838:  # the fp8 pass itself is what runs at the configs' sizes: e5m2 never re-runs;
        # e4m3 with its first-tile max at 2^2 re-runs ~16-19 % of the waves on random q / k (measured round 6; with the
        # max at 2^0 the underflow guard sent 92-100 % of them back)
        assert rerun < (0.05 if prec & 0xff in (4, 7) else 0.5), rerun
        report(f"fp8 re-run fraction prec {prec} S={S} N={N}: {rerun:.3f}")


@pytest.mark.parametrize("prec", [3, 4, 6, 7, 6 | QK_BF16, 7 | QK_BF16])
def test_item_attention_fp8_wide_score_spread(prec):
    """Scores spread wide (the ATT_SCALE = 2 situation of DESIGN 5.5, here x5): later key tiles overflow the first
    tile's fp8 scale for some queries, whose waves re-run on the exact bf16 path.  Every output (row, head) must be
    one of the two outcomes -- the quantised fp8 result or the exact softmax -- and the re-run must have happened."""
    S, N, T = 1200, 1000, 2
    q, k, v, Npad = _qkv_case(S, N, T, seed=77 + prec)
    q = q * 5.0
    got = _launch_layer(q, k, v, Npad, N, prec)
    assert torch.isfinite(got).all()
    err, rerun = _f8_outcomes(got, q, k, v, N, prec)
    print(f"wide spread prec {prec}: (row, head)s closer to the exact path {rerun:.3f}, worst {err.max():.3e}")
    assert err.max().item() < F8_QBAND * v.abs().max().item()
    assert rerun > 0.0


@pytest.mark.parametrize("prec", [3, 4, 6, 7, 6 | QK_BF16, 7 | QK_BF16])
@pytest.mark.parametrize("N", [1000, 10000])
def test_item_attention_fp8_underflow_guard(prec, N):
    """one large score in the (first-processed) partial key tile and every other key ~11 octaves
    lower.  e4m3 flushes those keys to 0 under the first tile's scale, losing most of the softmax mass; the row-sum
    guard (L < nk 2^(EMIN+6)) must send such waves to the exact path, so the output matches the exact softmax."""
    S, T = N + 64, 1
    q, k, v, Npad = _qkv_case(S, N, T, seed=N + prec)
    d = q.shape[-1]
    u = torch.ones(d) / math.sqrt(d)
    q[...] = u * 4.0                       # every query along u, |q| = 4
    k[...] = k * 0.01                      # ordinary keys: scores ~ 0
    k[:, :, N - 1] = u * 4.0 * 1.41        # the partial tile's last key: s = 16 * 1.41 * log2(e) / sqrt(32) ~ 5.75
    k[:, :, : N - 1] -= u * 10.6           # every other key ~ -11 log2 units: 2^-11 each, (N - 1) 2^-11 in total
    got = _launch_layer(q, k, v, Npad, N, prec).double()
    exact = _layer_ref(q, k, v, N, (5 | (prec & QK_BF16)) if prec & 0xff >= 5 else 1)
    qref = _f8_layer_ref(q, k, v, N, prec)
    err, lost = (got - exact).abs().max().item(), (qref - exact).abs().max().item()
    print(f"underflow guard prec {prec} N={N}: max err vs exact {err:.3e} (the flushed fp8 result: {lost:.3e})")
    assert torch.isfinite(got).all()
    if prec & 0xff in (3, 6):  # e4m3: the far keys flush under the first tile's scale; the guard must re-run the waves
        assert err < 2e-2
    else:  # e5m2 holds them (22 octaves below its scale): the quantised result stands
        assert (got - qref).abs().max().item() < F8_QBAND * v.abs().max().item()


@pytest.mark.parametrize("prec", [1, 0, 3, 4, 5, 5 | QK_BF16])
def test_item_attention_overflow_backstop(prec):
    """Scores that jump far past the first key tile's max (p would overflow the fixed
    softmax reference) take the exact two-pass recompute and still match."""
    S, N, T = 300, 260, 1
    q, k, v, Npad = _qkv_case(S, N, T, seed=5)
    q[..., :] = q[..., :].sign() * 0.2 + 2.0  # all queries point along +1
    k[:, :, 200:] = 6.0                       # late keys: scores ~ 2*6*32/sqrt(32) = 68 -> 2^98 over tile 0
    k[:, :, 230:] = 9.0                       # ... and beyond the fp32 range of exp2(s - m_tile0)
    got = _launch_layer(q, k, v, Npad, N, prec)
    ref = _layer_ref(q, k, v, N, prec)
    assert torch.isfinite(got).all()
    assert (got.double() - ref).abs().max().item() < ATTN_TOL[prec & 0xff]


@pytest.mark.parametrize("prec", [1, 0, 3, 4])
@pytest.mark.parametrize("kscale", [-5.0, 7.0])
def test_item_attention_reference_rerun(kscale, prec):
    """Row sums outside [2^-60, 2^100) under the reference-free first pass (every score ~82 log2
    units below zero, or ~114 above) make the block re-run with the first tile's max; queries of the
    same blocks with ordinary scores (the first 100 rows) come out of that re-run unchanged."""
    S, N, T = 400, 320, 2
    q, k, v, Npad = _qkv_case(S, N, T, seed=11)
    q[:, :, 100:] = q[:, :, 100:].sign() * 0.1 + 2.0
    k[...] = k * 0.05 + kscale
    got = _launch_layer(q, k, v, Npad, N, prec)
    ref = _layer_ref(q, k, v, N, prec)
    assert torch.isfinite(got).all()
    err = (got.double() - ref).abs().max().item()
    print(f"rerun kscale {kscale} prec {prec}: {err:.3e}")
    assert err < (1e-4 if prec == 0 else ATTN_TOL[prec])


@pytest.mark.parametrize("prec", [1, 3, 4])
@pytest.mark.parametrize("N", [20, 65, 1838])
@pytest.mark.parametrize("kscale", [-0.6, -0.7, -0.8, -0.9])
def test_item_attention_padded_tile_small_sums(kscale, N, prec):
    """The partial key tile runs in the pipelined loop with its padded keys at p = 1 and the row sums
    started at -npad (44, 63 or 18 padded keys here; N = 20: the partial tile is the only one); scores of
    about 16 kscale log2 units put the true sums around 2^-12 npad, on both sides of the threshold below
    which the wave takes the exact re-run."""
    S, T = N + 40, 1
    q, k, v, Npad = _qkv_case(S, N, T, seed=N + 3)
    q[...] = q.sign() * 0.1 + 2.0
    k[...] = k * 0.02 + kscale
    got = _launch_layer(q, k, v, Npad, N, prec)
    ref = _layer_ref(q, k, v, N, prec)
    assert torch.isfinite(got).all()
    err = (got.double() - ref).abs().max().item()
    print(f"padded tile N={N} kscale {kscale} prec {prec}: {err:.3e}")
    assert err < ATTN_TOL[prec]


def _launch_cached(q, k0, v0, Npad, N):
    """All queries of every head against a head-0-only K / V^T in the train-KV cache layout
    (mmpfn_item_attention_cached: the kernel's kv_bstride = Npad * 32 path)."""
    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.engine import HipEngine  # noqa: F401

    T, H, S, d = q.shape
    kp = torch.full((T, Npad, d), float("nan"))
    kp[:, :N] = k0
    vt = torch.full((T, d, Npad), float("nan"))
    vt[:, :, :N] = v0.transpose(-1, -2)
    lib = _lib.load_library()
    ctx = lib.mmpfn_create(0, None)
    qd, kd, vd = q.to("cuda", torch.bfloat16), kp.to("cuda", torch.bfloat16), vt.to("cuda", torch.bfloat16)
    out = torch.zeros(T, S, H * d, device="cuda", dtype=torch.bfloat16)
    assert lib.mmpfn_item_attention_cached(ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), out.data_ptr(), S, T, H,
                                           Npad, N) == 0
    torch.cuda.synchronize()
    lib.mmpfn_destroy(ctx)
    return out.float().cpu()


@pytest.mark.parametrize("N", [20, 1838])
@pytest.mark.parametrize("kscale", [0.0, -0.6, -0.7, -0.9])
def test_item_attention_cache_path_small_sums(kscale, N):
    """The train-KV cache's launch (head-0 K / V^T only, column stride Npad * 32, every query a test row)
    through the same partial-tile cancellation, on both sides of the 2^-12 npad re-run threshold
    (ADVICE r03); kscale 0 is an ordinary case."""
    S, T, H = 97, 3, 6
    q, k, v, Npad = _qkv_case(S, N, T, seed=N + 11)
    if kscale:
        q[...] = q.sign() * 0.1 + 2.0
        k[...] = k * 0.02 + kscale
    k0, v0 = k[:, 0], v[:, 0]
    got = _launch_cached(q, k0, v0, Npad, N)
    qr, kr, vr = (t.to(torch.bfloat16).float() for t in (q, k0, v0))
    ref = _attn_ref(qr, kr[:, None].expand(T, H, N, 32), vr[:, None].expand(T, H, N, 32))
    ref = ref.permute(0, 2, 1, 3).reshape(T, S, H * 32)
    assert torch.isfinite(got).all()
    err = (got.double() - ref).abs().max().item()
    print(f"cache path N={N} kscale {kscale}: {err:.3e}")
    assert err < 2e-2


def test_engine_deterministic_and_no_nan_at_pad_ufes_size():
    """Full config-C geometry (N=1838, Q=460, F=21, mgm 64 / cap 24): run twice, bitwise equal;
    bf16 vs fp32 engine argmax agreement (size-independent properties)."""
    from synth import synth_image, synth_labels, synth_state_dict, synth_table

    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(mgm_heads=64, cap_heads=24)
    sd = synth_state_dict(state_dict_spec(cfg), 2)
    model = make_model(cfg, sd)
    S, N = 2298, 1838
    x = torch.from_numpy(synth_table(S, 21, 2, n_cat=18))[:, None, :].cuda()
    im = torch.from_numpy(synth_image(S, 1, 2)).cuda()
    y = torch.from_numpy(synth_labels(S, 6, 2)[:N]).cuda()
    with torch.inference_mode():
        a = model(None, x, im, y, single_eval_pos=N).cpu()
        b = model(None, x, im, y, single_eval_pos=N).cpu()
        with torch.autocast("cuda"):
            c = model(None, x, im, y, single_eval_pos=N).cpu()
    assert torch.equal(a, b)
    assert torch.isfinite(c).all()
    check_argmax(c.squeeze(1).numpy(), a.squeeze(1).numpy(), 0.995, "config C bf16 vs fp32 engine")


@pytest.mark.parametrize("prec", [1, 5])
@pytest.mark.parametrize("lanes,batch", [(2, 1), (3, 1), (1, 2), (1, 5), (2, 2), (2, 3)])
def test_forward_lanes_match_sequential(lanes, batch, prec):
    """Members batched into one forward ([M][T][S][E] state) and/or on concurrent lanes (own
    workspace + stream each) == one member after another, bitwise."""
    from synth import synth_image, synth_labels, synth_state_dict, synth_table

    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(nlayers=3, mgm_heads=8, cap_heads=4)
    sd = synth_state_dict(state_dict_spec(cfg), 4)
    model = make_model(cfg, sd)
    eng = model.engine()
    S, N, F = 300, 230, 9
    x = synth_table(S, F, 4, n_cat=3)
    im = torch.from_numpy(synth_image(S, 1, 4)).cuda()
    y = synth_labels(S, 3, 4)[:N]
    tok = eng.mixer_tokens(im, _lib.PREC_BF16)
    rng = np.random.default_rng(1)
    items = []
    for m in range(5):
        xm = torch.from_numpy(np.ascontiguousarray(x[:, rng.permutation(F)]))
        ym = rng.permutation(3)[y.astype(np.int64)].astype(np.float32)
        items.append((xm, tok, ym))
    with torch.inference_mode():
        seq = eng.forward_many(items, prec, lanes=1, batch=1)
        par = eng.forward_many(items, prec, lanes=lanes, batch=batch)
        eng.status()
    for a, b in zip(seq, par):
        assert torch.equal(a.cpu(), b.cpu())


def test_forward_many_generator_of_fresh_device_tensors():
    """``predict_proba``'s call form: ``forward_many`` pulls a generator whose members are built on the
    caller's stream AFTER the lanes forked (torch.cat of the train and test rows, then the caller goes
    on allocating and writing).  Lanes must order behind each member's producer and keep its blocks
    alive until they have read them: lanes=2 == lanes=1, bitwise."""
    from synth import synth_image, synth_labels, synth_state_dict, synth_table

    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(nlayers=3, mgm_heads=8, cap_heads=4)
    sd = synth_state_dict(state_dict_spec(cfg), 5)
    model = make_model(cfg, sd)
    eng = model.engine()
    S, N, F = 1200, 900, 12
    x = synth_table(S, F, 5, n_cat=3)
    im = torch.from_numpy(synth_image(S, 1, 5)).cuda()
    y = synth_labels(S, 3, 5)[:N]
    tok = eng.mixer_tokens(im, _lib.PREC_BF16)
    perms = [np.random.default_rng(m).permutation(F) for m in range(6)]

    def gen():
        for p in perms:
            xp = torch.from_numpy(np.ascontiguousarray(x[:, p]))
            x_full = torch.cat([xp[:N].cuda(), xp[N:].cuda()], 0)  # made on the caller's stream
            yield x_full, tok, y
            del x_full
            junk = torch.empty((S, F), device="cuda").fill_(float("nan"))  # reuses freed blocks
            junk.mul_(2.0)

    with torch.inference_mode():
        ref = eng.forward_many(list(gen()), _lib.PREC_BF16, lanes=1, batch=1)
        torch.cuda.synchronize()
        for lanes, batch in [(2, 1), (2, 2)]:
            par = eng.forward_many(gen(), _lib.PREC_BF16, lanes=lanes, batch=batch)
            eng.status()
            for a, b in zip(ref, par):
                assert torch.equal(a.cpu(), b.cpu()), (lanes, batch)


def test_deepcopy_keeps_the_original_engine():
    """``deepcopy(model)`` shares the packed weights; re-loading weights into the copy must not close
    the original's engine (InferenceEngineCacheKV keeps one model copy per member)."""
    import copy

    z, meta, cfg, sd = load_case("pad_ufes_12l")
    model = make_model(cfg, sd)
    before = run_case(z, model)
    other = copy.deepcopy(model)
    assert run_case(z, other).tolist() == before.tolist()  # shared engine, same weights
    sd2 = {k: v * 0.5 if k.endswith("mlp.linear2.weight") else v for k, v in torch_sd(sd).items()}
    other.load_state_dict(sd2)
    changed = run_case(z, other)
    assert not np.array_equal(changed, before)
    np.testing.assert_array_equal(run_case(z, model), before)


def test_forward_batch_fp32_matches_reference():
    """fp32 parity mode through the batched forward (members stacked) against the goldens."""
    from multimodalpfn_amd import _lib

    z, meta, cfg, sd = load_case("pad_ufes_12l")
    model = make_model(cfg, sd)
    eng = model.engine()
    tok = eng.mixer_tokens(torch.from_numpy(z["image"]).cuda(), _lib.PREC_F32)
    item = (torch.from_numpy(z["x"]), tok, z["y_train"])
    with torch.inference_mode():
        outs = eng.forward_many([item, item, item], _lib.PREC_F32, lanes=1, batch=3)
    for o in outs:
        out = o.cpu().numpy()
        assert rel_err(out, z["logits"]) <= F32_TOL
        assert (out.argmax(1) == z["logits"].argmax(1)).all()


@pytest.mark.parametrize(
    "name,S,N,F,n_cls,seed",
    [("B: 4096 support x 100 features, tabular", 5120, 4096, 100, 2, 1),
     ("E: 10k support rows, long context", 12000, 10000, 20, 4, 4)],
)
def test_large_config_matches_oracle_on_device(name, S, N, F, n_cls, seed):
    """BASELINE configs B and E at full size, tabular-only, 12 layers: the fp32 engine against
    the oracle evaluated in fp32 on the same GPU (the checker's math moved to the device; it is
    pinned by the reference goldens on CPU), and the bf16 engine's labels against fp32."""
    from synth import synth_labels, synth_state_dict, synth_table

    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    torch.backends.cuda.matmul.allow_tf32 = False
    cfg = ModelConfig(mgm_heads=8, cap_heads=4)
    sd = synth_state_dict(state_dict_spec(cfg), seed)
    model = make_model(cfg, sd)
    x = torch.from_numpy(synth_table(S, F, seed, nan_frac=0.01)).cuda()
    y = torch.from_numpy(synth_labels(S, n_cls, seed)[:N]).cuda()
    from multimodalpfn_amd import _lib

    f8 = {}
    with torch.inference_mode():
        f32 = model(None, x[:, None, :], None, y, single_eval_pos=N).squeeze(1).float().cpu().numpy()
        b16 = model(None, x[:, None, :], None, y, single_eval_pos=N,
                    precision=_lib.PREC_BF16).squeeze(1).float().cpu().numpy()
        h16 = model(None, x[:, None, :], None, y, single_eval_pos=N,
                    precision=_lib.PREC_F16).squeeze(1).float().cpu().numpy()
        if name[0] == "E":  # config E's fp8 path: P.V + row sums on block-scaled fp8 MFMA
            for fmt, code in (("e4m3", _lib.PREC_BF16_F8), ("e5m2", _lib.PREC_BF16_F8E5), ("f16+e4m3", _lib.PREC_F16_F8)):
                f8[fmt] = model(None, x[:, None, :], None, y, single_eval_pos=N,
                                precision=code).squeeze(1).float().cpu().numpy()
    w = {k: v.cuda() for k, v in torch_sd(sd).items()}
    ref = oracle_forward(oracle_spec(cfg), w, x, None, y).cpu().numpy()
    del w
    torch.cuda.empty_cache()
    assert np.isfinite(f32).all() and np.isfinite(b16).all()
    assert rel_err(f32, ref) <= F32_TOL, (name, rel_err(f32, ref))
    assert (f32.argmax(1) == ref.argmax(1)).all()
    eb = rel_err(b16, ref)
    print(f"bf16 {name}: rel err {eb:.3e}; fp32 rel err {rel_err(f32, ref):.3e}")
    assert eb <= LARGE_BF16_TOL[name[0]], (name, eb)
    check_argmax(b16, ref, BF16_AGREE, f"bf16 {name}")
    eh = rel_err(h16, ref)
    print(f"f16 {name}: rel err {eh:.3e}, argmax agreement {float((h16.argmax(1) == ref.argmax(1)).mean()):.4f}")
    assert eh <= LARGE_F16_TOL[name[0]], (name, eh)
    check_argmax(h16, ref, BF16_AGREE, f"f16 {name}")
    for fmt, out in f8.items():
        e8 = rel_err(out, ref)
        agree = float((out.argmax(1) == ref.argmax(1)).mean())
        print(f"fp8 P.V ({fmt}) {name}: rel err {e8:.3e}, argmax agreement {agree:.4f}")
        assert np.isfinite(out).all()
        assert e8 <= F8_TOL, (name, fmt, e8)
        check_argmax(out, ref, BF16_AGREE, f"fp8 {fmt} {name}")


@pytest.mark.parametrize("prec", [0, 1, 5])
def test_train_kv_cache_equals_full_forward(prec):  # (0 parity, 1 bf16, 5 fp16)
    """mmpfn_cache_build (train rows once) + mmpfn_cache_predict (test rows only) == the test
    rows of one full forward, bitwise (every kernel computes a row independently of the others;
    the encoders' statistics come from the train rows in both)."""
    from synth import synth_image, synth_labels, synth_state_dict, synth_table

    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(nlayers=4, mgm_heads=8, cap_heads=4)
    sd = synth_state_dict(state_dict_spec(cfg), 6)
    model = make_model(cfg, sd)
    eng = model.engine()
    S, N, F = 520, 400, 11
    x = torch.from_numpy(synth_table(S, F, 6, n_cat=4, nan_frac=0.02)).cuda()
    im = torch.from_numpy(synth_image(S, 1, 6)).cuda()
    y = synth_labels(S, 4, 6)[:N]
    with torch.inference_mode():
        tok = eng.mixer_tokens(im, prec)
        full = eng.forward(x, tok, y, prec)
        cache = eng.cache_build(x[:N], tok[:N], y, prec)
        T = (F + 1) // 2 + tok.shape[1] + 1
        assert cache.nbytes >= cfg.nlayers * 2 * T * 448 * 32 * (2 if prec else 4)  # head-0 K + V^T per layer
        a = eng.cache_predict(cache, x[N:], tok[N:])
        b = eng.cache_predict(cache, x[N:N + 37], tok[N:N + 37])  # any test batch size
        eng.status()
        cache.free()
    assert torch.equal(a, full)
    assert torch.equal(b, full[:37])


@pytest.mark.parametrize("mixer,mgm,cap,S", [("MGM+CAP", 64, 24, 300), ("MGM+CAP", 8, 4, 777), ("MGM", 16, 2, 513)])
def test_mixer_bf16_matches_fp32(mixer, mgm, cap, S):
    """bf16 mixer path (large-tile DMA-ring GLU GEMM for the MGM head bank, fused k_norm + K|V
    projection, CAP attention on bf16 keys) against the fp32 parity path on the same weights and
    image rows, row counts that leave partial 256-row tiles; bf16 tolerance 3e-2 relative."""
    from synth import synth_image, synth_state_dict

    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(nlayers=1, mixer_type=mixer, mgm_heads=mgm, cap_heads=cap)
    sd = synth_state_dict(state_dict_spec(cfg), 9)
    eng = make_model(cfg, sd).engine()
    im = torch.from_numpy(synth_image(S, 1, 9)).cuda()
    with torch.inference_mode():
        ref = eng.mixer_tokens(im, _lib.PREC_F32)
        got = eng.mixer_tokens(im, _lib.PREC_BF16)
        eng.status()
    assert got.shape == ref.shape
    assert torch.isfinite(got).all()
    err = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
    assert err < 3e-2, err


@pytest.mark.parametrize("mixer,mgm,cap,S,n_mod", [("MGM+CAP", 64, 24, 300, 1), ("MGM+CAP", 64, 24, 97, 2),
                                                   ("MGM+CAP", 8, 4, 777, 1), ("MGM", 16, 2, 513, 1)])
def test_mixer_f16_head_bank(mixer, mgm, cap, S, n_mod):
    """PREC_F16's mixer: the MGM head bank on fp16 operands (LN output, GLU hidden, weights; the same big-tile
    kernels in their f16 form), the pooler from an fp16 token read on in the bf16 mode.  Against the fp32 parity
    path: the head bank alone (MGM tokens) must sit well inside the bf16 mode's error (fp16 keeps 3 more mantissa
    bits; measured ~7x on the golden cases), and the whole mixer no worse than the bf16 mode."""
    from synth import synth_image, synth_state_dict

    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(nlayers=1, mixer_type=mixer, mgm_heads=mgm, cap_heads=cap)
    sd = synth_state_dict(state_dict_spec(cfg), 11)
    eng = make_model(cfg, sd).engine()
    im = torch.from_numpy(synth_image(S, n_mod, 11)).cuda()

    def rel(a, b):
        return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-6)

    with torch.inference_mode():
        m32, m16, mbf = (eng.mgm(im, p) for p in (_lib.PREC_F32, _lib.PREC_F16, _lib.PREC_BF16))
        t32, t16, tbf = (eng.mixer_tokens(im, p) for p in (_lib.PREC_F32, _lib.PREC_F16, _lib.PREC_BF16))
        eng.status()
    assert torch.isfinite(m16).all() and torch.isfinite(t16).all()
    e16, ebf = rel(m16, m32), rel(mbf, m32)
    print(f"{mixer} mgm {mgm} n_mod {n_mod}: MGM tokens f16 {e16:.2e} bf16 {ebf:.2e}; "
          f"mixer f16 {rel(t16, t32):.2e} bf16 {rel(tbf, t32):.2e}")
    assert e16 < 2e-3 and e16 < 0.5 * ebf, (e16, ebf)
    assert rel(t16, t32) <= 1.1 * rel(tbf, t32) + 1e-4


def test_item_attention_entry_rejects_16bit_and_fp8_codes():
    """``mmpfn_item_attention`` runs the bf16 and the two fp32 element forms only: the fp16 Q / K and
    fp8 P.V codes 3-7 belong to ``mmpfn_item_attention_layer_ex`` and must be refused, not run on the fp32 kernel."""
    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.engine import HipEngine  # noqa: F401

    lib = _lib.load_library()
    ctx = lib.mmpfn_create(0, None)
    S, N, T, H, d, Npad = 70, 40, 1, 6, 32, 64
    q = torch.zeros(T, H, S, d, device="cuda", dtype=torch.float32)
    k = torch.zeros(T, H, Npad, d, device="cuda", dtype=torch.float32)
    vt = torch.zeros(T, H, d, Npad, device="cuda", dtype=torch.float32)
    out = torch.full((T, S, H * d), 7.0, device="cuda", dtype=torch.float32)
    try:
        for code in (3, 4, 5, 6, 7, 8, -1):
            rc = lib.mmpfn_item_attention(ctx, q.data_ptr(), k.data_ptr(), vt.data_ptr(), out.data_ptr(), S, T, H,
                                          Npad, 0, N, N, -1, code)
            assert rc == _lib.MMPFN_ERR_INVALID, (code, rc)
        torch.cuda.synchronize()
        assert (out == 7.0).all()  # nothing ran
        assert lib.mmpfn_item_attention(ctx, q.data_ptr(), k.data_ptr(), vt.data_ptr(), out.data_ptr(), S, T, H,
                                        Npad, 0, N, N, -1, _lib.PREC_F32) == 0
        torch.cuda.synchronize()
    finally:
        lib.mmpfn_destroy(ctx)


def test_f16_falls_back_to_bf16_on_wide_tables():
    """PREC_F16's layer kernels hold at most 64 tokens per row; wider tables run the bf16 mode.  The
    forward, the train-KV cache and every sublayer tap apply the same rule (capi.cpp f16_fits), so PREC_F16 equals
    PREC_BF16 bitwise there: 140 features = 71 tokens per row.  (The engine is specialised for E = 192 in 6 heads;
    mmpfn_set_model refuses other widths.)"""
    from synth import synth_labels, synth_state_dict, synth_table

    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    cfg = ModelConfig(nlayers=2, mgm_heads=8, cap_heads=4)
    sd = synth_state_dict(state_dict_spec(cfg), 21)
    model = make_model(cfg, sd)
    eng = model.engine()
    S, N, F = 260, 200, 140
    x = torch.from_numpy(synth_table(S, F, 21, n_cat=2)).cuda()
    y = synth_labels(S, 3, 21)[:N]
    with torch.inference_mode():
        h = eng.forward(x, None, y, _lib.PREC_F16)
        b = eng.forward(x, None, y, _lib.PREC_BF16)
        eng.status()
        assert torch.isfinite(h).all()
        assert torch.equal(h, b)
        ch, cb = eng.cache_build(x[:N], None, y, _lib.PREC_F16), eng.cache_build(x[:N], None, y, _lib.PREC_BF16)
        ph, pb = eng.cache_predict(ch, x[N:], None), eng.cache_predict(cb, x[N:], None)
        ch.free()
        cb.free()
        assert torch.equal(ph, pb)
        assert torch.equal(ph, h)
        X = eng.embed_state(x, None, y, _lib.PREC_F32)
        assert X.shape[1] > 64
        assert torch.equal(eng.feature_attention(0, X, _lib.PREC_F16), eng.feature_attention(0, X, _lib.PREC_BF16))
        assert torch.equal(eng.item_attention_block(0, X, N, _lib.PREC_F16),
                           eng.item_attention_block(0, X, N, _lib.PREC_BF16))


F16_CASES = sorted(p.stem for p in (GOLDEN / "f16").glob("*.npz"))
F16_REF_FACTOR = 3.0  # the fp16 mode's deviation from the fp32 reference <= 3x the reference's own fp16 deviation
# (measured 0.60-2.72x over the nine fixtures: MGM head bank on fp16 operands, item Q / K in bf16; 0.68-2.16x with fp16
# item Q / K; 3.17x at image_only while the head bank ran on bf16 operands)


def _load_f16_case(name):
    """tests/golden/f16/<name>.npz (make_f16_golden.py: the reference forward under its fp16 autocast) with the
    case's inputs, config and synthetic weights (from the make_golden file of the same name, or its own)."""
    import json

    from synth import synth_state_dict

    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec

    f = np.load(GOLDEN / "f16" / f"{name}.npz")
    z = np.load(GOLDEN / f"{name}.npz") if (GOLDEN / f"{name}.npz").exists() else f
    meta = json.loads(str(z["meta"]))
    cfg = ModelConfig(**meta["cfg"])
    return f, z, cfg, synth_state_dict(state_dict_spec(cfg), meta["wseed"])


@pytest.mark.parametrize("case", F16_CASES)
def test_f16_mode_within_reference_fp16_deviation(case):
    """The fp16 mode against the reference's OWN fp16 autocast arithmetic (VERDICT r04 missing #2): three numbers
    per case -- engine-fp16 vs reference-fp16, engine-fp16 vs reference-fp32, reference-fp16 vs reference-fp32 --
    and the band is the reference's own deviation: the engine's fp16 logits may move from the fp32 reference by at
    most F16_REF_FACTOR x what the reference's fp16 run moves (argmax agreement with both >= 0.995)."""
    from multimodalpfn_amd import _lib

    f, z, cfg, sd = _load_f16_case(case)
    out = run_case(z, make_model(cfg, sd), precision=_lib.PREC_F16)
    r16, r32 = f["logits_f16"], f["logits_f32"]
    e_ours32, e_ours16, e_ref = rel_err(out, r32), rel_err(out, r16), rel_err(r16, r32)
    report(f"F16REF {case}: engine-f16 vs ref-f16 {e_ours16:.3e}, engine-f16 vs ref-f32 {e_ours32:.3e}, "
           f"ref-f16 vs ref-f32 {e_ref:.3e} (ratio {e_ours32 / e_ref:.2f}, band {F16_REF_FACTOR:g})")
    assert np.isfinite(out).all()
    assert e_ours32 <= F16_REF_FACTOR * e_ref, (case, e_ours32, e_ref)
    check_argmax(out, r32, BF16_AGREE, f"f16 vs ref-f32 {case}")
    check_argmax(out, r16, BF16_AGREE, f"f16 vs ref-f16 {case}")

