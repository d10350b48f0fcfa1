"""CPU restatement of the MMPFN ``PerFeatureTransformer`` forward (TEST INFRASTRUCTURE).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may use this module.  It is never part of the product path.

Every function cites the reference code it restates (paths relative to
``/root/reference``; ``T/`` = ``mmpfn/models/mmpfn/model/``):

* input grouping / y padding ........ ``T/transformer.py:626-718``
* x encoder steps ................... ``T/loading.py:308-371`` + ``T/encoders.py``
* y encoder ......................... ``T/loading.py:374-398``, ``T/encoders.py:428-493,949-974``
* MGM / CAP / MoE mixers ............ ``T/transformer.py:33-128,755-761``
* token append + subspace pos-emb ... ``T/transformer.py:765-788,925-933,1003-1039``
* 12-layer stack .................... ``T/transformer.py:154-179``, ``T/layer.py:272-457``
* multi-head attention .............. ``T/multi_head_attention.py:371-517,547-736``
* MLP ............................... ``T/mlp.py:93-138``
* decoder ........................... ``T/transformer.py:388-403,850-853``

The dead debug correlation loop (``T/transformer.py:810-813``) has no effect on
the outputs and is omitted.

All math is plain torch on CPU in ``dtype`` (float32 by default, float64 for
tight pinning).  Weights are passed as a flat dict keyed by the reference's
``state_dict`` names (checkpoint ABI).
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

NAN_INDICATOR = -2.0  # T/encoders.py:431
POS_INF_INDICATOR = 2.0  # T/encoders.py:432
NEG_INF_INDICATOR = 4.0  # T/encoders.py:433


@dataclass
class OracleSpec:
    """Model hyper-parameters (reference ``InferenceConfig`` + mixer args)."""

    emsize: int = 192
    nhead: int = 6
    nlayers: int = 12
    nhid: int = 768
    features_per_group: int = 2  # model grouping (PerFeatureTransformer arg)
    encoder_features: int = 2  # checkpoint config.features_per_group (get_encoder num_features)
    n_out: int = 10
    mixer_type: str = "MGM+CAP"  # "MGM", "MGM+CAP", "MoE"
    mgm_heads: int = 64
    cap_heads: int = 24
    remove_outliers_sigma: float | None = 12.0  # utils.py:703-745, constants.py:181
    model_seed: int = 0  # PerFeatureTransformer(seed=...) T/transformer.py:413,421-424
    two_sets_of_queries: bool = False
    ln_eps: float = 1e-5


# --------------------------------------------------------------------------------------
# reductions with the reference's NaN semantics (T/encoders.py:17-50)
# --------------------------------------------------------------------------------------


def _nanmean_clip(x: torch.Tensor) -> torch.Tensor:
    """``torch_nanmean`` (T/encoders.py:17-34): sum of non-NaN / max(count, 1)."""
    m = torch.isnan(x)
    num = (~m).to(x.dtype).sum(0)
    val = torch.where(m, torch.zeros_like(x), x).sum(0)
    return val / num.clip(min=1.0)


def _nanstd(x: torch.Tensor) -> torch.Tensor:
    """``torch_nanstd`` (T/encoders.py:37-50): unbiased, mean NOT clipped."""
    m = torch.isnan(x)
    num = (~m).to(x.dtype).sum(0)
    val = torch.where(m, torch.zeros_like(x), x).sum(0)
    mean = val / num
    return torch.sqrt(torch.nansum((mean.unsqueeze(0) - x) ** 2, dim=0) / (num - 1))


# --------------------------------------------------------------------------------------
# encoders
# --------------------------------------------------------------------------------------


def encode_x(spec: OracleSpec, w: dict, x: torch.Tensor, n_train: int) -> torch.Tensor:
    """x encoder: ``[S, F]`` -> ``[S, G, E]``.

    Steps (``get_encoder`` T/loading.py:308-371):
      0 RemoveEmptyFeatures (T/encoders.py:496-527; constancy over ALL rows)
      1 NanHandling keep_nans (T/encoders.py:428-493; train nanmean fill)
      2 VariableNumFeatures on nan indicators, no rescale (T/encoders.py:579-655)
      3 InputNormalization: 12-sigma soft outlier clip + train-stat z-score, clip +-100
        (T/encoders.py:133-162, 53-99, 658-782)
      4 VariableNumFeatures(main): x * sqrt(nf / used), zero-pad to nf (T/encoders.py:608-655)
      5 Linear(2*nf -> E, bias=False) on cat(main, nan_ind) (T/encoders.py:382-425)

    ``nf`` is the encoder width (checkpoint ``config.features_per_group``,
    T/loading.py:473-475); ``fpg`` is the model's grouping (yaml
    ``features_per_group``), which may be smaller (salary: 1).
    """
    S, Fdim = x.shape
    fpg = spec.features_per_group
    pad = (fpg - Fdim % fpg) % fpg  # T/transformer.py:630-648
    if pad:
        x = torch.cat([x, torch.zeros(S, pad, dtype=x.dtype, device=x.device)], 1)
    G = x.shape[1] // fpg
    x = x.reshape(S, G, fpg)  # "s b (f n) -> s (b f) n" with b=1 (T/transformer.py:652-657,742)

    # 0: remove constant features, left-compacted per group, zero-filled
    sel = (x[1:] == x[0:1]).sum(0) != (S - 1)  # [G, fpg]  (T/encoders.py:515)
    xc = torch.zeros_like(x)
    for g in range(G):
        idx = torch.nonzero(sel[g]).flatten()
        if idx.numel():
            xc[:, g, : idx.numel()] = x[:, g, idx]
    x = xc

    # 1: NaN handling (feature means on train rows, torch.nanmean; T/encoders.py:461)
    means = torch.nanmean(x[:n_train], dim=0)
    isinf = torch.isinf(x)
    ind = (
        torch.isnan(x).to(x.dtype) * NAN_INDICATOR
        + (isinf & (torch.sign(x) == 1)).to(x.dtype) * POS_INF_INDICATOR
        + (isinf & (torch.sign(x) == -1)).to(x.dtype) * NEG_INF_INDICATOR
    )
    bad = torch.isnan(x) | isinf
    x = torch.where(bad, means.unsqueeze(0).expand_as(x), x)

    # 3: input normalization on train rows
    if spec.remove_outliers_sigma is not None:
        n_sigma = spec.remove_outliers_sigma
        data = x[:n_train]
        m, sd = _nanmean_clip(data), _nanstd(data)
        lo, hi = m - sd * n_sigma, m + sd * n_sigma
        clean = torch.where((data > hi) | (data < lo), torch.full_like(data, float("nan")), data)
        m, sd = _nanmean_clip(clean), _nanstd(clean)
        lo, hi = m - sd * n_sigma, m + sd * n_sigma
        x = torch.maximum(-torch.log(1 + torch.abs(x)) + lo, x)
        x = torch.minimum(torch.log(1 + torch.abs(x)) + hi, x)
    mean = _nanmean_clip(x[:n_train])
    std = _nanstd(x[:n_train]) + 1e-20
    if S == 1 or n_train == 1:
        std = torch.ones_like(std)
    x = torch.clip((x - mean) / std, min=-100, max=100)

    # 4: rescale by the number of used (non-constant) features per group
    sel2 = (x[1:] == x[0:1]).sum(0) != (S - 1)  # [G, fpg]
    used = torch.clip(sel2.sum(-1, keepdim=True), min=1).to(x.dtype)  # [G, 1]
    nf = spec.encoder_features
    x = x * torch.sqrt(nf / used)
    if nf > fpg:  # VariableNumFeatures zero-padding of main and nan indicators
        zp = torch.zeros(S, G, nf - fpg, dtype=x.dtype, device=x.device)
        x = torch.cat([x, zp], -1)
        ind = torch.cat([ind, zp], -1)

    # 5: linear embed
    feats = torch.cat([x, ind], dim=-1)  # [S, G, 2*nf]
    W = w["encoder.5.layer.weight"] if "encoder.5.layer.weight" in w else w["encoder.6.layer.weight"]
    return feats @ W.to(x.dtype).T


def encode_y(spec: OracleSpec, w: dict, y_train: torch.Tensor, S: int) -> torch.Tensor:
    """y encoder: ``[N]`` -> ``[S, E]`` (T/loading.py:374-398).

    NaN-pad test rows (T/transformer.py:682-718), NanHandling (fill with train
    mean, indicator -2), class-index target encoding ``(y > unique_train).sum()``
    (T/encoders.py:954-974), Linear(2 -> E, bias).
    """
    N = y_train.shape[0]
    y = torch.full((S,), float("nan"), dtype=y_train.dtype, device=y_train.device)
    y[:N] = y_train
    mean = torch.nanmean(y[:N])
    ind = torch.isnan(y).to(y.dtype) * NAN_INDICATOR
    y = torch.where(torch.isnan(y), mean, y)
    uniq = torch.unique(y[:N])
    yc = (y.unsqueeze(-1) > uniq).sum(-1).to(y.dtype)
    feats = torch.stack([yc, ind], -1)
    W = w["y_encoder.2.layer.weight"].to(y.dtype)
    b = w["y_encoder.2.layer.bias"].to(y.dtype)
    return feats @ W.T + b


# --------------------------------------------------------------------------------------
# mixers (image / text projection heads)
# --------------------------------------------------------------------------------------


def _ln_affine(x, wgt, bias, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), wgt, bias, eps)


def _linear(x, w, pre, bias=True):
    y = x @ w[pre + ".weight"].to(x.dtype).T
    if bias:
        y = y + w[pre + ".bias"].to(x.dtype)
    return y


def oracle_mixer(spec: OracleSpec, w: dict, image: torch.Tensor) -> torch.Tensor:
    """Image/text projection heads: ``[S, n_mod, 768]`` -> ``[S, C, E]``.

    MGM (T/transformer.py:33-48): per head ``LN(768)->Linear(768,768)->GLU->Linear(384,E)``,
    heads concatenated head-major on the token axis.
    CAP (T/transformer.py:60-88): learned queries cross-attend the MGM tokens with
    ``nn.MultiheadAttention(E, cap_heads)``; ``out_norm(out) + ffn(out)``.
    MoE (T/transformer.py:91-128): modality 0 only, softmax gate (top_k >= n_experts
    so no masking, T/transformer.py:301), gate-weighted expert outputs as tokens.
    """
    dt = image.dtype
    S = image.shape[0]
    if spec.mixer_type == "MoE":
        x = image[:, 0]  # T/transformer.py:109 (x[0,:,0] after unsqueeze(0))
        probs = torch.softmax(_linear(x, w, "moe.gate"), dim=-1)
        n_exp = probs.shape[-1]
        top_k = max(spec.mgm_heads, spec.cap_heads)
        assert top_k >= n_exp, "top-k masking path not exercised by the reference config"
        outs = []
        for i in range(n_exp):
            p = f"moe.experts.{i}"
            h = _ln_affine(x, w[p + ".0.weight"].to(dt), w[p + ".0.bias"].to(dt))
            h = F.gelu(_linear(h, w, p + ".1"))
            h = _linear(h, w, p + ".4")
            outs.append((probs[:, i : i + 1] * h).unsqueeze(-2))
        return torch.cat(outs, dim=-2)

    tok = oracle_mgm(spec, w, image)
    if spec.mixer_type == "MGM":
        return tok
    assert spec.mixer_type == "MGM+CAP"
    return oracle_cap(spec, w, tok)


def oracle_mgm(spec: OracleSpec, w: dict, image: torch.Tensor) -> torch.Tensor:
    """MultiheadGatedMLP (T/transformer.py:33-57): ``[S, n_mod, 768]`` -> ``[S, mgm*n_mod, E]``."""
    dt = image.dtype
    outs = []
    for hh in range(spec.mgm_heads):
        p = f"mgm.projs.{hh}"
        h = _ln_affine(image, w[p + ".0.weight"].to(dt), w[p + ".0.bias"].to(dt))
        h = _linear(h, w, p + ".1")
        a, b = h.chunk(2, dim=-1)
        h = a * torch.sigmoid(b)  # nn.GLU
        outs.append(_linear(h, w, p + ".4"))
    return torch.cat(outs, dim=-2)  # [S, mgm*n_mod, E]


def oracle_cap(spec: OracleSpec, w: dict, tok: torch.Tensor) -> torch.Tensor:
    """CrossAttentionPooler (T/transformer.py:60-88): MGM tokens ``[S, M, E]`` -> ``[S, cap, E]``."""
    dt = tok.dtype
    S = tok.shape[0]
    E = spec.emsize
    nh = spec.cap_heads
    hd = E // nh
    src = _ln_affine(tok, w["cap.k_norm.weight"].to(dt), w["cap.k_norm.bias"].to(dt))
    qn = _ln_affine(w["cap.queries"].to(dt), w["cap.q_norm.weight"].to(dt), w["cap.q_norm.bias"].to(dt))
    q = qn @ w["cap.q_proj.weight"].to(dt).T  # [cap, E]
    W_in = w["cap.mha.in_proj_weight"].to(dt)
    b_in = w["cap.mha.in_proj_bias"].to(dt)
    qp = q @ W_in[:E].T + b_in[:E]  # [cap, E]
    kp = src @ W_in[E : 2 * E].T + b_in[E : 2 * E]  # [S, M, E]
    vp = src @ W_in[2 * E :].T + b_in[2 * E :]
    cap = q.shape[0]
    M = src.shape[1]
    qh = qp.reshape(cap, nh, hd).permute(1, 0, 2)  # [nh, cap, hd]
    kh = kp.reshape(S, M, nh, hd).permute(0, 2, 1, 3)  # [S, nh, M, hd]
    vh = vp.reshape(S, M, nh, hd).permute(0, 2, 1, 3)
    att = torch.softmax((qh.unsqueeze(0) @ kh.transpose(-1, -2)) / math.sqrt(hd), dim=-1)
    o = (att @ vh).permute(0, 2, 1, 3).reshape(S, cap, E)
    o = _linear(o, w, "cap.mha.out_proj")
    ffn = _linear(F.gelu(_linear(o, w, "cap.ffn.0")), w, "cap.ffn.3")
    return _ln_affine(o, w["cap.out_norm.weight"].to(dt), w["cap.out_norm.bias"].to(dt)) + ffn


def subspace_pos_emb(spec: OracleSpec, w: dict, n_tokens: int, dtype) -> torch.Tensor:
    """Feature positional embedding "subspace" (T/transformer.py:421-424,925-933).

    A fresh CPU generator (default seed unless ``model_seed`` is truthy) draws
    ``randn(n_tokens, E//4)`` which is mapped by ``Linear(E//4 -> E)``.
    """
    gen = torch.Generator(device="cpu")
    if spec.model_seed:
        gen.manual_seed(spec.model_seed)
    r = torch.randn((n_tokens, spec.emsize // 4), generator=gen, dtype=torch.float32)
    r = r.to(dtype=dtype, device=w["feature_positional_embedding_embeddings.weight"].device)
    return _linear(r, w, "feature_positional_embedding_embeddings")


# --------------------------------------------------------------------------------------
# layer stack
# --------------------------------------------------------------------------------------


def _attn(q, k, v, use_sdpa=False):
    """softmax(q k^T / sqrt(d)) v over the last two axes (T/multi_head_attention.py:718-729)."""
    if use_sdpa:
        return F.scaled_dot_product_attention(q, k, v)
    d = q.shape[-1]
    logits = (q @ k.transpose(-1, -2)) * math.sqrt(1.0 / d)
    return torch.softmax(logits, dim=-1) @ v


def _ln(x, eps):
    return F.layer_norm(x, (x.shape[-1],), None, None, eps)


def feat_sublayer(spec: OracleSpec, w: dict, l: int, X: torch.Tensor, use_sdpa=False):
    """Attention between features + residual + LN (T/layer.py:332-339,437-455); ``X`` ``[S, T, E]``."""
    dt = X.dtype
    p = f"transformer_encoder.layers.{l}"
    wqkv = w[p + ".self_attn_between_features._w_qkv"].to(dt)  # [3, H, d, E] (T/multi_head_attention.py:423-430)
    wout = w[p + ".self_attn_between_features._w_out"].to(dt)  # [H, d, E]
    qkv = torch.einsum("ste,jhde->sjhtd", X, wqkv)  # [S, 3, H, T, d]
    o = _attn(qkv[:, 0], qkv[:, 1], qkv[:, 2], use_sdpa)  # [S, H, T, d]
    o = torch.einsum("shtd,hde->ste", o, wout)
    return _ln(X + o, spec.ln_eps)


def item_sublayer(spec: OracleSpec, w: dict, l: int, X: torch.Tensor, n_train: int, use_sdpa=False):
    """Attention between items + residual + LN (T/layer.py:341-379,437-455), per token column:
    train rows on all KV heads, test rows on head 0's K/V broadcast (reuse_first_head_kv)."""
    S = X.shape[0]
    dt = X.dtype
    pi = f"transformer_encoder.layers.{l}.self_attn_between_items"
    if spec.two_sets_of_queries:
        wq_all = w[pi + "._w_q"].to(dt)  # [2, H, d, E]
        wq_tr, wq_te = wq_all[0], wq_all[1]
        wkv = w[pi + "._w_kv"].to(dt)  # [2, H, d, E]
    else:
        wqkv = w[pi + "._w_qkv"].to(dt)
        wq_tr = wq_te = wqkv[0]
        wkv = wqkv[1:]
    wout = w[pi + "._w_out"].to(dt)
    Xc = X.transpose(0, 1)  # [T, S, E]
    Xtr = Xc[:, :n_train]
    k = torch.einsum("tne,hde->thnd", Xtr, wkv[0])  # [T, H, N, d]
    v = torch.einsum("tne,hde->thnd", Xtr, wkv[1])
    outs = []
    if n_train > 0:
        q = torch.einsum("tne,hde->thnd", Xtr, wq_tr)
        outs.append(_attn(q, k, v, use_sdpa))  # train rows: all 6 KV heads
    if n_train < S:
        q = torch.einsum("tne,hde->thnd", Xc[:, n_train:], wq_te)
        k0 = k[:, :1].expand_as(k)  # test rows: head-0 K/V broadcast (reuse_first_head_kv)
        v0 = v[:, :1].expand_as(v)
        outs.append(_attn(q, k0, v0, use_sdpa))
    o = torch.cat(outs, dim=2)  # [T, H, S, d]
    o = torch.einsum("thsd,hde->ste", o, wout)
    return _ln(X + o, spec.ln_eps)


def mlp_sublayer(spec: OracleSpec, w: dict, l: int, X: torch.Tensor):
    """MLP (T/mlp.py:93-104): Linear(no bias) -> GELU(erf) -> Linear(no bias), residual, LN."""
    dt = X.dtype
    p = f"transformer_encoder.layers.{l}"
    h = F.gelu(X @ w[p + ".mlp.linear1.weight"].to(dt).T)
    return _ln(X + h @ w[p + ".mlp.linear2.weight"].to(dt).T, spec.ln_eps)


def layer_forward(spec: OracleSpec, w: dict, l: int, X: torch.Tensor, n_train: int, use_sdpa=False):
    """One ``PerFeatureEncoderLayer`` (post-norm; T/layer.py:272-457).

    ``X``: ``[S, T, E]``.  feature-attn -> LN -> item-attn -> LN -> MLP -> LN.
    """
    X = feat_sublayer(spec, w, l, X, use_sdpa)
    X = item_sublayer(spec, w, l, X, n_train, use_sdpa)
    return mlp_sublayer(spec, w, l, X)


def embed_inputs(spec, w, x, image, y_train, dtype=torch.float32, mixer_tokens=None):
    """Build the transformer input ``[S, T, E]`` (T/transformer.py:586-797)."""
    N = y_train.shape[0]
    S = x.shape[0] if x is not None else image.shape[0]
    parts = []
    if x is not None:
        parts.append(encode_x(spec, w, x.to(dtype), N))
    if image is not None:
        if mixer_tokens is None:
            mixer_tokens = oracle_mixer(spec, w, image.to(dtype))
        parts.append(mixer_tokens.to(dtype))
    tok = torch.cat(parts, dim=1)  # token_append (T/transformer.py:1038)
    tok = tok + subspace_pos_emb(spec, w, tok.shape[1], dtype).unsqueeze(0)
    ytok = encode_y(spec, w, y_train.to(dtype), S)
    X = torch.cat([tok, ytok.unsqueeze(1)], dim=1)
    if torch.isnan(X).any():  # T/transformer.py:790-796
        raise ValueError("There should be no NaNs in the encoded x and y.")
    return X


@torch.inference_mode()
def oracle_forward(
    spec: OracleSpec,
    w: dict,
    x: torch.Tensor | None,
    image: torch.Tensor | None,
    y_train: torch.Tensor,
    *,
    dtype=torch.float32,
    use_sdpa: bool = False,
    taps: dict | None = None,
    mixer_tokens: torch.Tensor | None = None,
) -> torch.Tensor:
    """Full forward of one ensemble member: returns logits ``[Q, n_out]``.

    Mirrors ``model(None, X_full[S,1,F], image_full[S,n_mod,768], y_train[N],
    single_eval_pos=N)`` at ``T/../inference.py:343-348``.
    """
    N = y_train.shape[0]
    X = embed_inputs(spec, w, x, image, y_train, dtype, mixer_tokens)
    if taps is not None:
        taps["embedded_input"] = X.clone()
    for l in range(spec.nlayers):
        X = layer_forward(spec, w, l, X, N, use_sdpa)
        if taps is not None:
            taps[f"layer{l}"] = X.clone()
    h = X[N:, -1]  # test rows of the target token (T/transformer.py:850)
    h = F.gelu(_linear(h, w, "decoder_dict.standard.0"))
    return _linear(h, w, "decoder_dict.standard.2")
