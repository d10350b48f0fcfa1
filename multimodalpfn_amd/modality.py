"""Modality encoders on the device: the towers that turn raw images and texts
into the ``image [S, n_mod, 768]`` tokens the MMPFN path consumes.

The reference computes these embeddings once per dataset and caches them as ``.pt`` files:

* image -- DINOv2 ViT-B/14, ``vit_base(patch_size=14, img_size=518, init_values=1.0,
  num_register_tokens=0, block_chunks=0).forward_features(batch)["x_norm_clstoken"]``
  (``mmpfn/datasets/pad_ufes_20.py:66-107``, ``petfinder.py:100-146``; the model in
  ``mmpfn/models/dino_v2/models/vision_transformer.py``);
* text -- ELECTRA-base, ``AutoModel.from_pretrained("google/electra-base-discriminator")
  (**tokenizer(text, truncation=True, max_length=512)).last_hidden_state[:, 0, :]``
  (``petfinder.py:150-181``; transformers' ``ElectraModel``).

Here both run in ``libmmpfn_hip.so`` (``include/mmpfn_modality.h``): bf16 MFMA GEMMs on 256 x 256
tiles fed by an LDS-DMA ring, a head-dim-64 flash attention, fused LayerNorm / LayerScale /
residual epilogues; ``precision="f32"`` runs the reference's fp32 arithmetic.  The modules below
are parameter containers with the reference's state-dict names (so ``load_state_dict`` of the
reference checkpoints works unchanged); their forward methods move pointers only.  Without a ROCm
GPU they raise -- there is no CPU compute path.  The pretrained weights and the WordPiece
vocabulary are not available offline: parity is pinned with seeded random weights against the
reference's own ``vit_base`` and transformers' ``ElectraModel`` (``tests/golden/make_modality_golden.py``),
and the text tower takes token ids (``input_ids`` / ``attention_mask`` / ``token_type_ids``, what the
reference's tokenizer returns).
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Any

import numpy as np
import torch
from torch import nn

from multimodalpfn_amd import _lib

__all__ = [
    "DinoVisionTransformer",
    "vit_base",
    "ElectraConfigLite",
    "ElectraTextEncoder",
    "embed_images",
    "embed_texts",
]


def _precision(precision: str, device: torch.device) -> int:
    if precision == "bf16":
        return _lib.PREC_BF16
    if precision == "f32":
        return _lib.PREC_F32
    if precision == "auto":  # the reference runs fp32 (no autocast in its embedding code)
        return _lib.PREC_BF16 if torch.is_autocast_enabled("cuda") else _lib.PREC_F32
    raise ValueError(f"precision must be 'auto', 'f32' or 'bf16', got {precision!r}")


class _EncoderContext:
    """One ``mmpfn_enc`` context on a CUDA (HIP) device with the tower's weights uploaded."""

    def __init__(self, desc: _lib.EncDesc, state_dict: dict, device: torch.device):
        if not torch.cuda.is_available():
            raise RuntimeError("the modality encoders need a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _lib.load_library()
        dev = torch.device(device)
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        self.enc = self.lib.mmpfn_enc_create(idx, ctypes.c_void_p(self._stream()))
        if not self.enc:
            raise _lib.EngineError(f"mmpfn_enc_create failed on device {idx}")
        self.desc = desc
        self._check(self.lib.mmpfn_enc_set_model(self.enc, ctypes.byref(desc)), "mmpfn_enc_set_model")
        for name, t in state_dict.items():
            a = t.detach().to("cpu", torch.float32).contiguous().numpy()
            self._check(self.lib.mmpfn_enc_load_weight(self.enc, name.encode(), a.ctypes.data_as(ctypes.c_void_p), a.size),
                        f"mmpfn_enc_load_weight({name})")
        self._check(self.lib.mmpfn_enc_finalize(self.enc), "mmpfn_enc_finalize")

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _check(self, rc: int, what: str) -> None:
        _lib.check_enc(self.lib, self.enc, rc, what)

    def bind(self) -> None:
        self._check(self.lib.mmpfn_enc_set_stream(self.enc, ctypes.c_void_p(self._stream())), "mmpfn_enc_set_stream")

    def close(self) -> None:
        if getattr(self, "enc", None):
            self.lib.mmpfn_enc_destroy(self.enc)
            self.enc = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class _DeviceTower(nn.Module):
    """Parameter container whose forward runs on a lazily built device context (one per device)."""

    _skip_state = ("mask_token",)  # held for state-dict compatibility, not used by the forward

    def __init__(self):
        super().__init__()
        self._contexts: dict[str, _EncoderContext] = {}

    def _desc(self) -> _lib.EncDesc:  # pragma: no cover - abstract
        raise NotImplementedError

    def _drop_contexts(self) -> None:
        for c in self._contexts.values():
            c.close()
        self._contexts.clear()

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        self._drop_contexts()
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def _apply(self, fn, recurse=True):  # .to() / .half() etc.: the device copy is rebuilt on next use
        self._drop_contexts()
        return super()._apply(fn, recurse)

    def context(self, device: torch.device | str | None = None) -> _EncoderContext:
        dev = torch.device(device) if device is not None else torch.device("cuda")
        if dev.type != "cuda":
            raise RuntimeError(f"the modality encoders run on a ROCm GPU, not {dev}")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        key = str(dev)
        ctx = self._contexts.get(key)
        if ctx is None:
            sd = {k: v for k, v in self.state_dict().items() if k.split(".")[-1] not in self._skip_state}
            ctx = _EncoderContext(self._desc(), sd, dev)
            self._contexts[key] = ctx
        return ctx

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_contexts"] = {}
        return st


# ---------------------------------------------------------------------------------- image tower
class _PatchEmbed(nn.Module):
    def __init__(self, patch: int, in_chans: int, dim: int):
        super().__init__()
        self.proj = nn.Conv2d(in_chans, dim, kernel_size=patch, stride=patch)  # container only


class _LayerScale(nn.Module):
    def __init__(self, dim: int, init_values: float):
        super().__init__()
        self.gamma = nn.Parameter(init_values * torch.ones(dim))


class _Attn(nn.Module):
    def __init__(self, dim: int):
        super().__init__()
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim, bias=True)


class _Mlp(nn.Module):
    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden, bias=True)
        self.fc2 = nn.Linear(hidden, dim, bias=True)


class _Block(nn.Module):
    def __init__(self, dim: int, hidden: int, init_values: float | None):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = _Attn(dim)
        self.ls1 = _LayerScale(dim, init_values) if init_values else nn.Identity()
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = _Mlp(dim, hidden)
        self.ls2 = _LayerScale(dim, init_values) if init_values else nn.Identity()


class DinoVisionTransformer(_DeviceTower):
    """``DinoVisionTransformer`` (vision_transformer.py:36-271) for the configuration the reference
    uses (``vit_base``: plain MLP FFN, LayerNorm eps 1e-6, bicubic pos-embed interpolation with
    offset 0.1, no register tokens, ``block_chunks=0``).  ``forward_features`` runs on the device."""

    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768, depth=12, num_heads=12,
                 mlp_ratio=4.0, qkv_bias=True, ffn_bias=True, proj_bias=True, drop_path_rate=0.0,
                 drop_path_uniform=False, init_values=None, ffn_layer="mlp", block_chunks=0,
                 num_register_tokens=0, interpolate_antialias=False, interpolate_offset=0.1,
                 precision: str = "auto", **kwargs: Any):
        super().__init__()
        if not (qkv_bias and ffn_bias and proj_bias):
            raise NotImplementedError("biasless projections are not used by the reference's vit_base")
        if ffn_layer != "mlp" or num_register_tokens or interpolate_antialias:
            raise NotImplementedError("only the reference's configuration (mlp FFN, no register tokens, "
                                      "no antialias) is built")
        if block_chunks != 0:  # BlockChunk naming ("blocks.0.{i}") is the FSDP training layout
            raise NotImplementedError("only block_chunks=0 (the reference's vit_base call) is supported")
        if embed_dim % num_heads or embed_dim // num_heads != 64:
            raise NotImplementedError("head_dim must be 64")
        img = img_size if isinstance(img_size, int) else img_size[0]
        self.patch_size = int(patch_size)
        self.embed_dim = self.num_features = int(embed_dim)
        self.num_heads = int(num_heads)
        self.n_blocks = int(depth)
        self.num_register_tokens = 0
        self.interpolate_offset = float(interpolate_offset)
        self.interpolate_antialias = False
        self.precision = precision
        self._init_values = init_values
        self._grid = img // self.patch_size
        hidden = int(embed_dim * mlp_ratio)
        self._hidden = hidden
        self.patch_embed = _PatchEmbed(self.patch_size, in_chans, embed_dim)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, 1 + self._grid * self._grid, embed_dim))
        self.mask_token = nn.Parameter(torch.zeros(1, embed_dim))
        self.register_tokens = None
        self.blocks = nn.ModuleList([_Block(embed_dim, hidden, init_values) for _ in range(depth)])
        self.chunked_blocks = False
        self.norm = nn.LayerNorm(embed_dim, eps=1e-6)
        self.head = nn.Identity()
        self._in_chans = in_chans

    def _desc(self) -> _lib.EncDesc:
        d = _lib.EncDesc()
        d.kind = _lib.MMPFN_ENC_VIT
        d.dim, d.depth, d.heads, d.mlp_hidden = self.embed_dim, self.n_blocks, self.num_heads, self._hidden
        d.ln_eps = 1e-6
        d.patch, d.in_chans, d.pos_grid = self.patch_size, self._in_chans, self._grid
        d.interp_offset = self.interpolate_offset
        d.layerscale = int(bool(self._init_values))
        return d

    def _run(self, x: torch.Tensor, want_tokens: bool):
        if x.dim() != 4 or x.shape[1] != self._in_chans:
            raise ValueError(f"expected images [B, {self._in_chans}, H, W], got {tuple(x.shape)}")
        B, _, H, W = x.shape
        if H % self.patch_size or W % self.patch_size:
            raise ValueError(f"image size ({H}, {W}) must be a multiple of the patch size {self.patch_size}")
        dev = x.device if x.device.type == "cuda" else None
        ctx = self.context(dev)
        prec = _precision(self.precision, ctx.device)
        xd = x.to(ctx.device, torch.float32).contiguous()
        cls = torch.empty((B, self.embed_dim), device=ctx.device, dtype=torch.float32)
        L = 1 + (H // self.patch_size) * (W // self.patch_size)
        tok = torch.empty((B, L, self.embed_dim), device=ctx.device, dtype=torch.float32) if want_tokens else None
        ctx.bind()
        ctx._check(ctx.lib.mmpfn_vit_forward(ctx.enc, xd.data_ptr(), B, H, W, cls.data_ptr(),
                                             None if tok is None else tok.data_ptr(), prec), "mmpfn_vit_forward")
        return cls, tok

    def forward_features(self, x, masks=None):
        """``forward_features`` (vision_transformer.py:255-271).  ``x_prenorm`` (the residual stream before
        the final norm) is not materialised and is returned as None."""
        if isinstance(x, list):
            return [self.forward_features(xi, m) for xi, m in zip(x, masks if masks is not None else [None] * len(x))]
        if masks is not None:
            raise NotImplementedError("mask_token substitution (iBOT masking) is a training path")
        cls, tok = self._run(x, want_tokens=True)
        return {
            "x_norm_clstoken": cls,
            "x_norm_regtokens": tok[:, 1:1],
            "x_norm_patchtokens": tok[:, 1:],
            "x_prenorm": None,
            "masks": masks,
        }

    def cls_embeddings(self, x: torch.Tensor) -> torch.Tensor:
        """``forward_features(x)["x_norm_clstoken"]`` only: the last block runs on the CLS rows alone."""
        return self._run(x, want_tokens=False)[0]

    def forward(self, *args, is_training=False, **kwargs):
        """``forward`` (vision_transformer.py:329-334): the head (Identity) of the CLS token."""
        if is_training:
            return self.forward_features(*args, **kwargs)
        return self.head(self.cls_embeddings(*args, **kwargs))


def vit_base(patch_size=16, num_register_tokens=0, **kwargs) -> DinoVisionTransformer:
    """``vit_base`` (vision_transformer.py:355-366)."""
    return DinoVisionTransformer(patch_size=patch_size, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4,
                                 num_register_tokens=num_register_tokens, **kwargs)


# ---------------------------------------------------------------------------------- text tower
@dataclass
class ElectraConfigLite:
    """The ``ElectraConfig`` fields the forward uses (defaults: google/electra-base-discriminator)."""

    vocab_size: int = 30522
    embedding_size: int = 768
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_act: str = "gelu"
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    pad_token_id: int = 0

    @classmethod
    def from_any(cls, cfg) -> "ElectraConfigLite":
        if isinstance(cfg, cls):
            return cfg
        get = cfg.get if isinstance(cfg, dict) else (lambda k, d=None: getattr(cfg, k, d))
        out = cls()
        for f in out.__dataclass_fields__:
            v = get(f, None)
            if v is not None:
                setattr(out, f, v)
        return out


@dataclass
class TextEncoderOutput:
    last_hidden_state: torch.Tensor | None
    cls: torch.Tensor


class _BertSelf(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.query = nn.Linear(d, d)
        self.key = nn.Linear(d, d)
        self.value = nn.Linear(d, d)


class _BertSelfOut(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.dense = nn.Linear(d, d)
        self.LayerNorm = nn.LayerNorm(d, eps=eps)


class _BertAttn(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.self = _BertSelf(d)
        self.output = _BertSelfOut(d, eps)


class _BertInter(nn.Module):
    def __init__(self, d, f):
        super().__init__()
        self.dense = nn.Linear(d, f)


class _BertOut(nn.Module):
    def __init__(self, d, f, eps):
        super().__init__()
        self.dense = nn.Linear(f, d)
        self.LayerNorm = nn.LayerNorm(d, eps=eps)


class _BertLayer(nn.Module):
    def __init__(self, d, f, eps):
        super().__init__()
        self.attention = _BertAttn(d, eps)
        self.intermediate = _BertInter(d, f)
        self.output = _BertOut(d, f, eps)


class _Encoder(nn.Module):
    def __init__(self, c: ElectraConfigLite):
        super().__init__()
        self.layer = nn.ModuleList([_BertLayer(c.hidden_size, c.intermediate_size, c.layer_norm_eps)
                                    for _ in range(c.num_hidden_layers)])


class _Embeddings(nn.Module):
    def __init__(self, c: ElectraConfigLite):
        super().__init__()
        self.word_embeddings = nn.Embedding(c.vocab_size, c.embedding_size)
        self.position_embeddings = nn.Embedding(c.max_position_embeddings, c.embedding_size)
        self.token_type_embeddings = nn.Embedding(c.type_vocab_size, c.embedding_size)
        self.LayerNorm = nn.LayerNorm(c.embedding_size, eps=c.layer_norm_eps)


class ElectraTextEncoder(_DeviceTower):
    """transformers' ``ElectraModel`` forward (embeddings, optional ``embeddings_project``, post-LN BERT
    layers; GELU = erf) with the same state-dict names; ``__call__(input_ids, attention_mask,
    token_type_ids)`` returns ``.last_hidden_state`` like the reference's ``text_encoder(**inputs)``."""

    def __init__(self, config=None, precision: str = "auto"):
        super().__init__()
        c = ElectraConfigLite.from_any(config if config is not None else ElectraConfigLite())
        if c.hidden_act not in ("gelu",):
            raise NotImplementedError(f"hidden_act {c.hidden_act!r} (ELECTRA uses erf GELU)")
        if c.hidden_size % c.num_attention_heads or c.hidden_size // c.num_attention_heads != 64:
            raise NotImplementedError("head_dim must be 64")
        self.config = c
        self.precision = precision
        self.embeddings = _Embeddings(c)
        if c.embedding_size != c.hidden_size:
            self.embeddings_project = nn.Linear(c.embedding_size, c.hidden_size)
        self.encoder = _Encoder(c)

    @classmethod
    def from_hf(cls, model, precision: str = "auto") -> "ElectraTextEncoder":
        """From an instantiated transformers ``ElectraModel`` (e.g. ``AutoModel.from_pretrained(local_dir)``)."""
        enc = cls(model.config, precision=precision)
        sd = {k: v for k, v in model.state_dict().items() if not k.endswith(("position_ids", "token_type_ids"))}
        enc.load_state_dict(sd)
        return enc

    def _desc(self) -> _lib.EncDesc:
        c = self.config
        d = _lib.EncDesc()
        d.kind = _lib.MMPFN_ENC_TEXT
        d.dim, d.depth, d.heads, d.mlp_hidden = c.hidden_size, c.num_hidden_layers, c.num_attention_heads, c.intermediate_size
        d.ln_eps = c.layer_norm_eps
        d.vocab, d.max_pos, d.type_vocab, d.embedding_size = (c.vocab_size, c.max_position_embeddings,
                                                               c.type_vocab_size, c.embedding_size)
        return d

    def _run(self, input_ids, attention_mask=None, token_type_ids=None, want_hidden=True):
        ids = torch.as_tensor(input_ids)
        if ids.dim() == 1:
            ids = ids[None]
        B, L = ids.shape
        c = self.config
        if L > c.max_position_embeddings:
            raise IndexError(f"sequence length {L} > max_position_embeddings {c.max_position_embeddings}")
        if ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= c.vocab_size):
            raise IndexError("index out of range in self (input_ids)")
        dev = ids.device if ids.device.type == "cuda" else None
        ctx = self.context(dev)
        prec = _precision(self.precision, ctx.device)
        idd = ids.to(ctx.device, torch.int32).contiguous()
        md = None if attention_mask is None else torch.as_tensor(attention_mask).reshape(B, L).to(ctx.device, torch.int32).contiguous()
        td = None
        if token_type_ids is not None:
            tt = torch.as_tensor(token_type_ids).reshape(B, L)
            if tt.numel() and (int(tt.min()) < 0 or int(tt.max()) >= c.type_vocab_size):
                raise IndexError("index out of range in self (token_type_ids)")
            td = tt.to(ctx.device, torch.int32).contiguous()
        cls = torch.empty((B, c.hidden_size), device=ctx.device, dtype=torch.float32)
        hid = torch.empty((B, L, c.hidden_size), device=ctx.device, dtype=torch.float32) if want_hidden else None
        ctx.bind()
        ctx._check(ctx.lib.mmpfn_text_forward(ctx.enc, idd.data_ptr(), None if md is None else md.data_ptr(),
                                              None if td is None else td.data_ptr(), B, L, cls.data_ptr(),
                                              None if hid is None else hid.data_ptr(), prec), "mmpfn_text_forward")
        return TextEncoderOutput(last_hidden_state=hid, cls=cls)

    def forward(self, input_ids=None, attention_mask=None, token_type_ids=None, **kwargs):
        if kwargs.get("inputs_embeds") is not None or kwargs.get("position_ids") is not None:
            raise NotImplementedError("inputs_embeds / position_ids are not used by the reference")
        return self._run(input_ids, attention_mask, token_type_ids, want_hidden=True)

    def cls_embeddings(self, input_ids, attention_mask=None, token_type_ids=None) -> torch.Tensor:
        """``last_hidden_state[:, 0]`` only (the last layer runs on the CLS rows alone)."""
        return self._run(input_ids, attention_mask, token_type_ids, want_hidden=False).cls


# ---------------------------------------------------------------------------------- dataset helpers
def embed_images(encoder: DinoVisionTransformer, images, batch_size: int = 16) -> torch.Tensor:
    """The reference's embedding loop (pad_ufes_20.py:86-103): ``images [N, n_img, C, H, W]`` in
    batches of ``batch_size`` rows -> ``[N, n_img, D]`` CLS embeddings (on the host, like the
    reference's ``.cpu()`` before its ``torch.save``)."""
    imgs = torch.as_tensor(images)
    N, n_img = imgs.shape[:2]
    out = []
    for i in range(0, N, batch_size):
        batch = imgs[i:i + batch_size]
        flat = batch.reshape(-1, *batch.shape[2:])
        embs = encoder.cls_embeddings(flat.to("cuda", non_blocking=True))
        out.append(embs.reshape(-1, n_img, embs.shape[-1]).cpu())
    return torch.cat(out, 0)


def embed_texts(encoder: ElectraTextEncoder, token_ids, batch_size: int = 64) -> torch.Tensor:
    """The reference's text loop (petfinder.py:170-181) on pre-tokenised inputs: ``token_ids[i][j]``
    = the ids of text j of row i (what ``tokenizer(text, truncation=True, max_length=512)["input_ids"]``
    returns).  Texts are batched with padding + attention mask (equal to one call per text, which the
    reference makes) -> ``[N, n_text, D]``."""
    rows = [list(r) for r in token_ids]
    n_text = len(rows[0]) if rows else 0
    flat = [np.asarray(t, dtype=np.int64) for r in rows for t in r]
    outs = []
    for i in range(0, len(flat), batch_size):
        chunk = flat[i:i + batch_size]
        L = max(len(t) for t in chunk)
        ids = np.zeros((len(chunk), L), np.int64)
        mask = np.zeros((len(chunk), L), np.int64)
        for j, t in enumerate(chunk):
            ids[j, :len(t)] = t
            mask[j, :len(t)] = 1
        outs.append(encoder.cls_embeddings(torch.from_numpy(ids).cuda(), torch.from_numpy(mask).cuda()).cpu())
    D = encoder.config.hidden_size
    return torch.cat(outs, 0).reshape(len(rows), n_text, D) if outs else torch.empty((0, n_text, D))
