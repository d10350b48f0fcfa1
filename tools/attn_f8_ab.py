"""Time the sample-axis attention layer (mmpfn_item_attention_layer_ex) in several precision codes at one
shape, with the error of each against torch fp32 on the GPU.  Libraries: MMPFN_LIBS=name=path,... (default:
the in-tree build).  Usage: python tools/attn_f8_ab.py [reps] [codes, e.g. 1,3,4,5,6,7]
Shape: ATT_T / ATT_S / ATT_N (default config E: T = 11, S = 12000, N = 10000); ATT_SCALE scales q (wider
score spreads)."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from multimodalpfn_amd import _lib  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
codes = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "1,3,4,5,6,7").split(",")]
T, H, d = int(os.environ.get("ATT_T", 11)), 6, 32
S, N = int(os.environ.get("ATT_S", 12000)), int(os.environ.get("ATT_N", 10000))
sc = float(os.environ.get("ATT_SCALE", "1"))
Npad = (N + 63) // 64 * 64
libs = [kv.split("=") for kv in os.environ.get("MMPFN_LIBS", "tree=").split(",")]
g = torch.Generator().manual_seed(0)
q = (torch.randn(T, H, S, d, generator=g) * sc).cuda()
k = torch.randn(T, H, Npad, d, generator=g).cuda()
vt = torch.randn(T, H, d, Npad, generator=g).cuda()
# reference (fp32 on the GPU): train rows on their own heads, test rows on head 0
kk, vv = k[:, :, :N].float(), vt[:, :, :, :N].transpose(-1, -2).float()
ref = torch.empty(T, S, H * d, device="cuda")
for t in range(T):
    for h in range(H):
        for (a, b, kh) in ((0, N, h), (N, S, 0)):
            s = (q[t, h, a:b].float() @ kk[t, kh].T) / d ** 0.5
            ref[t, a:b, h * d:(h + 1) * d] = torch.softmax(s, -1) @ vv[t, kh]
for name, path in libs:
    lib = _lib.load_library(path or None)
    ctx = lib.mmpfn_create(0, None)
    for code in codes:
        f16 = code >= 5
        dt = torch.float16 if f16 else torch.bfloat16
        qd, kd, vd = q.to(dt), k.to(dt), vt.bfloat16()
        o = torch.empty(T, S, H * d, device="cuda", dtype=dt)

        def launch():
            assert lib.mmpfn_item_attention_layer_ex(ctx, qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), o.data_ptr(), S,
                                                     T, H, Npad, N, code) == 0

        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            launch()
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        err = (o.float() - ref).abs().max().item()
        fl = 4.0 * T * S * N * H * d
        print(f"{name:10s} code {code}: {ms:.4f} ms/launch ({fl / ms / 1e9:.0f} TFLOP/s), max |err| {err:.3e}", flush=True)
    lib.mmpfn_destroy(ctx)
