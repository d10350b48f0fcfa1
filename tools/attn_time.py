"""Time the sample-axis attention layer kernel (mmpfn_item_attention_layer) of the library
named by MMPFN_LIB at the config-C shape and check it against a torch fp32 reference on the GPU.
Usage: MMPFN_LIB=path python3 tools/attn_time.py [reps]"""
import math
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from multimodalpfn_amd import _lib  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
T, H, d = int(os.environ.get("ATT_T", 36)), 6, 32
S, N = int(os.environ.get("ATT_S", 2298)), int(os.environ.get("ATT_N", 1838))
Npad = (N + 63) // 64 * 64
lib = _lib.load_library(os.environ.get("MMPFN_LIB") or None)
ctx = lib.mmpfn_create(0, None)
g = torch.Generator().manual_seed(0)
# ATT_PREC=f16: the fp16 mode's forward kernel (q, k bf16, out fp16, V^T bf16; the headline's launch; ATT_FORM=tap:
# the fp16 q / k form of the kernel-level tap instead), else bf16
f16 = os.environ.get("ATT_PREC", "bf16") == "f16"
tap16 = f16 and os.environ.get("ATT_FORM") == "tap"
qdt = torch.float16 if tap16 else torch.bfloat16
q = torch.randn(T, H, S, d, generator=g).cuda()
k = torch.randn(T, H, Npad, d, generator=g).cuda()
if os.environ.get("ATT_QROUND") == "bf16":  # fp16 operands holding bf16 values: the same bits toggle as in bf16 mode
    q, k = q.bfloat16().float(), k.bfloat16().float()
q, k = q.to(qdt), k.to(qdt)
vt = torch.randn(T, H, d, Npad, generator=g).cuda().bfloat16()
o = torch.empty(T, S, H * d, device="cuda", dtype=torch.float16 if f16 else torch.bfloat16)
st = torch.cuda.current_stream()


def launch():
    if f16:
        rc = lib.mmpfn_item_attention_layer_ex(ctx, q.data_ptr(), k.data_ptr(), vt.data_ptr(), o.data_ptr(), S, T, H,
                                               Npad, N, 5 if tap16 else 5 | _lib.ATTN_QK_BF16)  # MMPFN_PREC_F16
    else:
        rc = lib.mmpfn_item_attention_layer(ctx, q.data_ptr(), k.data_ptr(), vt.data_ptr(), o.data_ptr(), S, T, H,
                                            Npad, N)
    assert rc == 0


for _ in range(3):
    launch()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    launch()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
fl = 4.0 * T * S * N * H * d
# reference on a few columns
cols = [0, T // 2, T - 1]
qf, kf, vf = q[cols].float(), k[cols, :, :N].float(), vt[cols, :, :, :N].float().transpose(-1, -2)
s = qf @ kf.transpose(-1, -2) / math.sqrt(d)
ref_tr = torch.softmax(s[:, :, :N], -1) @ vf
s0 = qf[:, :, N:] @ kf[:, :1].transpose(-1, -2) / math.sqrt(d)
ref_te = torch.softmax(s0, -1) @ vf[:, :1]
ref = torch.cat([ref_tr[:, :, :N], ref_te], 2).permute(0, 2, 1, 3).reshape(len(cols), S, H * d)
err = (o[cols].float() - ref).abs().max().item()
print(f"{os.path.basename(os.environ.get('MMPFN_LIB', 'default'))}: {ms*1e3:.1f} us  {fl/ms/1e9:.1f} TFLOP/s  "
      f"frac {fl/ms/1e9/2500:.3f}  maxerr {err:.2e}")
