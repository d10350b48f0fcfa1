"""Per-block timeline of attn_item2_kernel from a -DA2_STAMPS build (diagnostics only).
Usage: MMPFN_LIB=multimodalpfn_amd/libmmpfn_var_st.so python3 tools/attn_stamps.py"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from multimodalpfn_amd import _lib  # noqa: E402

T, H, d, S, N = 36, 6, 32, 2298, 1838
Npad = (N + 63) // 64 * 64
lib = _lib.load_library(os.environ["MMPFN_LIB"])
lib.mmpfn_dbg_attn_stamps.argtypes = [ctypes.c_void_p]
ctx = lib.mmpfn_create(0, None)
g = torch.Generator().manual_seed(0)
q = torch.randn(T, H, S, d, generator=g).cuda().bfloat16()
k = torch.randn(T, H, Npad, d, generator=g).cuda().bfloat16()
vt = torch.randn(T, H, d, Npad, generator=g).cuda().bfloat16()
o = torch.empty(T, S, H * d, device="cuda", dtype=torch.bfloat16)
for _ in range(20):
    lib.mmpfn_item_attention_layer(ctx, q.data_ptr(), k.data_ptr(), vt.data_ptr(), o.data_ptr(), S, T, H, Npad, N)
torch.cuda.synchronize()
buf = np.zeros(4096 * 4, dtype=np.uint64)
assert lib.mmpfn_dbg_attn_stamps(buf.ctypes.data) == 0
st = buf.reshape(4096, 4).astype(np.int64)
nb = int((st[:, 0] > 0).sum())
st = st[:nb]
t0 = st[:, 0].min()
st = (st - t0) / 100.0  # us (100 MHz)
span = st[:, 3].max()
print(f"blocks {nb}, kernel span {span:.1f} us")
dur = st[:, 3] - st[:, 0]
print(f"block duration us: mean {dur.mean():.1f} p10 {np.percentile(dur,10):.1f} p90 {np.percentile(dur,90):.1f} max {dur.max():.1f}")
print(f"prologue (start->first barrier) mean {(st[:,1]-st[:,0]).mean():.2f} us; loop mean {(st[:,2]-st[:,1]).mean():.1f} us; "
      f"epilogue mean {(st[:,3]-st[:,2]).mean():.2f} us")
bins = np.linspace(0, span, 21)
conc = [int(((st[:, 0] <= b) & (st[:, 3] > b)).sum()) for b in bins[:-1]]
print("blocks running over time:", conc)
print("block starts per bin:", np.histogram(st[:, 0], bins)[0].tolist())
