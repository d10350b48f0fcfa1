"""Per-block timeline of attn_item2_kernel from a -DA2_STAMPS build (diagnostics only).
Usage: MMPFN_LIB=multimodalpfn_amd/libmmpfn_var_st.so ATT_T=72 ATT_S=2298 ATT_N=1838 python3 tools/attn_stamps.py

Stamps per block (s_memrealtime, 100 MHz): 0 start, 1 after setup (Q, tile-0 staging), 2 after the
first tile, 3 after the loop, 4 end (wave 0), 5 HW_ID (SIMD / CU / SH / SE of wave 0)."""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from multimodalpfn_amd import _lib  # noqa: E402

T, H, d = int(os.environ.get("ATT_T", 72)), 6, 32
S, N = int(os.environ.get("ATT_S", 2298)), int(os.environ.get("ATT_N", 1838))
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
    assert lib.mmpfn_item_attention_layer(ctx, q.data_ptr(), k.data_ptr(), vt.data_ptr(), o.data_ptr(), S, T, H,
                                          Npad, N) == 0
torch.cuda.synchronize()
buf = np.zeros(16384 * 6, dtype=np.uint64)
assert lib.mmpfn_dbg_attn_stamps(buf.ctypes.data) == 0
st = buf.reshape(16384, 6).astype(np.int64)
nb = int((st[:, 0] > 0).sum())
st = st[:nb]
hw = st[:, 5]
t = (st[:, :5] - st[:, 0].min()) / 100.0  # us
span = t[:, 4].max()
ntiles = (N + 63) // 64
print(f"T={T} S={S} N={N}: blocks {nb}, tiles per block {ntiles}, kernel span {span:.1f} us")
dur = t[:, 4] - t[:, 0]
print(f"block duration us: mean {dur.mean():.2f} p10 {np.percentile(dur, 10):.2f} p50 {np.median(dur):.2f} "
      f"p90 {np.percentile(dur, 90):.2f} max {dur.max():.2f}")
print(f"phases (mean us): setup {(t[:, 1] - t[:, 0]).mean():.2f}, first tile {(t[:, 2] - t[:, 1]).mean():.2f}, "
      f"tiles 2..n {(t[:, 3] - t[:, 2]).mean():.2f} ({(t[:, 3] - t[:, 2]).mean() / max(1, ntiles - 1):.3f} per tile), "
      f"epilogue {(t[:, 4] - t[:, 3]).mean():.2f}")
# residency per CU: CU = (XCD = block % 8, SE, SH, CU id) from HW_ID
cu_id = (hw >> 8) & 0xF
sh_id = (hw >> 12) & 1
se_id = (hw >> 13) & 7
xcd = np.arange(nb) & 7
cu = ((xcd * 8 + se_id) * 2 + sh_id) * 16 + cu_id
ucu = np.unique(cu)
busy = np.zeros(len(ucu))
first = np.zeros(len(ucu))
last = np.zeros(len(ucu))
for i, c in enumerate(ucu):
    sel = cu == c
    busy[i] = dur[sel].sum()
    first[i], last[i] = t[sel, 0].min(), t[sel, 4].max()
print(f"CUs seen {len(ucu)}; blocks per CU mean {nb / len(ucu):.2f}; mean resident blocks per CU over the span "
      f"{busy.sum() / len(ucu) / span:.3f}; over each CU's own first..last {np.mean(busy / (last - first)):.3f}")
print(f"CU last-block end: p10 {np.percentile(last, 10):.1f} p50 {np.median(last):.1f} max {last.max():.1f} us")
bins = np.linspace(0, span, 21)
conc = [int(((t[:, 0] <= b) & (t[:, 4] > b)).sum()) for b in bins[:-1]]
print("blocks running over time:", conc)
# back-to-back gaps: for each block, the end of the latest earlier-finishing block on the same CU
gaps = []
for c in ucu:
    idx = np.where(cu == c)[0]
    ends = np.sort(t[idx, 4])
    for j in idx:
        prev = ends[ends <= t[j, 0] + 1e-9]
        if len(prev) and t[j, 0] > 0.5:
            gaps.append(t[j, 0] - prev[-1])
gaps = np.array(gaps)
if len(gaps):
    print(f"start - latest earlier end on the CU (us): mean {gaps.mean():.2f} p50 {np.median(gaps):.2f} "
          f"p90 {np.percentile(gaps, 90):.2f}")
