"""Diagnostics: per-phase cycle stamps of attn_pipe_kernel (needs `make -C multimodalpfn_amd/csrc dbg`).

One fp16-mode launch at config C's bench shape (T = 72 token columns, S = 2298, N = 1838) and one at config E
(T = 11, S = 12000, N = 10000), random q / k / v.  The kernel's 8 stamped blocks (4 waves each) record s_memtime
(shader cycles) at: start, Q loaded, prologue barrier, the end of every pipelined step (the first 42), the loop's
drain, the row-sum check, the stores.  Printed per shape: the cycles of each phase (median over the 32 waves),
the per-step distribution, and the phase shares of the wave's lifetime.

Run on the GPU box:  MMPFN_LIB=multimodalpfn_amd/libmmpfn_hip_dbg.so python3 tools/attn_stamps.py
"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("MMPFN_DIAGNOSTICS", "1")
os.environ.setdefault("MMPFN_LIB", str(ROOT / "multimodalpfn_amd" / "libmmpfn_hip_dbg.so"))
from multimodalpfn_amd import _lib  # noqa: E402

NST = 48


def report(a, grid, ntiles, label):
    nstep = min(ntiles, NST - 6)
    ok = [w for w in range(32) if a[w, 0] and a[w, NST - 1] and a[w, 2 + nstep]]  # active waves only
    a = a[ok]
    rel = a - a[:, 0:1]
    steps = np.diff(a[:, 2:3 + nstep], axis=1)  # step t = stamp 3 + t - stamp 2 + t
    life = rel[:, NST - 1]
    ph = {
        "Q load (start -> Q fragments)": np.median(rel[:, 1]),
        "prologue (tiles 0-1 staged, barrier)": np.median(a[:, 2] - a[:, 1]),
        f"pipelined steps (first {nstep} of {ntiles})": np.median(a[:, 2 + nstep] - a[:, 2]),
        "remaining steps + drain": np.median(a[:, NST - 3] - a[:, 2 + nstep]),
        "row-sum check (+ any re-run)": np.median(a[:, NST - 2] - a[:, NST - 3]),
        "normalise + stores": np.median(a[:, NST - 1] - a[:, NST - 2]),
    }
    med = np.median(life)
    print(f"{label}: grid {grid} blocks, {ntiles} key tiles, {len(ok)} stamped active waves; "
          f"wave lifetime median {med:.0f} cycles ({med / 2.4e3:.1f} us at 2.4 GHz)")
    for name, v in ph.items():
        print(f"  {name:44s} {v:9.0f} cycles  {100 * v / med:5.1f} %")
    s = steps.reshape(-1)
    print(f"  per step (tile, 64 keys x 64 queries per wave): median {np.median(s):.0f}, mean {s.mean():.0f}, "
          f"p10 {np.percentile(s, 10):.0f}, p90 {np.percentile(s, 90):.0f}, max {s.max():.0f} cycles")
    print(f"  step 0 / 1 / 2 medians {np.median(steps[:, 0]):.0f} / {np.median(steps[:, 1]):.0f} / "
          f"{np.median(steps[:, 2]):.0f}; steps 4.. median {np.median(steps[:, 4:]):.0f}")
    print("  median over waves per step index: " + " ".join(f"{v:.0f}" for v in np.median(steps, axis=0)))
    t0 = a[:, 0].min()
    print("  wave start offsets (kcycles, by block x wave): " + " ".join(f"{(v - t0) / 1e3:.1f}" for v in a[:, 0]))
    print("  wave end offsets   (kcycles, by block x wave): " + " ".join(f"{(v - t0) / 1e3:.1f}" for v in a[:, NST - 1]))


def read(lib):
    st = (ctypes.c_ulonglong * (8 * 4 * NST))()
    meta = (ctypes.c_int * 4)()
    assert lib.mmpfn_dbg_attn_stamps(st, meta) == 0
    return np.array(st, dtype=np.int64).reshape(32, NST), meta[0], meta[1]


def run_forward(lib):
    """The engine's own launch: two batched config-C members (T = 72, Q pre-scaled by the QKV weights), fp16 mode;
    the stamps are the last layer's attention launch."""
    sys.path.insert(0, str(ROOT / "tools"))
    os.environ["MMPFN_PROF_BATCH"] = "2"
    import prof_forward

    sys.argv = [sys.argv[0], "2"]
    prof_forward.main()
    a, grid, ntiles = read(lib)
    report(a, grid, ntiles, "engine forward, config C, T=72 (last layer's launch)")


def run(lib, ctx, T, S, N, reps=5):
    H, d = 6, 32
    Npad = (N + 63) // 64 * 64
    g = torch.Generator().manual_seed(0)
    q = torch.randn(T, H, S, d, generator=g).cuda().half()
    k = torch.randn(T, H, Npad, d, generator=g).cuda().half()
    vt = torch.randn(T, H, d, Npad, generator=g).cuda().bfloat16()
    o = torch.empty(T, S, H * d, device="cuda", dtype=torch.float16)
    for _ in range(reps):
        assert lib.mmpfn_item_attention_layer_ex(ctx, q.data_ptr(), k.data_ptr(), vt.data_ptr(), o.data_ptr(), S, T,
                                                 H, Npad, N, 5) == 0
    torch.cuda.synchronize()
    a, grid, ntiles = read(lib)
    report(a, grid, ntiles, f"layer entry (Q scaled in-kernel), T={T} S={S} N={N}")


def main():
    lib = _lib.load_library()
    lib.mmpfn_dbg_attn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.mmpfn_dbg_attn_stamps.restype = ctypes.c_int
    run_forward(lib)
    ctx = lib.mmpfn_create(0, None)
    run(lib, ctx, 72, 2298, 1838)
    run(lib, ctx, 11, 12000, 10000, reps=2)
    lib.mmpfn_destroy(ctx)


if __name__ == "__main__":
    main()
