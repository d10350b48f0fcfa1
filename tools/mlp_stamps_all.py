"""Diagnostics: every wave of one mlp_rows_kernel launch stamped (a `-DMMPFN_STAMPS_ALL` variant build:
tools/src_variant.sh stamps_all <file> <no-op sed> -DMMPFN_STAMPS_ALL).

The engine's own launch (two batched config-C members, fp16 mode, the last layer's MLP with the fused attention
out-projection: 165 456 rows, 1 293 blocks of 4 waves x 32 rows).  Stamps per wave: start, O / X landed,
out-projection halves, LayerNorm, H(0), each of the 24 hidden chunks, stores.  Printed: phase medians, the chunk-time
distribution, blocks per CU over the launch and how the CUs' last blocks end (the grid's tail)."""
import ctypes
import os
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tools")]
os.environ.setdefault("MMPFN_DIAGNOSTICS", "1")
NST = 32


def main():
    os.environ["MMPFN_PROF_BATCH"] = "2"
    import prof_forward

    from multimodalpfn_amd import _lib

    sys.argv = [sys.argv[0], "2"]
    prof_forward.main()
    lib = _lib.load_library()
    lib.mmpfn_dbg_mlp_stamps_all.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nb = (2 * 2298 * 36 + 127) // 128
    buf = (ctypes.c_ulonglong * (nb * 8 * (NST + 2)))()
    assert lib.mmpfn_dbg_mlp_stamps_all(buf, nb) == 0
    a = np.array(buf, dtype=np.int64).reshape(nb * 8, NST + 2)[: nb * 4]  # index block * 4 + wave
    out = os.environ.get("MMPFN_STAMPS_OUT")
    if out:
        np.save(out, a)
    hw, xcc, st = a[:, 0], a[:, 1], a[:, 2:]
    ok = (st[:, 0] > 0) & (st[:, NST - 1] > 0)
    st, hw, xcc = st[ok], hw[ok], xcc[ok]
    life = st[:, NST - 1] - st[:, 0]
    ph = [("O / X / Wout half 0 landed", 0, 1), ("out-projection half 0", 1, 2), ("out-projection half 1", 2, 3),
          ("LayerNorm, W1(0) landed", 3, 4), ("H(0)", 4, 5), ("24 hidden chunks", 5, 29), ("stores", 29, NST - 1)]
    med = np.median(life)
    print(f"waves {len(st)}; wave lifetime median {med:.0f} cycles, p10 {np.percentile(life, 10):.0f}, "
          f"p90 {np.percentile(life, 90):.0f}")
    for name, i, j in ph:
        v = np.median(st[:, j] - st[:, i])
        print(f"  {name:32s} {v:8.0f} cycles  {100 * v / med:5.1f} %")
    ch = np.diff(st[:, 5:30], axis=1)
    print(f"  per chunk: median {np.median(ch):.0f}, mean {ch.mean():.0f}, p10 {np.percentile(ch, 10):.0f}, "
          f"p90 {np.percentile(ch, 90):.0f} cycles; by chunk index: " + " ".join(f"{x:.0f}" for x in np.median(ch, 0)))
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = list(zip(xcc & 15, se, sh, cu))
    blocks = defaultdict(list)  # CU -> [(start, end)] per block (wave 0 rows only: one entry per block)
    seen = set()
    for w in range(len(st)):
        blocks[key[w]].append((st[w, 0], st[w, NST - 1]))
    per_xcd = defaultdict(list)
    for k, v in blocks.items():
        per_xcd[k[0]].append((min(s for s, _ in v), max(e for _, e in v), len(v) / 4))
    for x in sorted(per_xcd):
        v = per_xcd[x]
        t0 = min(s for s, _, _ in v)
        ends = np.array([e - t0 for _, e, _ in v])
        nbk = np.array([n for _, _, n in v])
        print(f"  XCD {x}: {len(v)} CUs, blocks per CU {nbk.min():.0f}-{nbk.max():.0f}, CU finish (kcycles after the "
              f"XCD's first start) min {ends.min() / 1e3:.0f} median {np.median(ends) / 1e3:.0f} max {ends.max() / 1e3:.0f}")
    del seen
    # the slots of a few CUs: each block's (start, end) in kcycles after the CU's first start
    for k in list(blocks)[:4]:
        v = sorted(set((int(s), int(e)) for s, e in blocks[k]))
        bl = defaultdict(lambda: [1 << 62, 0])
        for s_, e_ in v:
            pass
        t0 = min(s_ for s_, _ in v)
        starts = sorted(set(round((s_ - t0) / 1e3) for s_, _ in v))
        print(f"  CU {k}: wave starts (kcycles) {starts}")


if __name__ == "__main__":
    main()
