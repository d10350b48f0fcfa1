"""Diagnostics: every wave of one attn_pipe_kernel launch stamped (a `-DMMPFN_STAMPS_ALL` variant build:
tools/src_variant.sh stamps_all attention_pipe.hip <no-op sed> -DMMPFN_STAMPS_ALL).

The engine's own launch (two batched config-C members, T = 72, fp16 mode, the last layer of the second forward).
Each wave records HW_ID / XCC_ID and s_memtime at start, after its prologue barrier and after each of its 29 loop
steps.  The waves are grouped by (XCC, SE, CU, SIMD) and every step of every wave is classified by how many OTHER
waves of its SIMD (and of its CU) were inside their loop at the step's midpoint; the step time is reported per
class.  Question answered: are the slow steps (2x the median) the ones that share their SIMD with a partner wave's
loop, or does something else (the launch round, the block's position) make them slow?
"""
import ctypes
import os
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tools")]
os.environ.setdefault("MMPFN_DIAGNOSTICS", "1")
NST = 36


def main():
    os.environ["MMPFN_PROF_BATCH"] = "2"
    import prof_forward

    from multimodalpfn_amd import _lib

    sys.argv = [sys.argv[0], "2"]
    prof_forward.main()
    lib = _lib.load_library()
    lib.mmpfn_dbg_attn_stamps_all.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nb = 4176
    buf = (ctypes.c_ulonglong * (nb * 4 * (NST + 2)))()
    assert lib.mmpfn_dbg_attn_stamps_all(buf, nb) == 0
    a = np.array(buf, dtype=np.int64).reshape(nb * 4, NST + 2)
    out = os.environ.get("MMPFN_STAMPS_OUT")
    if out:
        np.save(out, a)
    hw, xcc, st = a[:, 0], a[:, 1], a[:, 2:]
    nstep = 29
    active = (st[:, 2] > 0) & (st[:, 2 + nstep] > 0)  # waves that ran the loop (idle waves stamp no steps)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key_cu = list(zip(xcc & 15, se, sh, cu))
    loop0, loop1 = st[:, 2], st[:, 2 + nstep]  # in-loop interval [after prologue, after last step]
    groups_simd, groups_cu = defaultdict(list), defaultdict(list)
    for w in range(len(a)):
        if st[w, 0] == 0:
            continue
        groups_cu[key_cu[w]].append(w)
        groups_simd[key_cu[w] + (int(simd[w]),)].append(w)
    print(f"waves {int((st[:, 0] > 0).sum())}, in loop {int(active.sum())}, CUs {len(groups_cu)}, "
          f"SIMDs {len(groups_simd)}; waves per SIMD over the launch: "
          f"{np.mean([len(v) for v in groups_simd.values()]):.1f}")
    res = defaultdict(list)
    res_cu = defaultdict(list)
    for g, ws in groups_simd.items():
        cu_ws = groups_cu[g[:4]]
        for w in ws:
            if not active[w]:
                continue
            for k in range(nstep):
                t0, t1 = st[w, 2 + k], st[w, 3 + k]
                mid = (t0 + t1) // 2
                n_simd = sum(1 for v in ws if v != w and active[v] and loop0[v] <= mid < loop1[v])
                n_cu = sum(1 for v in cu_ws if v != w and active[v] and loop0[v] <= mid < loop1[v])
                res[n_simd].append(t1 - t0)
                res_cu[n_cu].append(t1 - t0)
    for name, r in (("other in-loop waves on the same SIMD", res), ("other in-loop waves on the same CU", res_cu)):
        print(name)
        for n in sorted(r):
            v = np.array(r[n])
            print(f"  {n}: {len(v):7d} steps, median {np.median(v):6.0f}, mean {v.mean():6.0f}, p10 "
                  f"{np.percentile(v, 10):6.0f}, p90 {np.percentile(v, 90):6.0f} cycles")
    # step time by step index and by the block's start order within its CU
    steps = np.diff(st[active][:, 2:3 + nstep], axis=1)
    print("median step time by step index: " + " ".join(f"{x:.0f}" for x in np.median(steps, axis=0)))
    life = (st[:, 35] - st[:, 0])[st[:, 35] > 0]
    print(f"wave lifetime median {np.median(life):.0f}, blocks per CU over the launch "
          f"{np.mean([len(v) for v in groups_cu.values()]) / 4:.1f}")


if __name__ == "__main__":
    main()
