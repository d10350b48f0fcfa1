"""Diagnostics: per-phase cycle stamps of one feat_block_kernel block (needs `make -C multimodalpfn_amd/csrc dbg`).

Run on the GPU box:  MMPFN_LIB=multimodalpfn_amd/libmmpfn_hip_dbg.so python tools/stamps.py
"""

import ctypes
import os
import subprocess
import sys

os.environ.setdefault("MMPFN_DIAGNOSTICS", "1")
os.environ.setdefault("MMPFN_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                "multimodalpfn_amd", "libmmpfn_hip_dbg.so"))
import tools_prof_forward  # noqa: E402


def main():
    sys.argv = [sys.argv[0], "3"]
    tools_prof_forward.main()
    from multimodalpfn_amd import _lib

    lib = _lib.load_library()
    buf = (ctypes.c_ulonglong * 32)()
    rc = lib.mmpfn_dbg_featblock_stamps(buf)
    assert rc == 0, rc
    st = list(buf)
    names = {0: "start", 1: "phase0 (X load, W0 stage)", 20: "Wout staged", 21: "out-proj MFMA"}
    for h in range(6):
        names[2 + 3 * h] = f"head{h} QKV"
        names[3 + 3 * h] = f"head{h} attention"
        names[4 + 3 * h] = f"head{h} W stash"
    prev = st[0]
    for k in sorted(names):
        if k == 0 or st[k] == 0:
            continue
        print(f"{names[k]:28s} {st[k] - prev:8d} cycles (memtime ticks)")
        prev = st[k]
    print("total", prev - st[0])


if __name__ == "__main__":
    main()
