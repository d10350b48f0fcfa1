"""Per-predict GPU timeline from a rocprofv3 kernel trace of tools/api_profile.py: windows start at each
mixer LayerNorm (ln_rows_kernel, first GPU kernel of a predict); span, busy (union of kernels), gaps."""
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50])
              for r in csv.DictReader(open(sys.argv[1])))
starts = [i for i, r in enumerate(rows) if "ln_rows_kernel" in r[2]]
for a, b in zip(starts, starts[1:] + [len(rows)]):
    win = rows[a:b]
    busy, cs, ce, gaps = 0, None, None, []
    for s, e, n in win:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
                gaps.append(((s - ce) / 1e3, n))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    span = win[-1][1] - win[0][0]
    big = sorted(gaps, reverse=True)[:4]
    print(f"span {span / 1e3:8.1f} us busy {busy / 1e3:8.1f} us  gaps " + ", ".join(f"{g:.0f}us<{n[:28]}" for g, n in big))
