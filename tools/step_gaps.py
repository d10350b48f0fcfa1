"""GPU idle time inside the bench's timed steps from a rocprofv3 kernel trace: busy fraction of the span of
steps [s0, s1) (a step = 24 two-member item-attention launches at config C) and the gaps > 15 us with the
kernels either side.  Usage: python3 tools/step_gaps.py run_kernel_trace.csv [s0 s1]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
s0, s1 = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (10, 30)
att = [r for r in rows if "attn_pipe" in r["Kernel_Name"] and r["Grid_Size_X"] == "1069056"]
t0, t1 = int(att[24 * s0]["Start_Timestamp"]), int(att[24 * s1 - 1]["End_Timestamp"])
win = [r for r in rows if int(r["Start_Timestamp"]) >= t0 and int(r["End_Timestamp"]) <= t1]
busy, gaps, ce, prev = 0, [], None, None
cs = None
for r in win:
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if ce is None:
        cs, ce, prev = a, b, r
        continue
    if a > ce:
        busy += ce - cs
        gaps.append((a - ce, prev["Kernel_Name"][:40], r["Kernel_Name"][:40]))
        cs = a
    if b > ce:
        ce, prev = b, r
busy += ce - cs
n = s1 - s0
print(f"steps {s0}-{s1}: {(t1 - t0) / 1e6 / n:.3f} ms per step, GPU busy {busy / (t1 - t0):.3f}, "
      f"idle {(t1 - t0 - busy) / 1e6 / n:.3f} ms per step ({sum(g for g, _, _ in gaps if g > 15000) / 1e6 / n:.3f} in gaps > 15 us)")
for g, a, b in gaps[: len(gaps) // n + 1]:
    if g > 15000:
        print(f"  gap {g / 1e3:7.1f} us after {a:40s} before {b}")
