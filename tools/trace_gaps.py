"""Idle gaps of the GPU in a rocprofv3 kernel trace: union of kernel intervals vs span, largest gaps.
python tools/trace_gaps.py run_kernel_trace.csv [gap_us_threshold]"""
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60])
              for r in csv.DictReader(open(sys.argv[1])))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
busy, cur_s, cur_e, gaps = 0, None, None, []
prev_name = ""
for s, e, n in rows:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append(((s - cur_e) / 1e3, prev_name, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev_name = n
busy += cur_e - cur_s
span = rows[-1][1] - rows[0][0]
print(f"span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f} %), kernels {len(rows)}")
big = [g for g in gaps if g[0] >= thr]
print(f"gaps >= {thr} us: {len(big)}, total {sum(g[0] for g in big) / 1e3:.2f} ms")
for g in sorted(big, reverse=True)[:25]:
    print(f"  {g[0]:9.1f} us  after {g[1]}  before {g[2]}")
