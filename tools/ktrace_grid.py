"""Summarise a rocprofv3 kernel_trace.csv per (kernel, grid): launches, average and total
duration -- separates launch shapes that kernel_stats.csv averages together (e.g. the
bench's roofline launches of the attention kernel from the batched forward's)."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("mmpfn::(anonymous namespace)::", "").replace("void ", "")
    name = name.replace("_ZN5mmpfn12_GLOBAL__N_1", "").split("(")[0]
    acc[(name, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(sum(v) for v in acc.values())
print(f"{'kernel':44s} {'grid':>9s} {'wg':>4s} {'n':>5s} {'avg_us':>9s} {'total_ms':>9s} {'%':>5s}")
for (name, g, wg), v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:n]:
    print(f"{name[:44]:44s} {g:9d} {wg:4d} {len(v):5d} {sum(v)/len(v):9.1f} {sum(v)/1e3:9.2f} {100*sum(v)/tot:5.1f}")
print(f"total {tot/1e3:.2f} ms")
