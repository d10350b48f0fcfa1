"""Average rocprofv3 --pmc counters per kernel over the dispatches of a run (csv dirs)."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(list))
meta = {}
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = r["Kernel_Name"]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[k] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"], r["Accum_VGPR_Count"])
for k, cs in sorted(agg.items(), key=lambda kv: -max(sum(v) for v in kv[1].values())):
    short = k.split("(")[0][-60:]
    print(f"== {short}  grid,wg,lds,vgpr,agpr={meta[k]}")
    print("   " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))
