"""Per-launch HBM bytes of attn_pipe_kernel from two rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE).

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  On gfx950 FETCH_SIZE counts half the bytes of a
16-B-per-lane streaming read (MI355X_MICROARCH.md, HBM section): the kernel's K, V^T and Q reads
are all 16 B per lane, so the read bytes are 2 x FETCH_SIZE; WRITE_SIZE is exact for its 8-B
stores' 64-B lines.  Output: one JSON object on stdout."""
import csv
import json
import os
import sys

T, H, d, S, N = int(os.environ.get("ATT_T", 36)), 6, 32, 2298, 1838
NPAD = (N + 63) // 64 * 64
vals = {}
for path in sys.argv[1:]:
    for r in csv.DictReader(open(f"{path}/run_counter_collection.csv")):
        if "attn_pipe_kernel" in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
read_b = 2.0 * fetch * 1024
write_b = write * 1024
alg_read = T * H * S * d * 2 + 2 * T * H * N * d * 2  # Q + K + V^T (16-bit), keys up to nk
alg_write = T * S * H * d * 2
print(json.dumps({
    "kernel": "attn_pipe_kernel",
    "precision": os.environ.get("ATT_PREC", "bf16"),
    "shape": {"T": T, "H": H, "d": d, "S": S, "N": N},
    "launches": len(vals["FETCH_SIZE"]),
    "FETCH_SIZE_KiB_avg": round(fetch, 1),
    "WRITE_SIZE_KiB_avg": round(write, 1),
    "hbm_read_bytes": round(read_b),
    "hbm_write_bytes": round(write_b),
    "hbm_bytes_per_launch": round(read_b + write_b),
    "algorithmic_bytes_per_launch": alg_read + alg_write,
    "correction": "read = 2 x FETCH_SIZE (gfx950, 16-B/lane streaming reads); write = WRITE_SIZE",
}, indent=1))
