"""Per-kernel SQ counter summary (sums over launches) of tools/layer_pmc.sh's two passes."""
import collections
import re
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
nl = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("void ", "").replace("mmpfn::(anonymous namespace)::", "")
        k = re.sub(r"\(.*", "", k)[:44]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        nl[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    w = c.get("SQ_WAVE_CYCLES", 0)
    if w < 1e7:
        continue
    busy = c.get("SQ_BUSY_CYCLES", 1)
    print(f"{k}  launches {len(nl[k]) // 2}")
    print(f"  per wave-cycle: wait_inst {c['SQ_WAIT_INST_ANY'] / w:.2f} (lds {c['SQ_WAIT_INST_LDS'] / w:.2f})  "
          f"wait_any {c['SQ_WAIT_ANY'] / w:.2f}  active_any {c['SQ_ACTIVE_INST_ANY'] / w:.2f}  "
          f"valu {c['SQ_ACTIVE_INST_VALU'] / w:.2f}  lds {c['SQ_ACTIVE_INST_LDS'] / w:.2f}")
    print(f"  insts: valu {c['SQ_INSTS_VALU']:.3g} trans {c['SQ_INSTS_VALU_TRANS_F32']:.3g} mfma {c['SQ_INSTS_MFMA']:.3g} "
          f"lds {c['SQ_INSTS_LDS']:.3g}  lds_bank_conflict/idx_active {c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_LDS_IDX_ACTIVE']):.3f}")
    print(f"  mfma_busy {c['SQ_VALU_MFMA_BUSY_CYCLES']:.3g}  sq_busy {busy:.3g}  grbm_active {c['GRBM_GUI_ACTIVE']:.3g}  "
          f"mfma_busy/(grbm*1024) {c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1, c['GRBM_GUI_ACTIVE'] * 1024 / 8):.3f}")
