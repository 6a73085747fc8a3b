"""Per gap phase: the classify kernel's memory-side read latency at the L2 /
fabric interface (Little's law: TCC_EA0_RDREQ_LEVEL, the outstanding reads
summed per cycle, over TCC_EA0_RDREQ, the reads issued), its DRAM-credit stall
cycles and active cycles, medians over dispatches.
Usage: python3 scripts/r6_pmc_lat.py <dir>   (one subdirectory per phase)"""
import csv
import glob
import json
import os
import statistics
import sys

root = sys.argv[1]
out = {}
for d in sorted(glob.glob(os.path.join(root, "*/"))):
    ph = os.path.basename(d.rstrip("/"))
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "mosrx_classify" not in row.get("Kernel_Name", ""):
                    continue
                k = row["Dispatch_Id"]
                per.setdefault(k, {})
                c = row["Counter_Name"]
                per[k][c] = per[k].get(c, 0.0) + float(row["Counter_Value"])
    rows = [v for v in per.values() if v.get("TCC_EA0_RDREQ_sum")]
    if not rows:
        continue
    med = lambda key: statistics.median(r.get(key, 0.0) for r in rows)  # noqa: E731
    out[ph] = {"dispatches": len(rows),
               "read_latency_cycles": round(statistics.median(r["TCC_EA0_RDREQ_LEVEL_sum"] / r["TCC_EA0_RDREQ_sum"]
                                                              for r in rows), 1),
               "rdreq": med("TCC_EA0_RDREQ_sum"), "rdreq_dram": med("TCC_EA0_RDREQ_DRAM_sum"),
               "dram_credit_stall_cycles": med("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"),
               "gui_active": med("GRBM_GUI_ACTIVE")}
print(json.dumps(out, indent=1))
