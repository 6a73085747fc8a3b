"""Round 6: HBM bytes per launch of the classify kernel in
the gap phases -- device-resident back to back, right after an SDMA copy, and
inside the backend -- from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(separate runs; FETCH_SIZE x 2, the gfx950 wide-read correction; KiB per
dispatch).  Usage: python3 scripts/r6_pmc_gap.py <dir>  (dirs <phase>_<counter>)"""
import csv
import glob
import json
import os
import statistics
import sys


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter and "mosrx_classify" in row.get("Kernel_Name", ""):
                    k = row.get("Dispatch_Id")
                    vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


root = sys.argv[1]
out = {}
for d in sorted(glob.glob(os.path.join(root, "*_FETCH_SIZE"))):
    ph = os.path.basename(d)[:-len("_FETCH_SIZE")]
    f = per_dispatch(d, "FETCH_SIZE")
    w = per_dispatch(os.path.join(root, ph + "_WRITE_SIZE"), "WRITE_SIZE")
    out[ph] = {"dispatches": len(f),
               "fetch_MB_x2": round(2 * statistics.median(f) * 1024 / 1e6, 2) if f else None,
               "write_MB": round(statistics.median(w) * 1024 / 1e6, 2) if w else None}
print(json.dumps(out, indent=1))
