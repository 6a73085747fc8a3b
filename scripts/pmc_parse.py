"""Per-launch HBM bytes from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE is corrected by x2 for gfx950 wide streaming reads, as
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) prescribes; WRITE_SIZE is
taken as is.  Both counters are in KiB per dispatch.
Usage: python3 scripts/pmc_parse.py <key> <fetch_dir> <write_dir> <kernel_substring> <out.json>"""
import csv
import glob
import json
import os
import statistics
import sys


def per_dispatch(d, counter, ksub):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter and ksub in row.get("Kernel_Name", ""):
                    k = row.get("Dispatch_Id")
                    vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


key, fdir, wdir, ksub, out = sys.argv[1:6]
fetch = per_dispatch(fdir, "FETCH_SIZE", ksub)
write = per_dispatch(wdir, "WRITE_SIZE", ksub)
res = json.load(open(out)) if os.path.exists(out) else {}
fk = statistics.median(fetch) if fetch else None
wk = statistics.median(write) if write else None
res[key] = {
    "fetch_kib_raw_median": fk, "write_kib_median": wk, "dispatches": [len(fetch), len(write)],
    "hbm_bytes_per_launch": (int(fk * 1024 * 2 + (wk or 0) * 1024) if fk is not None else None),
    "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 wide-read correction) + --pmc WRITE_SIZE, "
              "separate passes, median per dispatch of scripts/pmc_run.py",
}
json.dump(res, open(out, "w"), indent=1)
print(key, res[key])
