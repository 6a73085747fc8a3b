"""Round 6: the backend's auto groups at 512 MiB and 1 GiB of frames per launch
(MOSRX_MAX_GROUP 512): saturated rate and device fraction."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mos-networking-stack_amd"))
import bench  # noqa: E402
import mosrx  # noqa: E402

legs = [("S64", 64_000_000), ("M1500", 3_000_000), ("IMIX", 20_000_000)]
for rep in range(2):
    for key, tgt in legs:
        tr = mosrx.Trace({"S64": mosrx.TRACE_S64, "M1500": mosrx.TRACE_M1500, "IMIX": mosrx.TRACE_IMIX}[key],
                         {"S64": 32768, "M1500": 65536, "IMIX": 262144}[key])
        for gb in (512 << 20, 1 << 30):
            r = bench.measure_backend(tr, key, tgt * (2 if gb > (512 << 20) else 1), cpu=0, group=0, group_bytes=gb)
            print(json.dumps({"key": key, "group_bytes_mib": gb >> 20, "rep": rep, "mpkts": round(r["mpkts"], 1),
                              "dev_frac": r["device_roofline_frac"], "dev_us": r["device_us_per_batch"],
                              "bpl": r["batches_per_launch"], "launches": r["kernel_launches"]}), flush=True)
