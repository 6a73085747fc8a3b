# round 6: the latency table with the batch-level probe
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6b
timeout -k 10 500 python -u scripts/r6_latency.py S64,M1500 0,2000 > gpurun_out/r6b/latency.jsonl 2> gpurun_out/r6b/latency.err || { tail -20 gpurun_out/r6b/latency.err; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r6b/latency.jsonl"):
    r = json.loads(l)
    if "saturated_mpkts" in r:
        print(r); continue
    print(r["key"], r["group"], r["load"], r["group_max_us"], "off", r["offered_mpkts"], "del", r["delivered_mpkts"],
          "avail", r["avail_us"], "cons", r["consumed_us"], "mean_grp", r["mean_group_frames"], "max_grp", r["max_group_frames"])
PY
