"""Per-dispatch kernel durations of rocprofv3 --kernel-trace runs of bench.py
rows (gpurun_out/prof3/kt_<row>/), split into the bench's phases: a new phase
where two dispatches are more than 300 us apart.  Prints n / median / gap per
phase.  Usage: python3 scripts/kt_phases.py M1500_1 IMIX_1 ..."""
import csv, statistics as st, sys
for W in sys.argv[1:]:
    rows = [r for r in csv.DictReader(open(f'gpurun_out/prof3/kt_{W}/kt_kernel_trace.csv')) if 'classify' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    segs, cur, last = [], [], None
    for r in rows:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if last is not None and s - last > 300_000:
            segs.append(cur); cur = []
        cur.append((s, e)); last = e
    segs.append(cur)
    out = []
    for sg in segs:
        d = [(e - s) / 1e3 for s, e in sg]
        gaps = [(sg[i + 1][0] - sg[i][1]) / 1e3 for i in range(len(sg) - 1)] or [0]
        out.append(f"n={len(sg)} med={st.median(d):.2f} gap={st.median(gaps):.2f}")
    print(W, ' | '.join(out))
