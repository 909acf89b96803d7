"""Timeline of one general-decoder run from a rocprofv3 kernel trace: the
last run's dispatches after its parse kernel, the union of busy intervals
(all kernels, per kernel), how many dispatches run at once, and the gaps
where none does.
    python tools/gpu/recon_timeline.py TRACE_DIR"""
import collections
import csv
import glob
import json
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("vts::", "").split("<")[0]
    grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0) * int(r.get("Grid_Size_Y") or 1)
    wg = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 1) * int(r.get("Workgroup_Size_Y") or 1)
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, r.get("Queue_Id", ""), r.get("Stream_Id", ""),
                 grid // max(1, wg)))
rows.sort()
parses = [i for i, r in enumerate(rows) if r[2].startswith("h264_parse")]
t_parse_end = rows[parses[-1]][1]
rec = [r for r in rows[parses[-1] + 1:] if r[0] >= t_parse_end - 1000]
t0, t1 = min(r[0] for r in rec), max(r[1] for r in rec)


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if cs is not None else 0)


ev = sorted([(r[0], 1) for r in rec] + [(r[1], -1) for r in rec])
conc = collections.Counter()
c, last = 0, t0
for t, d in ev:
    conc[c] += t - last
    c += d
    last = t
per = collections.defaultdict(list)
for r in rec:
    per[r[2]].append((r[0], r[1]))
out = {"span_ms": round((t1 - t0) / 1e6, 2), "busy_union_ms": round(union([(r[0], r[1]) for r in rec]) / 1e6, 2),
       "dispatches": len(rec), "queues": len(set(r[3] for r in rec)),
       "ms_at_concurrency": {k: round(v / 1e6, 2) for k, v in sorted(conc.items())},
       "per_kernel": {k: {"n": len(v), "union_ms": round(union(v) / 1e6, 2),
                          "sum_ms": round(sum(e - s for s, e in v) / 1e6, 2)} for k, v in per.items()}}
# per kernel: dispatch duration against its workgroup count; per queue: the
# idle time between one dispatch's end and the next one's start
byk = collections.defaultdict(list)
for r in rec:
    byk[r[2]].append((r[5], (r[1] - r[0]) / 1e3))
out["duration_us_by_workgroups"] = {}
for k, v in byk.items():
    v.sort()
    qs = [v[int(q * (len(v) - 1))] for q in (0, 0.25, 0.5, 0.75, 1.0)]
    out["duration_us_by_workgroups"][k] = [(w, round(d, 1)) for w, d in qs]
    small = [d for w, d in v if w <= 16]
    if small:
        out["duration_us_by_workgroups"][k + " (<=16 wg, median)"] = round(sorted(small)[len(small) // 2], 1)
gaps = collections.defaultdict(list)
byq = collections.defaultdict(list)
for r in rec:
    byq[r[3]].append(r)
for q, v in byq.items():
    v.sort()
    for a, b in zip(v, v[1:]):
        gaps[q].append(max(0, b[0] - a[1]) / 1e3)
out["queue_gaps_us"] = {q: {"n": len(g), "median": round(sorted(g)[len(g) // 2], 1), "sum_ms": round(sum(g) / 1e3, 2)}
                        for q, g in gaps.items() if g}
out["queue_busy_ms"] = {q: round(union([(r[0], r[1]) for r in v]) / 1e6, 2) for q, v in byq.items()}
print(json.dumps(out, indent=1))
