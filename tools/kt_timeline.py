"""Per-stream timeline of one general-decoder run from a rocprofv3 kernel trace.
    python tools/kt_timeline.py KERNEL_TRACE_CSV
Takes the last decode in the trace (from the last parse launch on), and for the
reconstruction kernels after it reports, per stream: launches, busy time,
span, the gaps between consecutive launches (by the kernel that follows the
gap), and for the whole run the union of busy time over the streams."""
import csv
import json
import sys
from collections import defaultdict

RECON = ("h264_inter_full", "h264_intra_v2", "h264_intra_full", "h264_bs_full", "h264_deblock_lds", "h264_deblock_full",
         "h264_deblock_plane")


def short(name):
    for k in RECON + ("h264_parse_full_cabac", "h264_parse_full", "h264_derive", "nal_unescape"):
        if k in name:
            return k
    return name.split("(")[0][-40:]


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                   r.get("Stream_Id") or r.get("Queue_Id")))
    ks.sort()
    parse_starts = [k[0] for k in ks if k[2].startswith("h264_parse_full")]
    t0 = parse_starts[-1]
    run = [k for k in ks if k[0] >= t0]
    parse_end = max(k[1] for k in run if k[2].startswith("h264_parse_full"))
    rec = [k for k in run if k[2] in RECON]
    out = {"parse_ms": (parse_end - t0) / 1e6, "recon_span_ms": (max(k[1] for k in rec) - min(k[0] for k in rec)) / 1e6}
    by_stream = defaultdict(list)
    for k in rec:
        by_stream[k[3]].append(k)
    streams = {}
    for s, lst in by_stream.items():
        lst.sort()
        busy = sum(e - b for b, e, _, _ in lst)
        gaps = defaultdict(list)
        for prev, cur in zip(lst, lst[1:]):
            gaps[cur[2]].append(max(0, cur[0] - prev[1]))
        per = defaultdict(lambda: [0, 0])
        for b, e, n, _ in lst:
            per[n][0] += 1
            per[n][1] += e - b
        streams[str(s)] = {
            "launches": len(lst),
            "busy_ms": busy / 1e6,
            "span_ms": (lst[-1][1] - lst[0][0]) / 1e6,
            "kernels": {n: {"n": c, "busy_ms": t / 1e6, "mean_us": t / c / 1e3} for n, (c, t) in per.items()},
            "gap_before": {n: {"n": len(g), "total_ms": sum(g) / 1e6, "mean_us": sum(g) / len(g) / 1e3} for n, g in gaps.items()},
        }
    out["streams"] = streams
    # union of busy intervals over all streams
    iv = sorted((b, e) for b, e, _, _ in rec)
    tot, cb, ce = 0, iv[0][0], iv[0][1]
    for b, e in iv[1:]:
        if b > ce:
            tot += ce - cb
            cb, ce = b, e
        else:
            ce = max(ce, e)
    tot += ce - cb
    out["union_busy_ms"] = tot / 1e6
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
