"""Per-kernel busy time from a rocprofv3 kernel trace: the union of the
dispatch intervals divided by the dispatch count.  With interleaved GOP
groups two reconstruct dispatches run at once, so rocprofv3's mean duration
per dispatch is about twice the share of wall time each one takes; the union
is what bench.py's event span / launches measures.

    python tools/kernel_busy.py <run_kernel_trace.csv> [name substring]
"""
import csv
import sys


def busy(path: str, needle: str) -> tuple[int, float, float]:
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                for r in csv.DictReader(open(path)) if needle in r["Kernel_Name"])
    tot, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            tot, cs, ce = tot + ce - cs, s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    return len(iv), tot / len(iv), sum(e - s for s, e in iv) / len(iv)


if __name__ == "__main__":
    needle = sys.argv[2] if len(sys.argv) > 2 else "h264_recon_score<4>"
    n, u, m = busy(sys.argv[1], needle)
    print(f"{needle}: {n} dispatches, busy (union of intervals) {u / 1e3:.2f} us per dispatch, "
          f"mean dispatch duration {m / 1e3:.2f} us")
