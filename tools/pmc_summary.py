"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch).

    python tools/pmc_summary.py DIR [DIR ...] [--json out.json]

Each DIR holds one pass (rocprofv3 -d DIR ... --pmc ...).  HBM traffic per
dispatch follows MI355X_MICROARCH.md's HBM section: FETCH_SIZE (KB) x 2 on
gfx950 (wide coalesced reads are tallied at half their bytes) + WRITE_SIZE
(KB), x 1024 to bytes.
"""
from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    m = re.search(r"(h264_\w+|thumb_sad|score_\w+)(<\d+>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name.split("(")[0][-60:]


def load(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in Path(d).rglob("*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--json")
    a = ap.parse_args()
    acc = load(a.dirs)
    out = {}
    for k, cs in sorted(acc.items()):
        if not any(x in k for x in ("h264", "thumb_sad", "score_")):
            continue
        row = {c: sum(v) / len(v) for c, v in cs.items()}
        row["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
            row["hbm_bytes_per_dispatch"] = (2 * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024
        if "SQ_WAVE_CYCLES" in row and row["SQ_WAVE_CYCLES"]:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in row:
                    row[c + "_frac"] = row[c] / row["SQ_WAVE_CYCLES"]
        out[k] = row
    for k, row in out.items():
        print(k)
        for c, v in sorted(row.items()):
            print(f"    {c:32s} {v:,.3f}")
    if a.json:
        Path(a.json).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
