"""tools/kt_timeline.py on a small synthetic rocprofv3 kernel trace: the last
decode is taken from its last parse launch on, per-stream busy time, kernel
means and the gaps before each kernel are reported, and the union of busy
time counts overlapping streams once."""
import csv
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
FIELDS = ["Kind", "Agent_Id", "Queue_Id", "Stream_Id", "Thread_Id", "Dispatch_Id", "Kernel_Id", "Kernel_Name",
          "Correlation_Id", "Start_Timestamp", "End_Timestamp"]


def _row(name, stream, t0, t1):
    return {"Kind": "KERNEL_DISPATCH", "Agent_Id": "Agent 2", "Queue_Id": 1, "Stream_Id": stream, "Thread_Id": 1,
            "Dispatch_Id": 1, "Kernel_Id": 1, "Kernel_Name": name, "Correlation_Id": 1,
            "Start_Timestamp": t0, "End_Timestamp": t1}


def test_timeline_of_the_last_decode(tmp_path):
    ns = 1_000_000  # 1 ms
    rows = [
        # an earlier decode: ignored
        _row("vts::h264_parse_full_cabac(vts::FullParseArgs)", 1, 0, 5 * ns),
        _row("vts::h264_inter_full(vts::FullReconArgs)", 2, 6 * ns, 7 * ns),
        # the last decode: parse, then two streams of level launches
        _row("vts::h264_parse_full_cabac(vts::FullParseArgs)", 1, 100 * ns, 110 * ns),
        _row("vts::h264_inter_full(vts::FullReconArgs)", 2, 111 * ns, 112 * ns),
        _row("vts::h264_deblock_plane<false>(vts::FullReconArgs)", 2, 113 * ns, 115 * ns),
        _row("vts::h264_inter_full(vts::FullReconArgs)", 5, 114 * ns, 116 * ns),
        _row("vts::h264_bs_full(vts::FullReconArgs)", 3, 110 * ns, 111 * ns),
    ]
    path = tmp_path / "run_kernel_trace.csv"
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        w.writerows(rows)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "kt_timeline.py"), str(path)], check=True,
                         capture_output=True, text=True).stdout
    d = json.loads(out)
    assert d["parse_ms"] == 10.0
    assert d["recon_span_ms"] == 6.0  # 110 .. 116 ms
    s2 = d["streams"]["2"]
    assert s2["launches"] == 2 and s2["busy_ms"] == 3.0
    assert s2["kernels"]["h264_deblock_plane"]["n"] == 1
    assert s2["gap_before"]["h264_deblock_plane"]["total_ms"] == 1.0
    # 110-111 (bS), 111-112, 113-116 (two streams overlapping at 114-115)
    assert d["union_busy_ms"] == 5.0
