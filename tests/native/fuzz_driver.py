"""Child process of tests/test_fuzz_host.py (run with the sanitizer runtimes
preloaded): feeds every mutated file to the sanitizer build of the host
parsers (libfz.so) and prints one JSON line of outcomes.  A sanitizer report
or a crash ends this process with a non-zero status; the parent asserts it
did not.  TEST INFRASTRUCTURE."""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

lib = C.CDLL(sys.argv[1])
files = [Path(p) for p in sys.argv[3:]]
out_dir = Path(sys.argv[2])
lib.vts_probe_duration.argtypes = [C.c_char_p, C.POINTER(C.c_double)]
lib.vts_keyframe_pts.argtypes = [C.c_char_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
lib.vts_extract_segment.argtypes = [C.c_char_p, C.c_double, C.c_double, C.c_char_p]
lib.fz_schedule.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
lib.fh_decode.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                          C.c_char_p, C.c_int]
stats = {"files": 0, "probe_ok": 0, "schedule_ok": 0, "decode_ok": 0, "remux_ok": 0, "keyframes_ok": 0}
cap = 64 * 640 * 480 * 3 // 2
frames = np.zeros(cap, np.uint8)
for f in files:
    b = str(f).encode()
    stats["files"] += 1
    d = C.c_double(-1.0)
    rc = lib.vts_probe_duration(b, C.byref(d))
    assert rc == 0 and d.value >= 0.0, (f, rc, d.value)  # reference convention: a float, never an error
    stats["probe_ok"] += d.value > 0
    pts = np.zeros(4096, np.int64)
    n, ts = C.c_int64(0), C.c_int64(0)
    rc = lib.vts_keyframe_pts(b, pts.ctypes.data, len(pts), C.byref(n), C.byref(ts))
    assert rc <= 0, (f, rc)
    stats["keyframes_ok"] += rc == 0
    err = C.create_string_buffer(512)
    rc = lib.fz_schedule(b, err, 512)
    assert rc in (0, -1), (f, rc)
    stats["schedule_ok"] += rc == 0
    rc = lib.vts_extract_segment(b, 0.2, 1.0, str(out_dir / "cut.mp4").encode())
    assert rc <= 0, (f, rc)
    stats["remux_ok"] += rc == 0
    got, w, h = C.c_int64(0), C.c_int(0), C.c_int(0)
    rc = lib.fh_decode(b, 0, frames.ctypes.data, cap, C.byref(got), C.byref(w), C.byref(h), err, 512)
    assert rc in (0, -1), (f, rc)
    stats["decode_ok"] += rc == 0
print(json.dumps(stats), flush=True)
