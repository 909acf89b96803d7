"""hipMalloc timing on a fresh process: fresh blocks of 1 / 8 / 37 GiB, the
same after a free, and a hipMemset of the big block (what vts_open's
whole-video buffers cost: the RGB thumbnails of a 2-h 720p video are 37 GB)."""
import ctypes
import json
import time

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
hip.hipDeviceSynchronize.argtypes = []
hip.hipSetDevice(0)
hip.hipDeviceSynchronize()
out = {}


def malloc(n):
    p = ctypes.c_void_p()
    t = time.perf_counter()
    rc = hip.hipMalloc(ctypes.byref(p), n)
    hip.hipDeviceSynchronize()
    return p, rc, (time.perf_counter() - t) * 1e3


for gib in (1, 8, 37):
    p, rc, ms = malloc(gib << 30)
    out[f"fresh_{gib}g_ms"] = round(ms, 1)
    if gib == 37:
        t = time.perf_counter()
        hip.hipMemset(p, 0, 37 << 30)
        hip.hipDeviceSynchronize()
        out["memset_37g_ms"] = round((time.perf_counter() - t) * 1e3, 1)
        t = time.perf_counter()
        hip.hipFree(p)
        out["free_37g_ms"] = round((time.perf_counter() - t) * 1e3, 1)
        p, rc, ms = malloc(37 << 30)
        out["again_37g_ms"] = round(ms, 1)
    hip.hipFree(p)
print(json.dumps(out))
