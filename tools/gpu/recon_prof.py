"""Reconstruction section times of a VTS_EXP_RPROF build (tools/exp/lib_rprof.so
copied over vtseg/libvtseg.so): one decode of the given video, then the
s_memtime totals per section of h264_deblock_plane (dp_plane) and
h264_intra_v2, summed over every wave, and per step (deblock: one macroblock
step of a wave's row groups; intra: one level of a workgroup's waves)."""
import ctypes as C
import json
import sys

sys.path.insert(0, "video-transformer_amd")
import torch  # noqa: F401  (libvtseg binds to torch's HIP runtime)
from vtseg import _lib, scene

DBK = ["wait_rows", "ring_in_vertical", "horizontal", "write_back", "loop_head_loads", "-", "still_steps", "steps"]
INTRA = ["setup_bucket_sort", "level_tail", "level_barrier", "mb_loads", "mb_luma", "mb_chroma", "wave_levels", "mbs"]
v = scene.VideoScorer(sys.argv[1], device=0, decoder="general")
v.run()
torch.cuda.synchronize()
fn = getattr(_lib.lib(), "vts_debug_recon_prof", None)
if fn is None:
    sys.exit("not a VTS_EXP_RPROF build")
fn.argtypes = [C.c_void_p]
out = (C.c_ulonglong * 16)()
fn(out)
v.run()
torch.cuda.synchronize()
fn(out)
d, i = list(out[:8]), list(out[8:])
res = {"video": sys.argv[1], "timings": v.timings(),
       "deblock": {n: x for n, x in zip(DBK, d) if n != "-"},
       "intra": {n: x for n, x in zip(INTRA, i) if n != "-"}}
if d[7]:
    res["deblock_cycles_per_iteration"] = {n: round(x / d[7], 1) for n, x in zip(DBK[:5], d[:5])}
if i[7]:
    res["intra_cycles_per_wave_mb_step"] = {n: round(x / i[7], 1) for n, x in zip(INTRA[3:6], i[3:6])}
if i[6]:
    res["intra_cycles_per_wave_level"] = {n: round(x / i[6], 1) for n, x in zip(INTRA[:3], i[:3])}
print(json.dumps(res))
v.close()
