"""Parse section times of a VTS_EXP_PROF build (tools/exp/lib_prof.so copied
over vtseg/libvtseg.so): one decode of the given video, then the s_memtime
totals per section of h264_parse_full(_cabac) (summed over every slice)."""
import ctypes as C
import json
import sys

sys.path.insert(0, "video-transformer_amd")
import torch  # noqa: F401  (libvtseg binds to torch's HIP runtime)
from vtseg import _lib, scene

NAMES = ["setup", "begin_mb", "mb_syntax", "motion", "cbp_qp", "residual", "end_mb", "tail"]
v = scene.VideoScorer(sys.argv[1], device=0, decoder="general")
v.run()
torch.cuda.synchronize()
fn = getattr(_lib.lib(), "vts_debug_parse_prof", None)
if fn is None:
    sys.exit("this libvtseg.so is not a VTS_EXP_PROF build (tools/exp/build_full_variants.sh prof:-DVTS_EXP_PROF)")
fn.argtypes = [C.c_void_p]
out = (C.c_ulonglong * 8)()
fn(out)           # reset after the first run
v.run()
torch.cuda.synchronize()
fn(out)
tot = sum(out) or 1  # an all-zero read: no instrumented kernel ran
print(json.dumps({"video": sys.argv[1], "timings": v.timings(),
                  "sections": {n: [int(x), round(x / tot, 4)] for n, x in zip(NAMES, out)}}))
v.close()
