"""Write synthetic 720p general-decoder inputs in parallel (bench.py's
writer settings): python tools/gpu/write_streams.py KIND FRAMES OUT ...
KIND = content (x264-like coded content) or noise (random full syntax)."""
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "video-transformer_amd"))
from vtseg import scene  # noqa: E402

kind, frames, outs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]


def one(i_p):
    i, p = i_p
    extra = dict(content=True, gop_max_s=8.0) if kind == "content" else {}
    return scene.synth_write(p, width=1280, height=720, fps=30, n_frames=frames, seed=0x5EED + i, coding="full",
                             slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True,
                             transform_8x8=True, **extra)


with ThreadPoolExecutor(len(outs)) as ex:
    list(ex.map(one, enumerate(outs)))
print("wrote", outs, flush=True)
