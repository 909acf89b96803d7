# Round 4: the open sequence of the bench (allocator), the parser prefetch
# variants (prev = the committed build, pf2 = two row-above columns in
# flight, cur = + colocated motion requested first, deblocking bands code,
# splitting allocator, 128 GiB window cap) on the content and noise streams;
# then deblocking in bands (VTS_DBK_BANDS: parity, 1 / 2 / 3 same-process).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04k}
mkdir -p $O
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
with ThreadPoolExecutor(3) as ex:
    a = ex.submit(scene.synth_write, "/tmp/gcab.mp4", **kw)
    b = ex.submit(scene.synth_write, "/tmp/gcontent.mp4", content=True, gop_max_s=8.0, **kw)
    c = ex.submit(scene.synth_write, "/tmp/sub_long.mp4", width=1280, height=720, fps=30, n_frames=108000, seed=0x5EED)
    a.result(); b.result(); c.result()
print("streams written", flush=True)
PY
timeout -k 10 300 python - > $O/open_sequence.json 2> $O/open_sequence.err <<'PY' || { tail -20 $O/open_sequence.err; exit 1; }
# the bench's order: a long subset video's session, then the general streams'
import json, sys, time
sys.path.insert(0, "video-transformer_amd")
import torch
from vtseg import scene
out = []
for p in ("/tmp/sub_long.mp4", "/tmp/gcab.mp4", "/tmp/gcontent.mp4", "/tmp/gcab.mp4"):
    t0 = time.perf_counter()
    v = scene.VideoScorer(p, device=0)
    dt = time.perf_counter() - t0
    v.run(); torch.cuda.synchronize()
    t1 = time.perf_counter(); v.run(); torch.cuda.synchronize()
    out.append({"video": p, "open_s": round(dt, 3), "run_s": round(time.perf_counter() - t1, 3), "windows": v.windows(),
                "stages": v.open_timings(), "timings": v.timings()})
    print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    v.close()
print(json.dumps(out))
PY
cat $O/open_sequence.json
PASSES=2 bash tools/gpu/lib_ab.sh /tmp/gcontent.mp4 3 $O/ab_content prev pf2 cur || exit 1
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/gcab.mp4 3 $O/ab_noise prev pf2 cur || exit 1
VTS_DBK_BANDS=2 timeout -k 10 600 python -u -m pytest tests/test_full_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_bands2.log 2>&1 || { tail -40 $O/pytest_bands2.log; exit 1; }
tail -1 $O/pytest_bands2.log
for V in gcontent gcab; do
timeout -k 10 400 python tools/gpu/env_ab.py /tmp/$V.mp4 3 b1=VTS_DBK_BANDS=1 b2=VTS_DBK_BANDS=2 b3=VTS_DBK_BANDS=3 > $O/bands_$V.json 2> $O/bands_$V.err || { tail -20 $O/bands_$V.err; exit 1; }
cat $O/bands_$V.json
done
