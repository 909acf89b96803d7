# Round 5: where the 2-h video's open spends its alloc time after the bench's
# earlier sessions (devmem log).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 400 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, n_frames=18000, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True, seed=0x5EED)
with ThreadPoolExecutor(7) as ex:
    fs = [ex.submit(scene.synth_write, f"/tmp/sub{i}.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=11 + i) for i in range(4)]
    fs.append(ex.submit(scene.synth_write, "/tmp/gnoise.mp4", **kw))
    fs.append(ex.submit(scene.synth_write, "/tmp/gcontent.mp4", content=True, gop_max_s=8.0, **kw))
    fs.append(ex.submit(scene.synth_write, "/tmp/long.mp4", width=1280, height=720, fps=30, n_frames=216000, seed=0x5EED))
    for f in fs: f.result()
print("streams written", flush=True)
PY
VTS_DEVMEM_LOG=1 timeout -k 10 400 python tools/gpu/open_order_probe.py /tmp/long.mp4 /tmp/sub0.mp4,/tmp/sub1.mp4,/tmp/sub2.mp4,/tmp/sub3.mp4 /tmp/gnoise.mp4 /tmp/gcontent.mp4 > $O/order.json 2> $O/order.err || { tail -30 $O/order.err; exit 1; }
cat $O/order.json
grep -E "devmem|probe" $O/order.err | tail -60
