# Round 5: CABAC parse skip fast path + h264_derive with every macroblock's
# words loaded at once and prefetched one step ahead.  GPU parity suite, then
# same-box A/B (in-tree vs 6 parse waves per SIMD) on the 10-min 720p content
# and noise streams, and a kernel trace of the content stream.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
with ThreadPoolExecutor(2) as ex:
    a = ex.submit(scene.synth_write, "/tmp/gcab.mp4", **kw)
    b = ex.submit(scene.synth_write, "/tmp/gcontent.mp4", content=True, gop_max_s=8.0, **kw)
    a.result(); b.result()
print("streams written", flush=True)
PY
for V in gcontent gcab; do
  PASSES=2 timeout -k 10 500 bash tools/gpu/lib_ab.sh /tmp/$V.mp4 3 $O/ab_$V cur w6 || exit 1
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/kt_gcontent" -o run -- python3 "$GRAFT_REPO_ROOT/tools/gpu/env_ab.py" /tmp/gcontent.mp4 1 x= > "$GRAFT_REPO_ROOT/$O/kt_gcontent.log" 2>&1) || { tail -30 $O/kt_gcontent.log; exit 1; }
ST=$(find $O/kt_gcontent -name '*kernel_stats.csv' | head -1)
cp "$ST" $O/kt_gcontent_kernel_stats.csv
grep -E "parse|derive" $O/kt_gcontent_kernel_stats.csv
