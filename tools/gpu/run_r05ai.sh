# Round 5: intra macroblocks by capacity-aware rounds (h264_intra_v2) vs by
# dependency level (lib_levels: the tree before): GPU suite, same-box timing
# on 10-min 720p content and noise streams, and rocprofv3 kernel stats (the
# largest intra dispatch) for each library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ai
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?
tail -3 $O/pytest_gpu.txt
grep -n "FAILED\|ERROR" $O/pytest_gpu.txt | head -20
if [ $rc -gt 1 ] || grep -q "Memory access fault\|HSA_STATUS_ERROR\|hipErrorLaunchFailure" $O/pytest_gpu.txt; then exit 1; fi
export GPU_MAX_HW_QUEUES=16
timeout -k 10 400 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
with ThreadPoolExecutor(2) as ex:
    fs = [ex.submit(scene.synth_write, "/tmp/gcab.mp4", n_frames=18000, **kw),
          ex.submit(scene.synth_write, "/tmp/gcontent.mp4", n_frames=18000, content=True, gop_max_s=8.0, **kw)]
    for f in fs: f.result()
print("streams written", flush=True)
PY
cp video-transformer_amd/vtseg/libvtseg.so tools/exp/lib_cur.so
for V in gcontent gcab; do
  for L in cur levels levels cur; do
    cp tools/exp/lib_$L.so video-transformer_amd/vtseg/libvtseg.so
    timeout -k 10 240 python tools/gpu/env_ab.py /tmp/$V.mp4 3 $L= >> $O/ab_$V.jsonl 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
    tail -1 $O/ab_$V.jsonl
  done
  for L in cur levels; do
    cp tools/exp/lib_$L.so video-transformer_amd/vtseg/libvtseg.so
    (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_${L}_$V -o run -- python $GRAFT_REPO_ROOT/tools/gpu/env_ab.py /tmp/$V.mp4 1 $L= > $GRAFT_REPO_ROOT/$O/prof_${L}_$V.log 2>&1) || { tail -20 $O/prof_${L}_$V.log; cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
    f=$(find $O/prof_${L}_$V -name "*kernel_stats.csv" | head -1)
    grep -E "intra_v2|deblock_plane|inter_full" "$f" | cut -d, -f1-7 | sed "s/^/$L $V /"
  done
done
cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
