# Round 5: the per-picture reconstruction scheduler (h264_recon_sched) —
# (1) the full-decoder GPU parity tests with it (the default), (2) same-box A/B
# against the per-level launch chain (VTS_RECON_SCHED=0) on the 10-minute
# content and noise streams (digests must agree), (3) a kernel trace of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05g}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_full_gpu.py tests/test_decode_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python - <<'PY' || exit 1
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
for V in gcontent gcab; do
  timeout -k 10 300 python tools/gpu/env_ab.py /tmp/$V.mp4 3 sched=VTS_RECON_SCHED=1 lvl=VTS_RECON_SCHED=0 > $O/ab_$V.json 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; exit 1; }
  cat $O/ab_$V.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/tools/gpu/env_ab.py /tmp/gcontent.mp4 1 sched=VTS_RECON_SCHED=1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -1 | xargs grep -E "recon_sched|derive|parse_full" || true
