# Per-dispatch durations of the general decoder's reconstruction kernels
# (rocprofv3 kernel trace) on the x264-like 10-min 720p CABAC B stream:
# which levels (grid sizes) the intra / deblock / inter time goes to.
#   LIBS="cur ..." bash tools/gpu/run_recon_trace.sh   (tools/exp/lib_<name>.so, cur = in-tree)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-rtrace}
mkdir -p $O
cp video-transformer_amd/vtseg/libvtseg.so tools/exp/lib_cur.so
[ -f /tmp/gcab.mp4 ] || timeout -k 10 300 python - <<'PY'
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/gcab.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full",
                  slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
print("stream written")
PY
for lib in ${LIBS:-cur}; do
  cp tools/exp/lib_$lib.so video-transformer_amd/vtseg/libvtseg.so
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/t_$lib" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --video /tmp/gcab.mp4 --config 720p-10min --coding full --bframes --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-parity --extras none > "$GRAFT_REPO_ROOT/$O/t_$lib.json" 2> "$GRAFT_REPO_ROOT/$O/t_$lib.err") || { tail -20 $O/t_$lib.err; exit 1; }
  python - $O/t_$lib $lib <<'PY' | tee -a $O/summary.txt
import csv, collections, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = collections.Counter(); n = collections.Counter(); by = collections.defaultdict(list)
for r in rows:
    k = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('vts::', '')
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot[k] += d; n[k] += 1
    g = tuple(r.get(c, '') for c in ('Grid_Size_X', 'Grid_Size_Y', 'Grid_Size_Z') if c in r) or (r.get('Grid_Size', ''),)
    by[k].append((g, d))
print("== lib", sys.argv[2])
for k, v in tot.most_common(8):
    print(f"{k}: {n[k]} dispatches, {v/1e3:.2f} ms total")
for k in ('h264_intra_full', 'h264_deblock_full', 'h264_inter_full', 'h264_bs_full'):
    L = by.get(k, [])
    if not L: continue
    # the last run's dispatches (warmup first): second half
    L = L[len(L) // 2:] if len(L) > 2 else L
    L.sort(key=lambda t: -t[1])
    print(k, "top:", [(g, round(d)) for g, d in L[:8]], "median us:", round(sorted(d for _, d in L)[len(L) // 2]))
PY
done
cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
