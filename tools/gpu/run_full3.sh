# General decoder: parity tests, bench line, rocprofv3 kernel stats of a short run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_full_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { tail -60 gpurun_out/pytest_full.log; exit 1; }
tail -3 gpurun_out/pytest_full.log
timeout -k 10 600 python -u bench.py --config 720p-10min --coding full --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -30 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
python - <<'PY'
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/full720.mp4", width=1280, height=720, fps=30, n_frames=3600, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4)
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_full" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --video /tmp/full720.mp4 --config 720p-10min --coding full --steps 2 --warmup 1 --no-pmc --no-cpu-baseline --no-parity > "$GRAFT_REPO_ROOT/gpurun_out/prof_full.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof_full.err" || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof_full.err"; exit 1; }
cd "$GRAFT_REPO_ROOT"
find gpurun_out/prof_full -name '*kernel_stats.csv' -exec cut -d, -f1-7 {} \; | head -12
