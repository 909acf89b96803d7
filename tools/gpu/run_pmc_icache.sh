# Instruction-cache counters of the general decoder's kernels (CABAC B stream)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ -f /tmp/gcab.mp4 ] || timeout -k 10 300 python - <<'PY'
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/gcab.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full",
                  slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
PY
bash tools/gpu/pmc_kernel.sh "$GRAFT_REPO_ROOT/bench.py --video /tmp/gcab.mp4 --config 720p-10min --coding full --bframes --steps 1 --warmup 0 --no-pmc --no-cpu-baseline --no-parity --extras none" \
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES SQ_INSTS_SALU" > gpurun_out/pmc_icache.txt 2>&1
rc=$?; cat gpurun_out/pmc_icache.txt; [ $rc -eq 0 ] || touch gpurun_out/gpu_step_failed; exit $rc
