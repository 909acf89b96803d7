# PMC counters per dispatch of the general decoder's kernels on the x264-like
# 10-min 720p CABAC B stream (two passes, tools/gpu/pmc_kernel.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ -f /tmp/gcab.mp4 ] || timeout -k 10 300 python - <<'PY'
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/gcab.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full",
                  slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
print("stream written")
PY
bash tools/gpu/pmc_kernel.sh "$GRAFT_REPO_ROOT/bench.py --video /tmp/gcab.mp4 --config 720p-10min --coding full --bframes --steps 1 --warmup 0 --no-pmc --no-cpu-baseline --no-parity --extras none" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_BRANCH" \
  "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC" > gpurun_out/pmc_recon.txt 2>&1
rc=$?; cat gpurun_out/pmc_recon.txt; exit $rc
