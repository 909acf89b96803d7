# PMC counters of the general decoder kernels on a 3600-frame full-syntax 720p video.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python - <<'PY'
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/full720.mp4", width=1280, height=720, fps=30, n_frames=3600, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4)
PY
bash tools/gpu/pmc_kernel.sh "$GRAFT_REPO_ROOT/bench.py --video /tmp/full720.mp4 --config 720p-10min --coding full --steps 1 --warmup 0 --no-pmc --no-cpu-baseline --no-parity" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_BRANCH" \
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" > gpurun_out/pmc_parse.txt 2>&1
rc=$?
cat gpurun_out/pmc_parse.txt
exit $rc
