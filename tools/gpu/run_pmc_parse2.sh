# PMC counters of the general decoder's parser on 3600-frame full-syntax 720p
# videos, I/P and with B pictures.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python - <<'PY'
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/full720.mp4", width=1280, height=720, fps=30, n_frames=3600, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4)
scene.synth_write("/tmp/full720b.mp4", width=1280, height=720, fps=30, n_frames=3600, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4, bframes=True, weighted="implicit")
PY
for v in full720 full720b; do
bash tools/gpu/pmc_kernel.sh "$GRAFT_REPO_ROOT/bench.py --video /tmp/$v.mp4 --config 720p-10min --coding full --steps 1 --warmup 0 --no-pmc --no-cpu-baseline --no-parity" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_BRANCH" \
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" > gpurun_out/pmc_parse_$v.txt 2>&1 || { cat gpurun_out/pmc_parse_$v.txt; exit 1; }
grep -E "parse_full|inter_full" gpurun_out/pmc_parse_$v.txt
done
