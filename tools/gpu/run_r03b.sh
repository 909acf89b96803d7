# Round 3: PMC of the general decoder's parser on the bench's x264-like CABAC
# B stream (3 600 frames): instruction mix, issue / wait split, and the
# instruction cache (the parse kernel's code object is ~518 KB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03b
O=gpurun_out/r03b
python - <<'PY'
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/gcab.mp4", width=1280, height=720, fps=30, n_frames=3600, seed=0x5EED,
                  coding="full", slices_per_row=0, max_motion=4, bframes=True, weighted="implicit",
                  cabac=True, transform_8x8=True)
PY
ARGS="$GRAFT_REPO_ROOT/bench.py --video /tmp/gcab.mp4 --config 720p-10min --coding full --bframes --steps 1 --warmup 0 --no-pmc --no-cpu-baseline --no-parity --extras none"
timeout -k 10 300 bash tools/gpu/pmc_kernel.sh "$ARGS" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
  "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_WAIT_INST_LDS" > $O/pmc_sq.txt 2>&1 || { cat $O/pmc_sq.txt; exit 1; }
grep -E "parse_full" $O/pmc_sq.txt
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d "$GRAFT_REPO_ROOT/$O/sqc" -o run -- python3 $ARGS > "$GRAFT_REPO_ROOT/$O/sqc.log" 2>&1) || { tail -20 $O/sqc.log; exit 1; }
python - $O/sqc <<'PY'
import csv,collections,glob,sys
f=glob.glob(sys.argv[1]+"/**/*counter_collection.csv",recursive=True)[0]
acc=collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'].replace('(anonymous namespace)::','').split('(')[0]
    acc[k][r['Counter_Name']]+=float(r['Counter_Value'])
for k,d in acc.items():
    if 'rocclr' in k: continue
    print(k, {c:f"{v:.4g}" for c,v in d.items()})
PY
