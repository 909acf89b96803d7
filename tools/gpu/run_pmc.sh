# PMC counter passes (one counter group per run, kernel-trace only, no
# sys/runtime trace) over a short decode+score bench, then the summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline "$@" > "$GRAFT_REPO_ROOT/gpurun_out/pmc/p$i.log" 2>&1 \
    || { echo "pass $i ($set) failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc/p$i.log"; exit 1; }
done
cd "$GRAFT_REPO_ROOT"
python tools/pmc_summary.py gpurun_out/pmc/p1 gpurun_out/pmc/p2 gpurun_out/pmc/p3 gpurun_out/pmc/p4 gpurun_out/pmc/p5 --json gpurun_out/pmc/summary.json
