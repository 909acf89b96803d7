#!/bin/bash
# round 6 (d): CABAC engine device/host divergence check; PC sampling trial on the micro-benchmark
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06d
timeout -k 10 120 ./tools/micro/cabac_bins 200000 > gpurun_out/r06d/cabac_bins.jsonl 2>&1 || exit $?
cat gpurun_out/r06d/cabac_bins.jsonl
rocprofv3 -L > gpurun_out/r06d/list_avail.txt 2>&1 || true
grep -i -A3 "pc_sampl\|pc sampl" gpurun_out/r06d/list_avail.txt | head -40
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 50 --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r06d/pcs" -o pcs -- \
  "$GRAFT_REPO_ROOT/tools/micro/cabac_bins" 50000 > "$GRAFT_REPO_ROOT/gpurun_out/r06d/pcs.log" 2>&1
echo "pc sampling rc=$?"
tail -5 "$GRAFT_REPO_ROOT/gpurun_out/r06d/pcs.log"
find "$GRAFT_REPO_ROOT/gpurun_out/r06d/pcs" -type f | head
