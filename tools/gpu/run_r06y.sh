#!/bin/bash
# round 6 (y): kernel timeline of one content-stream run (what runs at once
# during reconstruction, and the gaps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06y
mkdir -p $O
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/tr" -o run -- python3 "$GRAFT_REPO_ROOT/tools/gpu/run_once.py" /tmp/c0.mp4 > "$GRAFT_REPO_ROOT/$O/run.out" 2> "$GRAFT_REPO_ROOT/$O/run.err") || { tail -20 $O/run.err; exit 1; }
cat $O/run.out
python tools/gpu/recon_timeline.py $O/tr > $O/timeline.json && cat $O/timeline.json
python - <<'PY'
import glob, csv
f = glob.glob("gpurun_out/r06y/tr/**/*kernel_trace.csv", recursive=True)[0]
print(open(f).readline())
PY
rm -rf $O/tr
