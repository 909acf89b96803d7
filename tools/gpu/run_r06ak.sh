#!/bin/bash
# round 6 (ak): kernel timeline of one content-stream run on the split parse
# (parse launches, derivations, then the reconstruction)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ak
mkdir -p $O
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/tr" -o run -- python3 "$GRAFT_REPO_ROOT/tools/gpu/run_once.py" /tmp/c0.mp4 > "$GRAFT_REPO_ROOT/$O/run.out" 2> "$GRAFT_REPO_ROOT/$O/run.err") || { tail -20 $O/run.err; exit 1; }
cat $O/run.out
python - $O/tr > $O/parse_derive.json <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("vts::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), r["Queue_Id"]))
rows.sort()
# the last run: from its last long parse launch
idx = [i for i, r in enumerate(rows) if r[2].startswith("h264_parse")]
last = rows[idx[-2]:] if len(idx) >= 2 else rows
t0 = last[0][0]
out = [{"k": r[2], "wg": r[3], "q": r[4], "start_ms": round((r[0] - t0) / 1e6, 3), "dur_ms": round((r[1] - r[0]) / 1e6, 3)}
       for r in last if not r[2].startswith(("h264_inter", "h264_intra", "h264_deblock", "h264_bs", "void thumb"))]
first_recon = next(((r[0] - t0) / 1e6 for r in last if r[2].startswith("h264_inter")), None)
print(json.dumps({"first_inter_start_ms": first_recon, "launches": out}, indent=1))
PY
cat $O/parse_derive.json
rm -rf $O/tr
