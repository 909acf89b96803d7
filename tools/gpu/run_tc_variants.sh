# Same-box A/B of transcode variants (tools/exp/lib_<name>.so) with tc_probe
#   bash tools/gpu/run_tc_variants.sh "<W H F>" name1 name2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS=$1; shift
LIB=video-transformer_amd/vtseg/libvtseg.so
cp $LIB gpurun_out/lib_intree.so
for pass in $(seq ${PASSES:-2}); do
  for v in "$@"; do
    cp tools/exp/lib_$v.so $LIB
    timeout -k 10 300 python tools/gpu/tc_probe.py $ARGS 3 > gpurun_out/tcv_$v.json 2> gpurun_out/tcv_$v.err || { tail -20 gpurun_out/tcv_$v.err; cp gpurun_out/lib_intree.so $LIB; exit 1; }
    python - "$v" <<'PY'
import json,sys
rows=[json.loads(l) for l in open(f"gpurun_out/tcv_{sys.argv[1]}.json")]
best=min(rows, key=lambda r: r["search_ms"])
print(f"{sys.argv[1]:>8} search {best['search_ms']:.2f} ms write {best['write_ms']:.2f} ms wall {min(r['wall_ms'] for r in rows):.1f} ms")
PY
  done
done
cp gpurun_out/lib_intree.so $LIB
