# Same-box A/B of the current tree against an older tree in tools/exp/old
# (its own bench.py + in-tree libvtseg.so), alternating, PASSES times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS=$1
for pass in $(seq ${PASSES:-3}); do
  for v in new old; do
    if [ $v = new ]; then B=bench.py; else B=tools/exp/old/bench.py; fi
    timeout -k 10 300 python $B --no-cpu-baseline --no-pmc $ARGS > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
    python - "$v" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/ab_{sys.argv[1]}.json"))
r=d["roofline"]; st=d["config"].get("stage_ms",{})
print(f"{sys.argv[1]:>5} {d['value']:>11.0f} fps {d['ms_per_step']:7.3f} ms kernel {r['kernel_ms']:.4f} ms frac {r['frac']:.4f} parse {st.get('parse_ms',0):.3f} recon {st.get('reconstruct_ms',0):.3f}")
PY
  done
done
