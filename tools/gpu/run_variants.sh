# A/B timing of libvtseg variants (tools/exp/lib_<name>.so): GPU tests on the
# in-tree library first, then the bench once per variant per pass.
#   bash tools/gpu/run_variants.sh "<bench args>" name1 name2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS=$1; shift
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
LIB=video-transformer_amd/vtseg/libvtseg.so
cp $LIB gpurun_out/lib_intree.so
for pass in $(seq ${PASSES:-2}); do
  for v in "$@"; do
    cp tools/exp/lib_$v.so $LIB
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc $ARGS > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { tail -20 gpurun_out/var_$v.err; exit 1; }
    python - "$v" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/var_{sys.argv[1]}.json"))
r=d["roofline"]; st=d["config"]["stage_ms"]
print(f"{sys.argv[1]:>10} {d['value']:>11.0f} fps {d['ms_per_step']:7.3f} ms  kernel {r['kernel_ms']:.4f} ms frac {r['frac']:.4f}  parse {st['parse_ms']:.3f} recon {st['reconstruct_ms']:.3f} score {st['score_ms']:.3f}")
PY
  done
done
cp gpurun_out/lib_intree.so $LIB
