# A/B of (library variant x bench argument set): GPU tests on the in-tree
# library first, then the bench once per pair per pass.
#   [SKIP_TESTS=1] VARS="base ntoff" bash tools/gpu/run_var_args.sh "<args 1>" "<args 2>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
LIB=video-transformer_amd/vtseg/libvtseg.so
cp $LIB gpurun_out/lib_intree.so
for pass in $(seq ${PASSES:-2}); do
  for v in $VARS; do
    cp tools/exp/lib_$v.so $LIB
    i=0
    for a in "$@"; do
      i=$((i+1))
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc $a > gpurun_out/va_${v}_$i.json 2> gpurun_out/va_${v}_$i.err || { tail -20 gpurun_out/va_${v}_$i.err; cp gpurun_out/lib_intree.so $LIB; exit 1; }
      python - "$v" "$i" "$a" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/va_{sys.argv[1]}_{sys.argv[2]}.json"))
r=d["roofline"]; st=d["config"]["stage_ms"]
print(f"{sys.argv[1]:>8} {sys.argv[3]:>24} {d['value']:>11.0f} fps {d['ms_per_step']:7.3f} ms  kernel {r['kernel_ms']:.4f} ms/launch  launches {d['config']['recon_launches']}  parse {st['parse_ms']:.3f} recon {st['reconstruct_ms']:.3f}")
PY
    done
  done
done
cp gpurun_out/lib_intree.so $LIB
