# Level-blocked kernel tests on the in-tree library, then the default bench
# once per libvtseg variant (tools/exp/lib_<name>.so) per pass.
#   bash tools/gpu/run_tbvar.sh "<bench args>" name1 name2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS=$1; shift
if [ "${TB_TESTS}" != none ]; then
  timeout -k 10 300 python -u -m pytest ${TB_TESTS:-tests/test_level_block_gpu.py} -q -x --timeout 120 --timeout-method thread > gpurun_out/tb_tests.log 2>&1 || { tail -30 gpurun_out/tb_tests.log; exit 1; }
  tail -1 gpurun_out/tb_tests.log
fi
LIB=video-transformer_amd/vtseg/libvtseg.so
cp $LIB gpurun_out/lib_intree.so
for pass in $(seq ${PASSES:-1}); do
  for v in "$@"; do
    [ $v = intree ] && cp gpurun_out/lib_intree.so $LIB || cp tools/exp/lib_$v.so $LIB
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc $ARGS > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { tail -20 gpurun_out/var_$v.err; cp gpurun_out/lib_intree.so $LIB; exit 1; }
    python - "$v" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/var_{sys.argv[1]}.json"))
r=d["roofline"]; st=d["config"]["stage_ms"]
print(f"{sys.argv[1]:>10} {d['value']:>11.0f} fps {d['ms_per_step']:7.3f} ms  {r['kernel']} {r['kernel_ms']:.4f} ms frac {r['frac']:.4f} parse {st['parse_ms']:.3f} recon {st['reconstruct_ms']:.3f}")
PY
  done
done
cp gpurun_out/lib_intree.so $LIB
