# Level-blocked kernel check: its tests + the decode parity tests, then the
# default bench line with and without level blocking (no PMC, no CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "${TB_TESTS}" != none ]; then
timeout -k 10 400 python -u -m pytest ${TB_TESTS:-tests/test_level_block_gpu.py tests/test_decode_gpu.py} -v --maxfail=4 --timeout 120 --timeout-method thread > gpurun_out/tb_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/tb_tests.log | sed 's/ *\[.*//' | tail -60
[ $rc -eq 0 ] || { grep -E "^E |Error|error" gpurun_out/tb_tests.log | head -40; exit 1; }
fi
for lb in ${TB_LB:-0 1}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --level-block $lb $1 > gpurun_out/tb_b$lb.json 2> gpurun_out/tb_b$lb.err || { tail -20 gpurun_out/tb_b$lb.err; exit 1; }
  python - "$lb" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/tb_b{sys.argv[1]}.json"))
r=d["roofline"]; st=d["config"].get("stage_ms",{})
print(f"lb={sys.argv[1]} {d['value']:>11.0f} fps {d['ms_per_step']:7.3f} ms {r['kernel']} {r['kernel_ms']:.4f} ms/launch frac {r['frac']:.4f} {r['frames_per_launch']} fr/launch  {st}")
PY
done
