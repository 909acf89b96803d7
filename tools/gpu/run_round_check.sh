# Round check: every GPU test, smoke,
# then the default bench line with its profiles (headline + general record).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r03final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
t0=$SECONDS
timeout -k 10 720 python bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench wall s: $((SECONDS - t0))"
cut -c1-400 $O/bench.json
