# Round 4 check: GPU parity suite on the 5-wave parser build, smoke, the
# self-launching 2-rank gloo rehearsal (bench.py --gpus 2), the default line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
cat $O/smoke.txt
if [ -z "$NO_GLOO" ]; then
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > $O/gloo2.json 2> $O/gloo2.err || { tail -30 $O/gloo2.err; exit 1; }
python -c "import json; d=json.load(open('$O/gloo2.json')); print('gloo2', d['value'], d['n_gpus'], d['world_size'], d['ranks_per_gpu'], d['parity']['all_ranks_equal'])"
fi
if [ -z "$NO_BENCH" ]; then
timeout -k 10 900 python bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['roofline']['frac'], d['parity']['all_equal'], d['general']['value'], d['general']['stage_ms'], d['e2e']['value'])"
fi
