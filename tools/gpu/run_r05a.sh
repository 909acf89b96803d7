# Round 5, first check after pruning the losing variants: full GPU parity
# suite, smoke, the default bench line (now with the 1080p record and the CPU
# baseline on every usable core) with its rocprofv3 summaries.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 900 python -u bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('bench', d['value'], d['roofline']['frac'], d['parity']['all_equal'], d['e2e'].get('value'), d['cpu_baseline'])
for k in ('general', 'general_content', 'long_video', 'hd_1080p'):
    r = d.get(k, {}); print(k, r.get('value'), r.get('stage_ms'), r.get('open_s'), r.get('windows'), r.get('cuts'), (r.get('parity') or {}).get('all_equal'), r.get('error'))
"
