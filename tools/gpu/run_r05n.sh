# Round 5: full GPU suite, smoke, then the default bench line (N=1, extras,
# rocprofv3 passes kept under the profile dir).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05n}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
VTS_DEVMEM_LOG=1 timeout -k 10 900 python -u bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('bench', d['value'], d['roofline']['frac'], d['parity']['all_equal'], d['e2e'].get('value'), d['cpu_baseline']['value'])
for k in ('general_batch', 'general', 'general_content', 'long_video', 'hd_1080p'):
    r = d.get(k, {}); print(k, r.get('value'), r.get('ms_per_step'), r.get('batch_over_single'), r.get('hbm_gb_per_session'), r.get('hbm_gb_per_session_after_runs'), r.get('stage_ms'), r.get('open_s'), r.get('open_stages_ms'), (r.get('parity') or {}).get('all_equal'), r.get('error'))
"
