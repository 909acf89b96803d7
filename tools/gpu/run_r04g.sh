# Round 4: content-mode streams on the GPU (parity against the oracle and the
# writer's reconstruction, cut detection), the 10-min 720p content stream's
# rate and decode stage times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_full_gpu.py -k "content" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python tools/gpu/content_probe.py /tmp/gcontent.mp4 3 > $O/content.json 2> $O/content.err || { tail -20 $O/content.err; exit 1; }
cat $O/content.json
