set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
( ls /opt/rocm/lib | grep -i -E 'decode|va' ; ls /usr/lib/x86_64-linux-gnu | grep -i -E 'libva|avcodec' ; which ffmpeg ffprobe ; rocm-smi --showproductname ; nproc ) > gpurun_out/box_probe.txt 2>&1 || true
timeout -k 10 400 python -m pytest tests/test_score_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --workload score --steps 10 --warmup 2 > gpurun_out/bench_score.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_score.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_score" -o prof -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload score --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_score.log" 2>&1 || { echo "rocprof failed"; tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof_score.log"; exit 1; }
echo done
