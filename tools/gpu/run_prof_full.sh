# rocprofv3 kernel trace + stats of the full-syntax benches (I/P and B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for b in "" "--bframes"; do
  n=full${b:+_b}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$n" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 720p-10min --coding full $b --steps 3 --warmup 1 --no-parity --no-cpu-baseline --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof_$n.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof_$n.err" || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_$n.err"; exit 1; }
done
