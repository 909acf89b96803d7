# Other BASELINE configurations per GPU: bash run_configs.sh "<bench args>" ...
# (each argument is one bench.py invocation's extra arguments)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
df -h /tmp | tail -1
free -g | head -2
i=0
for args in "$@"; do
  i=$((i+1))
  echo "== $args"
  timeout -k 10 1000 python bench.py --no-cpu-baseline $args > gpurun_out/cfg_$i.json 2> gpurun_out/cfg_$i.err || { tail -20 gpurun_out/cfg_$i.err; exit 1; }
  cat gpurun_out/cfg_$i.json
done
