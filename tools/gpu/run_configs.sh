# The other BASELINE configurations per GPU (bench.py --config ...).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
df -h /tmp | tail -1
free -g | head -2
for cfg in "$@"; do
  echo "== $cfg"
  timeout -k 10 900 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg_$cfg.json 2> gpurun_out/cfg_$cfg.err || { tail -20 gpurun_out/cfg_$cfg.err; exit 1; }
  cat gpurun_out/cfg_$cfg.json
done
