# GPU tests, then the decode+score bench for several GOP-group sizes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for g in -1 160 100 69 40 20; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --gops-per-launch $g > gpurun_out/sweep_$g.json 2> gpurun_out/sweep_$g.err || { tail -20 gpurun_out/sweep_$g.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sweep_$g.json'));print($g, d['value'], d['ms_per_step'], d['config']['recon_launches'], d['config']['stage_ms'])"
done
