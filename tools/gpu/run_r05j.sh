# Round 5: hipMalloc cost probe, then the deblocking store-ordering A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 120 python tools/gpu/alloc_probe.py > $O/alloc.json 2> $O/alloc.err || { tail -5 $O/alloc.err; exit 1; }
cat $O/alloc.json
TAG=r05j VARS="buf bufpf2" bash tools/gpu/run_r05i.sh
