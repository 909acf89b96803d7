# Round 3: BASELINE config [4] rehearsal -- one 2-h 1080p video per rank, two
# ranks on one GPU over gloo (the NCCL branch differs only in the backend),
# parity over every frame on every rank.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03f
mkdir -p $O
t0=$SECONDS
timeout -k 10 1100 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --config 1080p-2h --steps 3 --warmup 1 --dist-backend gloo --parity-frames all > $O/rehearsal_1080p_2h_2rank.json 2> $O/rehearsal_1080p_2h_2rank.err || { tail -30 $O/rehearsal_1080p_2h_2rank.err; exit 1; }
echo "wall s: $((SECONDS - t0))"
cut -c1-1500 $O/rehearsal_1080p_2h_2rank.json
