#!/bin/bash
# round 6 (av): the bench's two-rank path on the one-GPU box (both ranks on
# cuda:0, gloo: RCCL refuses two ranks on one device) on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06av
mkdir -p $O
export MASTER_ADDR=127.0.0.1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --extras none --no-pmc > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err
rc=$?
tail -4 $O/bench_2rank_gloo.err
tail -c 600 $O/bench_2rank_gloo.json
exit $rc
