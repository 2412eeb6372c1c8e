#!/bin/bash
# r03: the --gpus N bench path rehearsed on one GPU: 2 ranks over gloo on
# cuda:0 (alg-dist node-row sharded with the edge-range pipeline, C4 HOBE in
# row-range chunks sampled row-sharded + all-gathered). Not a scaling
# measurement (both ranks share one GPU).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_mgpu}
mkdir -p $O
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 0 --one-device --dist-backend gloo --no-cpu --no-extra > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err || { echo G2FAIL; tail -30 $O/bench_2rank_gloo.err; exit 11; }
tail -c 2500 $O/bench_2rank_gloo.json
