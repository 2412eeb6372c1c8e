# the --gpus 8 path rehearsed on one GPU (gloo, every rank on cuda:0, C3 legs
# only: eight C4 replicas would not fit one GPU's memory). Not a scaling figure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_8rank
mkdir -p $O
timeout -k 10 900 python3 -u bench.py --gpus 8 --one-device --dist-backend gloo --no-cpu --no-extra --no-c4 --steps 1 --warmup 0 > $O/bench_8rank_gloo_one_gpu.json 2> $O/bench_8rank.err || { echo FAIL; tail -20 $O/bench_8rank.err; exit 11; }
echo ok
