# the --gpus N path with 4 ranks rehearsed on one GPU (gloo; every rank on
# cuda:0): launcher, sharded alg-dist, row-sharded sampling and the sharded
# record-store fill with uneven 4-way splits. Not a scaling figure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_4rank
mkdir -p $O
timeout -k 10 1000 python3 -u bench.py --gpus 4 --one-device --dist-backend gloo --no-cpu --no-extra --steps 1 --warmup 0 > $O/bench_4rank_gloo_one_gpu.json 2> $O/bench_4rank.err || { echo FAIL; tail -20 $O/bench_4rank.err; exit 11; }
echo ok
