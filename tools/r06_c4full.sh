# the opt-in --c4-full leg on one GPU (whole C4 HOBE d=256 pipeline)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_c4full}
mkdir -p $O
timeout -k 10 1000 python3 -u bench.py --c4-full --no-c4 --no-cpu --no-extra --steps 1 --warmup 0 > $O/bench_c4full.json 2> $O/bench_c4full.err || { echo C4FULLFAIL; exit 13; }
echo c4full-ok
