set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c4b
mkdir -p $O
timeout -k 10 900 python -u tools/perf_hobe_c4_full.py > $O/c4_epoch_store.jsonl 2> $O/c4.err || exit 11
