set -o pipefail
O=gpurun_out/r05tb
mkdir -p $O
timeout -k 10 600 python -u tools/ab_tb_d256.py 3 0.01 > $O/ab_tb_d256.jsonl 2> $O/ab.err || exit 11
