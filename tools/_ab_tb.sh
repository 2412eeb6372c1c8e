set -o pipefail
O=gpurun_out/r05tb2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -k "fobe_records or hobe" > $O/train_tests.log 2>&1 || exit 10
timeout -k 10 600 python -u tools/ab_tb_d256.py 3 0.01 > $O/ab_tb_d256.jsonl 2> $O/ab.err || exit 11
