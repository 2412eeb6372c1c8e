set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05samp15
mkdir -p $O
timeout -k 10 300 python -u tools/sample_c4_probe.py 0.02 > $O/new.jsonl 2> $O/new.err || exit 11
timeout -k 10 600 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_c4.py -x -q --timeout 300 --timeout-method thread -k "hobe or sampler or fobe" > $O/tests.log 2>&1 || exit 10
