set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --one-device --dist-backend gloo --no-cpu > gpurun_out/mgpu2.json 2> gpurun_out/mgpu2.err || { echo MGPU_FAIL; tail -30 gpurun_out/mgpu2.err; exit 1; }
echo done
