#!/bin/bash
# One gpurun call that regenerates the round's measurement evidence (run from
# the repo root on the GPU box).  Every GPU step has its own time limit and the
# session stops after a fault/timeout (tools/gpu_step.sh).
#   tools/round_evidence.sh r01
set -e
tag=${1:-r01}
export TMPDIR=/tmp
tools/gpu_step.sh pytest_gpu 900 python -m pytest tests -m gpu -q
tools/gpu_step.sh bench 400 python bench.py
tools/profile_bench.sh "$tag" --steps 50 --warmup 10 --no-host --no-sizes
tools/gpu_step.sh sweep 600 python tools/sweep_kernel.py --quick
tools/gpu_step.sh latency 300 python tools/latency.py --world 2
PG_BENCH_ONE_GPU=1 tools/gpu_step.sh bench_n2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --transports xgmi,xgmi_push
PG_BENCH_ONE_GPU=1 tools/gpu_step.sh bench_n4 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 4 --steps 10 --warmup 2 --transports xgmi,xgmi_push --ring-timeout 400
PG_BENCH_ONE_GPU=1 tools/gpu_step.sh bench_n8 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29553 bench.py --gpus 8 --steps 10 --warmup 2 --transports xgmi,xgmi_push --ring-timeout 500
tools/gpu_step.sh host_pipe 300 python tools/host_pipe_probe.py
tools/gpu_step.sh host_direct 120 python tools/lab/host_direct_probe.py 256
tools/gpu_step.sh gather 200 python tools/lab/gather_probe.py 8 64 256
