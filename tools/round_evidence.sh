#!/bin/bash
# One gpurun call that regenerates the round's measurement evidence (run from
# the repo root on the GPU box).  Every GPU step has its own time limit and the
# session stops after a fault/timeout (tools/gpu_step.sh).
#   tools/round_evidence.sh r02 [a|b|c|all]
# Part a (tests, bench, profiles, edge lab), part b (latency, the N = 2 and 4
# one-GPU rehearsals) and part c (the N = 8 rehearsal) each fit one gpurun
# call's 1200 s limit; "all" runs all three.
set -e
tag=${1:-r02}
part=${2:-all}
export TMPDIR=/tmp
if [ "$part" = a ] || [ "$part" = all ]; then
tools/gpu_step.sh pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=25
tools/gpu_step.sh bench 400 python bench.py
tools/profile_bench.sh "$tag" --steps 50 --warmup 10 --no-host --no-sizes
tools/gpu_step.sh edge_lab 300 python tools/lab/run_edge_lab.py
fi
if [ "$part" = b ] || [ "$part" = all ]; then
tools/gpu_step.sh latency 300 python tools/latency.py --world 2 --transport xgmi --out gpurun_out/latency.csv
tools/gpu_step.sh latency_rccl 300 python tools/latency.py --world 2 --transport rccl --out gpurun_out/latency_rccl.csv
PG_BENCH_ONE_GPU=1 tools/gpu_step.sh bench_n2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-sizes \
  --transports xgmi,xgmi_push,xgmi_read,rccl --ring-div 4 --ring-timeout 350
PG_BENCH_ONE_GPU=1 tools/gpu_step.sh bench_n4 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 4 --steps 10 --warmup 2 --no-sizes \
  --transports xgmi,xgmi_push,xgmi_read,rccl --ring-div 4 --ring-timeout 450
fi
if [ "$part" = c ] || [ "$part" = all ]; then
PG_BENCH_ONE_GPU=1 tools/gpu_step.sh bench_n8 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29553 bench.py --gpus 8 --steps 10 --warmup 2 --no-sizes \
  --transports xgmi,xgmi_push,xgmi_read,rccl --ring-div 8 --ring-timeout 550
fi
