#!/bin/bash
# rocprofv3 passes over the same bench command (run on the GPU box from the
# repo root).  Kernel trace + stats in one pass; each PMC counter in its own
# pass (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2: MI355X_MICROARCH.md
# "rocprofv3 PMC slots"), never combined with runtime/sys tracing.
#   tools/profile_bench.sh TAG [bench args...]   -> gpurun_out/prof_TAG_{kt,fetch,write}/
set -e
tag=$1; shift
export TMPDIR=/tmp
tools/gpu_step.sh "prof_${tag}_kt" 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_${tag}_kt" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@"
tools/gpu_step.sh "prof_${tag}_fetch" 300 rocprofv3 --pmc FETCH_SIZE -d "gpurun_out/prof_${tag}_fetch" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@"
tools/gpu_step.sh "prof_${tag}_write" 300 rocprofv3 --pmc WRITE_SIZE -d "gpurun_out/prof_${tag}_write" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@"
