#!/bin/bash
# Run one GPU step under its own time limit; record its exit status; stop the
# whole session (exit non-zero) on a fault/abort/segfault/timeout, so no later
# step touches the GPU after trouble.  Ordinary failures (rc 1, e.g. a failed
# assertion) let the session continue.
#   tools/gpu_step.sh NAME SECONDS CMD...   (output -> gpurun_out/NAME.log)
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[$name] rc=$rc" | tee -a gpurun_out/steps.log
case $rc in
  0|1|2|5) exit 0 ;;
  *) echo "[$name] stopping session (rc=$rc)" | tee -a gpurun_out/steps.log; exit 99 ;;
esac
