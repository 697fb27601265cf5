#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that FAILS its
# checks (pytest rc 1) does not stop the chain, but a crash, abort, signal or
# time limit (any other non-zero status) ends it there: nothing more touches
# the GPU after a fault.   usage: tools/gpu_steps.sh SECONDS 'cmd' [SECONDS 'cmd' ...]
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
    t=$1; cmd=$2; shift 2
    echo "[gpu_steps] $(date +%T) start (${t}s): $cmd"
    timeout -k 10 "$t" bash -c "$cmd"
    rc=$?
    echo "[gpu_steps] $(date +%T) rc=$rc: $cmd"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "[gpu_steps] stopping: rc $rc"
        exit $rc
    fi
done
