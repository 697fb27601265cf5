#!/bin/bash
# Round-5 (session 4): kernel + HIP API trace of whole cfg3 steps (tools/pmc_step.py):
# when the host launches each binning kernel relative to the GPU's timeline.
set -u
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
LSR_STEPS=30 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/r05s4_host -o run -- python3 $ROOT/tools/pmc_step.py > $OUT/r05s4_host.log 2>&1 || { echo "trace failed"; tail -20 $OUT/r05s4_host.log; exit 1; }
find $OUT/r05s4_host -name "*.csv" | head
